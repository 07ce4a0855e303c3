"""Opt-in soft combining of repeated bits (AMOD_OPT_SOFT_COMBINE) — NOT reference
behaviour, so it is judged by error rate, not parity (majorityVote row;
BASELINE C5: BPSK repetition under AWGN). Acoustic BPSK rep3 data-chunk frames with
AWGN (noise divisor 1.5, ~1.8 dB): the reference's hard majority vote decodes 27 of 64
frames with a valid CRC, the |H|^2-weighted soft vote 35 (measured, tools/soft_sweep.py;
the reference's pilot-ratio phase estimate, not the vote, limits both below that). At
20 dB, and for repetition 1, the option changes nothing."""
import numpy as np
import pytest

import amodem
from amodem import _lib as L
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _frames(n, div, seed0, rep=3, mod="BPSK", config="acoustic", length=128):
    out = []
    pre = 2205  # buildChunkOFDMFrame's 0.05 s lead-in: windows start at pre1
    for i in range(n):
        case = {"config": config, "tx": {"kind": "chunk", "seq": i, "seed": 0xC5000000 + i, "len": length,
                                          "mod": mod, "rep": rep},
                "post": [{"op": "slice", "start": pre}, {"op": "noise", "snr": 0, "seed": seed0 + 7 * i, "div": div}]}
        out.append(O.build_case(case))
    lens = np.array([len(f) for f in out], np.int32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    return np.concatenate(out), offs, lens


def _decode(dm, cfg, x, offs, lens, options):
    rec, pay = dm.decode_batch(x, offs, lens, cfg=cfg, mode=L.MODE_CHUNK, options=options)
    return rec, pay


def test_soft_combining_beats_hard_vote_at_low_snr():
    cfg = amodem.preset("acoustic", "BPSK", 3)
    dm = amodem.Demodulator(0)
    for div, strict in ((1.5, True), (2.0, False)):
        x, offs, lens = _frames(64, div, 0x50F7)
        hard, _ = _decode(dm, cfg, x, offs, lens, 0)
        soft, sp = _decode(dm, cfg, x, offs, lens, L.OPT_SOFT_COMBINE)
        ok_h = int(((hard["status"] == 0) & (hard["crc_valid"] == 1)).sum())
        ok_s = int(((soft["status"] == 0) & (soft["crc_valid"] == 1)).sum())
        assert ok_s >= ok_h and (ok_s > ok_h or not strict), (div, ok_h, ok_s)
    dm.close()
    for i in np.nonzero((soft["status"] == 0) & (soft["crc_valid"] == 1))[0][:8]:
        d = amodem.to_reference(soft[i], sp[i].tobytes(), False)
        assert d["data"] == amodem.synth_payload(0xC5000000 + int(i), 128)


@pytest.mark.parametrize("rep,div", [(3, 100.0), (1, 3.0)])
def test_soft_option_is_neutral_when_clean_or_unrepeated(rep, div):
    cfg = amodem.preset("acoustic", "BPSK", rep)
    x, offs, lens = _frames(16, div, 0x1111, rep=rep)
    dm = amodem.Demodulator(0)
    hard, hp = _decode(dm, cfg, x, offs, lens, 0)
    soft, sp = _decode(dm, cfg, x, offs, lens, L.OPT_SOFT_COMBINE)
    dm.close()
    keys = ["status", "crc_valid", "seq_num", "data_len", "expected_crc", "actual_crc"]
    assert all(np.array_equal(hard[k], soft[k]) for k in keys)
    for i in range(len(hard)):
        assert amodem.to_reference(hard[i], hp[i].tobytes(), False) == amodem.to_reference(soft[i], sp[i].tobytes(),
                                                                                            False)


def test_soft_combining_qpsk_rep3():
    cfg = amodem.preset("standard", "QPSK", 3)
    x, offs, lens = _frames(64, 8.0, 0x50F7, rep=3, mod="QPSK", config="standard", length=256)
    dm = amodem.Demodulator(0)
    hard, _ = _decode(dm, cfg, x, offs, lens, 0)
    soft, _ = _decode(dm, cfg, x, offs, lens, L.OPT_SOFT_COMBINE)
    dm.close()
    ok_h = int(((hard["status"] == 0) & (hard["crc_valid"] == 1)).sum())
    ok_s = int(((soft["status"] == 0) & (soft["crc_valid"] == 1)).sum())
    assert ok_s >= ok_h, (ok_h, ok_s)


_FIELDS = ["status", "frame_type", "nbytes", "crc_valid", "seq_num", "data_len", "name_len", "expected_crc",
           "actual_crc", "aux"]


def _same(a, ap, b, bp):
    """per-frame equality of every decoded field and the payload bytes both decoded (not
    `flags`: the exact kernel marks its frames; not payload_valid: the fast path decodes
    only the symbols the parse reads, the exact kernel every symbol; not the fast path's
    approximate fine metric)"""
    bad = []
    for i in range(len(a)):
        pv = min(a["payload_valid"][i], b["payload_valid"][i])
        if any(a[k][i] != b[k][i] for k in _FIELDS) or ap[i, :pv].tobytes() != bp[i, :pv].tobytes():
            bad.append(i)
    return bad


@pytest.mark.parametrize("mod,config,rep,length,divs", [
    ("BPSK", "acoustic", 3, 128, (1.5, 2.0, 3.0, 6.0)),
    ("QPSK", "standard", 3, 256, (6.0, 8.0, 12.0)),
    ("BPSK", "narrowband", 5, 64, (2.0, 4.0)),
])
def test_fast_soft_equals_exact_soft(mod, config, rep, length, divs):
    """k_demod's soft-combining instance (per-symbol |H|^2-weighted group sums with error
    bounds) decides every repeat group as the exact kernel's fp64 soft vote
    does, frame for frame, on noisy chunk windows from ~1.8 dB up, and most frames stay on
    the fast path (a group inside its error bound routes its frame to the exact kernel)."""
    cfg = amodem.preset(config, mod, rep)
    dm = amodem.Demodulator(0)
    for d in divs:
        x, offs, lens = _frames(96, d, 0x5A5A + int(10 * d), rep=rep, mod=mod, config=config, length=length)
        fast, fp = _decode(dm, cfg, x, offs, lens, L.OPT_SOFT_COMBINE)
        ex, ep = _decode(dm, cfg, x, offs, lens, L.OPT_SOFT_COMBINE | L.OPT_FORCE_EXACT)
        assert (ex["flags"] & L.FLAG_EXACT).all()
        bad = _same(fast, fp, ex, ep)
        assert not bad, (d, bad[:5])
        on_fast = int(((fast["flags"] & L.FLAG_EXACT) == 0).sum())
        # about as many frames stay on the fast path as with the hard vote (whose guard
        # lists a frame for ANY decision inside its band; at low SNR both list many, QPSK
        # most: its max-log value is small wherever either component is)
        hard, _ = _decode(dm, cfg, x, offs, lens, 0)
        on_fast_hard = int(((hard["flags"] & L.FLAG_EXACT) == 0).sum())
        assert on_fast + max(4, len(fast) // 16) >= on_fast_hard, (d, on_fast, on_fast_hard)
        if mod == "BPSK" and d >= 3.0:
            assert on_fast >= 3 * len(fast) // 4, (d, on_fast)
    dm.close()


def test_fast_soft_received_mode_equals_exact():
    """the same through decodeReceivedSignal-shaped frames (preamble search, fine timing,
    legacy parse) with AWGN, BPSK rep 3"""
    cfg = amodem.preset("acoustic", "BPSK", 3)
    x, offs, lens = amodem.synth_legacy_batch(cfg, 48, payload_len=96, threads=8)
    sp = float(np.mean(x[x != 0] ** 2))
    dm = amodem.Demodulator(0)
    for snr_db, seed in ((6.0, 3), (9.0, 4), (14.0, 5)):
        rng = np.random.default_rng(seed)
        y = (x + rng.standard_normal(len(x)).astype(np.float32) * np.float32(np.sqrt(sp / 10 ** (snr_db / 10)))
             ).astype(np.float32)
        fast, fp = dm.decode_batch(y, offs, lens, cfg=cfg, options=L.OPT_SOFT_COMBINE)
        ex, ep = dm.decode_batch(y, offs, lens, cfg=cfg, options=L.OPT_SOFT_COMBINE | L.OPT_FORCE_EXACT)
        bad = [i for i in _same(fast, fp, ex, ep)]
        assert not bad, (snr_db, bad[:5])
        assert np.array_equal(fast["preamble_idx"], ex["preamble_idx"])
    dm.close()
