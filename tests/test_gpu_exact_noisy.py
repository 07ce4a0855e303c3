"""Exact-replica path under noise, against the C oracle (modem.js restated in fp64).

The replica's two sequential recurrences are restructured for the GPU:
- preprocessSignal's mean (modem.js:215-217): segments certified along the sequential
  order (no partial sum inside them can round), the rest summed sample by sample;
- detectPreamble (286-319): increments and metrics on every lane, only the three running
  sums sequential, and, for a frame the coarse stage listed with a proven hull of the
  argmax, the recurrence stops at the hull's end.
Both must leave every result field bit-equal to the oracle's: status, coarse index
(Schmidl-Cox argmax), preamble index, fine metric, bytes. Frames include samples far
below the running sum's ulp (forcing the per-sample segments) and AWGN at 6-12 dB (where
the fast path lists frames with ambiguous coarse decisions)."""
import numpy as np
import pytest

from helpers import open_with_env, ref_dict, struct_to_dict

import amodem
from amodem import _lib as L
from oracle import oracle as O


def as_golden(d: dict) -> dict:
    return {k: ({"hex": v.hex()} if isinstance(v, (bytes, bytearray)) else v) for k, v in d.items()}


pytestmark = pytest.mark.gpu


def _noisy_batch(preset, mod, rep, nframes, payload, snr_db, seed, tiny=False):
    cfg = amodem.preset(preset, mod, rep)
    x, offs, lens = amodem.synth_legacy_batch(cfg, nframes, payload_len=payload, threads=8)
    sp = float(np.mean(x[x != 0] ** 2))
    rng = np.random.default_rng(seed)
    x = (x + rng.standard_normal(len(x)).astype(np.float32) * np.float32(np.sqrt(sp / 10 ** (snr_db / 10)))).astype(np.float32)
    if tiny:  # samples far below any running sum's ulp, at random places of every frame
        for o, n in zip(offs, lens):
            idx = o + rng.integers(0, n, 6)
            x[idx] = np.array([1e-30, -3e-12, 7e-9, -2e-20, 1e-38, 5e-10], np.float32)
    return cfg, x, offs, lens


DEMOD_FLAGS = (1 << 7) | (1 << 6) | (1 << 5) | (1 << 9) | (1 << 10)


def _check_against_oracle(cfg_name, mod, rep, x, offs, lens, rec, pay):
    c = O.cfg(cfg_name)
    for i, (o, n) in enumerate(zip(offs, lens)):
        r, rp = O.decode(c, x[o:o + n], mod, rep, False)
        fl = int(rec["flags"][i])
        ref = ref_dict(struct_to_dict(r), rp.tobytes(), via_legacy=True)
        got = as_golden(amodem.to_reference(rec[i], pay[i].tobytes(), via_legacy=True))
        assert got == ref, (i, fl)
        if fl & (L.FLAG_EXACT | L.FLAG_REPLAY) and fl & ~(L.FLAG_EXACT | L.FLAG_REPLAY | DEMOD_FLAGS):
            # the replica's own Schmidl-Cox argmax and fine metric (demodulation-only
            # frames keep the fast path's plateau index, pinned in test_gpu_parity); a
            # replayed detection (REPLAY: demodulated by k_demod) reports the replica's too
            assert int(rec["coarse_idx"][i]) == r.coarse_idx, (i, fl)
            if r.coarse_idx >= 0:
                assert float(rec["fine_metric"][i]) == float(np.float32(r.fine_metric)), (i, fl)


@pytest.mark.parametrize("snr_db,tiny", [(6, False), (8, True), (12, True)])
def test_forced_exact_matches_oracle_under_noise(snr_db, tiny):
    cfg, x, offs, lens = _noisy_batch("acoustic", "BPSK", 3, 12, 64, snr_db, seed=snr_db, tiny=tiny)
    dm = amodem.Demodulator(0)
    rec, pay = dm.decode_batch(x, offs, lens, cfg=cfg, options=L.OPT_FORCE_EXACT)
    dm.close()
    assert (rec["flags"] & L.FLAG_EXACT).all()
    _check_against_oracle("acoustic", "BPSK", 3, x, offs, lens, rec, pay)


def _wide_guard_demodulator(cfg, x, offs, lens, **env):
    """A context whose guard bands are 50x the default (AMOD_GUARD_SCALE, read when the
    context opens): at these SNRs ambiguous coarse / fine decisions, and so the listed
    paths, become common instead of a few per 10^4 frames."""
    return open_with_env(0, AMOD_GUARD_SCALE=50, **env)


@pytest.mark.parametrize("preset,snr_db", [("acoustic", 6), ("standard", 7)])
def test_listed_coarse_frames_match_oracle(preset, snr_db):
    """Frames the fast path lists for an ambiguous coarse decision run the replica's
    recurrence only up to the proven hull: the argmax still equals the oracle's."""
    cfg, x, offs, lens = _noisy_batch(preset, "BPSK", 3, 48, 64, snr_db, seed=3)
    dm = _wide_guard_demodulator(cfg, x, offs, lens)
    rec, pay = dm.decode_batch(x, offs, lens, cfg=cfg)
    full, fpay = dm.decode_batch(x, offs, lens, cfg=cfg, options=L.OPT_FORCE_EXACT)
    dm.close()
    coarse_listed = (rec["flags"] & (1 << 3)) != 0  # AMOD_FLAG_COARSE
    listed = (rec["flags"] & (L.FLAG_EXACT | L.FLAG_REPLAY)) != 0
    assert (coarse_listed & listed).sum() > 0, np.unique(rec["flags"])  # the listed path is exercised
    for i in np.nonzero(coarse_listed & listed)[0]:
        assert int(rec["coarse_idx"][i]) == int(full["coarse_idx"][i]), i
        assert float(rec["fine_metric"][i]) == float(full["fine_metric"][i]), i
    for n in ("status", "preamble_idx", "frame_type", "nbytes", "data_len", "expected_crc", "actual_crc", "crc_valid"):
        assert (rec[n] == full[n]).all(), n
    _check_against_oracle(preset, "BPSK", 3, x, offs, lens, rec, pay)


def test_exact_mean_is_the_sequential_sum():
    """preprocessSignal's mean on the exact path equals numpy's sequential (cumsum) fp64
    sum over a frame with samples far below the running sum's ulp."""
    import torch
    cfg, x, offs, lens = _noisy_batch("acoustic", "BPSK", 3, 1, 64, 8, seed=5, tiny=True)
    fr = x[offs[0]:offs[0] + lens[0]].copy()
    seq = np.cumsum(fr.astype(np.float64))[-1] / len(fr)
    dev = torch.device("cuda", 0)
    xs = torch.from_numpy(np.concatenate([fr, np.zeros(4, np.float32)])).to(dev)
    off = torch.zeros(1, dtype=torch.int64, device=dev)
    ln = torch.tensor([len(fr)], dtype=torch.int32, device=dev)
    stride = amodem.payload_stride(cfg, len(fr))
    res = torch.zeros(96, dtype=torch.uint8, device=dev)
    pay = torch.zeros(stride, dtype=torch.uint8, device=dev)
    dbg = torch.zeros(L.C.sizeof(L.Debug), dtype=torch.uint8, device=dev)
    dm = amodem.Demodulator(0)
    dm.reserve(cfg, 1, len(fr))
    torch.cuda.synchronize()
    dm.decode_device(cfg, L.MODE_RECEIVED, xs.data_ptr(), off.data_ptr(), ln.data_ptr(), 1, res.data_ptr(),
                     pay.data_ptr(), stride, options=L.OPT_FORCE_EXACT, debug_ptr=dbg.data_ptr())
    dm.synchronize()
    d = L.Debug.from_buffer_copy(dbg.cpu().numpy().tobytes())
    dm.close()
    _, mean, _ = O.preprocess(fr)
    assert mean == seq
    assert d.mean == seq


def _mean_frames(n, seed):
    """Frames whose sequential mean rounds in many places: a large DC offset (the running
    sum climbs through many binades, rounding at the crossings), tiny samples far below
    its ulp, and samples of random exponents (64-sample blocks whose own prefix sums are
    not exact, summed sample by sample)."""
    rng = np.random.default_rng(seed)
    out = []
    for k in range(4):
        x = rng.standard_normal(n).astype(np.float64) * 0.3
        if k == 0:
            x += 3.7
        elif k == 1:
            x += -0.9
            x[rng.integers(0, n, 200)] = rng.choice([1e-30, -3e-12, 7e-9, -2e-20], 200)
        elif k == 2:
            x = np.sign(x) * np.exp2(rng.uniform(-45, 4, n))
        else:
            x = np.cumsum(x) * 1e-2  # slow drift: long runs in one binade, both signs
        out.append(x.astype(np.float32))
    return out


@pytest.mark.parametrize("n", [4096 + 77, 111300])
def test_exact_mean_rounding_events(n):
    """The mean's failing segments walk 64-sample blocks: every lane's fl(S + P_j), the
    first rounded one by TwoSum, the block continued from it. Bit-equal to numpy's
    sequential cumsum on frames built to round often (and to not be certifiable)."""
    import torch
    cfg = amodem.preset("acoustic", "BPSK", 3)
    frs = _mean_frames(n, seed=n)
    x = np.concatenate(frs + [np.zeros(4, np.float32)])
    F = len(frs)
    dev = torch.device("cuda", 0)
    xs = torch.from_numpy(x).to(dev)
    off = torch.tensor([i * n for i in range(F)], dtype=torch.int64, device=dev)
    ln = torch.full((F,), n, dtype=torch.int32, device=dev)
    stride = amodem.payload_stride(cfg, n)
    res = torch.zeros(96 * F, dtype=torch.uint8, device=dev)
    pay = torch.zeros(stride * F, dtype=torch.uint8, device=dev)
    dsz = L.C.sizeof(L.Debug)
    dbg = torch.zeros(dsz * F, dtype=torch.uint8, device=dev)
    dm = amodem.Demodulator(0)
    dm.reserve(cfg, F, n)
    torch.cuda.synchronize()
    dm.decode_device(cfg, L.MODE_RECEIVED, xs.data_ptr(), off.data_ptr(), ln.data_ptr(), F, res.data_ptr(),
                     pay.data_ptr(), stride, options=L.OPT_FORCE_EXACT, debug_ptr=dbg.data_ptr())
    dm.synchronize()
    raw = dbg.cpu().numpy().tobytes()
    dm.close()
    for i, fr in enumerate(frs):
        seq = np.cumsum(fr.astype(np.float64))[-1] / n
        d = L.Debug.from_buffer_copy(raw[i * dsz:(i + 1) * dsz])
        assert d.mean == seq, (i, d.mean, seq, np.sum(fr.astype(np.float64)) / n)


@pytest.mark.parametrize("preset,snr_db", [("acoustic", 8), ("acoustic", 9), ("standard", 7)])
def test_replayed_detection_equals_full_exact_path(preset, snr_db):
    """Detection replay: a frame listed only for detection-stage guards gets its
    detection from the fp64 replica and its symbols from k_demod (AMOD_FLAG_REPLAY);
    every result field and payload byte equals the whole-frame replica's
    (AMOD_NO_REPLAY) and the oracle's."""
    cfg, x, offs, lens = _noisy_batch(preset, "BPSK", 3, 48, 64, snr_db, seed=11)
    dm = _wide_guard_demodulator(cfg, x, offs, lens)
    rec, pay = dm.decode_batch(x, offs, lens, cfg=cfg)
    dm.close()
    dm = _wide_guard_demodulator(cfg, x, offs, lens, AMOD_NO_REPLAY=1)
    ref, rpay = dm.decode_batch(x, offs, lens, cfg=cfg)
    dm.close()
    replayed = (rec["flags"] & L.FLAG_REPLAY) != 0
    if preset == "acoustic":  # (standard at 7 dB: ambiguous coarse decisions end in detection errors)
        assert replayed.sum() > 0, np.unique(rec["flags"])
    assert not (ref["flags"] & L.FLAG_REPLAY).any()
    for n in ("status", "preamble_idx", "coarse_idx", "fine_metric", "frame_type", "nbytes", "data_len",
              "expected_crc", "actual_crc", "crc_valid"):
        assert (rec[n] == ref[n]).all(), n
    for i in range(len(offs)):
        pv = int(rec["payload_valid"][i])
        assert pay[i][:pv].tobytes() == rpay[i][:pv].tobytes(), i
    _check_against_oracle(preset, "BPSK", 3, x, offs, lens, rec, pay)


def test_listed_frames_across_consecutive_decodes():
    """The exact-list counters alternate between two sets from one decode to the next
    (each decode's list-B launch zeroes the set the previous one used, instead of a
    memset): repeated decodes on one context, with many frames listed and with batches
    of other sizes, forced-exact decodes and a buffer reallocation in between, return
    the same records every time, equal to the oracle's."""
    cfg, x, offs, lens = _noisy_batch("acoustic", "BPSK", 3, 48, 64, 6, seed=11)
    dm = _wide_guard_demodulator(cfg, x, offs, lens)
    first, fpay = dm.decode_batch(x, offs, lens, cfg=cfg)
    assert ((first["flags"] & (L.FLAG_EXACT | L.FLAG_REPLAY)) != 0).sum() > 0
    _check_against_oracle("acoustic", "BPSK", 3, x, offs, lens, first, fpay)
    big_offs = np.concatenate([offs, offs, offs, offs])
    big_lens = np.concatenate([lens, lens, lens, lens])
    for k in range(6):
        if k == 1:
            dm.decode_batch(x, offs[:5], lens[:5], cfg=cfg)
        if k == 2:
            dm.decode_batch(x, offs, lens, cfg=cfg, options=L.OPT_FORCE_EXACT)
        if k == 3:  # more frames than before: the counter and list buffer grows
            big, _ = dm.decode_batch(x, big_offs, big_lens, cfg=cfg)
            for n in ("status", "preamble_idx", "nbytes", "crc_valid", "flags"):
                assert (big[n] == np.concatenate([first[n]] * 4)).all(), n
        rec, pay = dm.decode_batch(x, offs, lens, cfg=cfg)
        assert rec.tobytes() == first.tobytes(), k
        assert (pay == fpay).all(), k
    dm.close()
