"""The QPSK / 16-QAM decision guard (DESIGN.md §4.1b "Guards": a decision whose margin to
a constellation boundary is inside the fp32 error band is not answered by the fast path;
the frame is listed for the fp64 replica, FLAG_DEMAP) exercised under AWGN, where it
must fire, against the CPU oracle frame by frame (constellationDemap / demodulateOFDM,
modem.js:140-150, 398-412): every reference-visible field and every byte the parse reads
equal. Noisy 16-QAM has three decision boundaries per axis: the most delicate guard."""
import numpy as np
import pytest

from helpers import ref_dict, struct_to_dict
from test_gpu_parity import as_golden, check_payload

import amodem
from amodem import _lib as L
from oracle import oracle as O

pytestmark = pytest.mark.gpu
FLAG_DEMAP = 1 << 7


@pytest.fixture(scope="module")
def dm():
    d = amodem.Demodulator(0)
    yield d
    d.close()


def _frames(kind, n, snr, seed0):
    """(preset, mod, rep, chunk, frames): n noisy frames from the oracle's recipes."""
    out = []
    for i in range(n):
        seed = 0x9E3779B9 ^ (50000 + 1000 * snr + i)
        if kind == "qam16_1k":
            case = {"config": "standard", "tx": {"kind": "legacy", "seed": seed, "len": 1024, "name": "f.bin",
                                                 "mod": "QAM16", "rep": 1}}
            mod, chunk, plen = "QAM16", False, 0
        elif kind == "qam16_chunk4k":
            case = {"config": "standard", "tx": {"kind": "chunk", "seq": i, "seed": seed, "len": 4096, "mod": "QAM16",
                                                 "rep": 1}}
            mod, chunk, plen = "QAM16", True, 4096
        else:  # qpsk_chunk2k: BASELINE C4's frame
            case = {"config": "standard", "tx": {"kind": "chunk", "seq": i, "seed": seed, "len": 2048, "mod": "QPSK",
                                                 "rep": 1}}
            mod, chunk, plen = "QPSK", True, 2048
        post = [{"op": "noise", "snr": snr, "seed": seed0 + 7919 * i}]
        if chunk:  # the StreamingReceiver's window: pre1 .. estimateFrameSamples(len + 11)
            win = amodem.estimate_frame_samples(plen + 11, mod, 1)
            post.append({"op": "slice", "start": 2205, "end": 2205 + win})
        case["post"] = post
        out.append(O.build_case(case))
    return "standard", mod, 1, chunk, out


@pytest.mark.parametrize("kind,n,snr", [("qam16_1k", 160, 10), ("qam16_1k", 160, 15), ("qam16_chunk4k", 96, 15),
                                        ("qpsk_chunk2k", 160, 8)])
def test_demap_guard_fires_and_matches_oracle(dm, kind, n, snr):
    preset, mod, rep, chunk, fr = _frames(kind, n, snr, 0xD3A0 + snr)
    lens = np.array([len(f) for f in fr], np.int32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    x = np.concatenate(fr).astype(np.float32)
    cfg = amodem.preset(preset, mod, rep)
    rec, pay = dm.decode_batch(x, offs, lens, cfg=cfg, mode=L.MODE_CHUNK if chunk else L.MODE_RECEIVED)
    c = O.cfg(preset)
    for i, f in enumerate(fr):
        r, refpay = O.decode(c, f, mod, rep, chunk)
        ref = ref_dict(struct_to_dict(r), refpay.tobytes(), via_legacy=not chunk)
        got = as_golden(amodem.to_reference(rec[i], pay[i].tobytes(), via_legacy=not chunk))
        assert got == ref, (kind, snr, i, int(rec[i]["flags"]))
        check_payload(rec[i], pay[i], refpay.tobytes(), False)
    demap = int(((rec["flags"] & FLAG_DEMAP) != 0).sum())
    assert demap > 0, f"{kind} at {snr} dB: the DEMAP guard never fired ({np.unique(rec['flags'])})"
    assert (rec["status"] == 0).sum() > 0


def test_c3_shaped_batch_at_15db_matches_oracle(dm):
    """2,000 16-QAM 1 KB legacy frames (BASELINE C3's frame) at 15 dB, one launch: every
    frame's status, CRC and reference fields equal the oracle's; the guard fires."""
    n = 2000
    cfg = amodem.preset("standard", "QAM16", 1)
    x, offs, lens = amodem.synth_legacy_batch(cfg, n, payload_len=1024, threads=16)
    xn = np.empty_like(x)
    for i in range(n):
        a, b = int(offs[i]), int(offs[i] + lens[i])
        xn[a:b] = O.add_noise(x[a:b], 15, 0xC3000 + i)
    rec, pay = dm.decode_batch(xn, offs, lens, cfg=cfg)
    c = O.cfg("standard")
    _, st, crc = O.bench_decode(c, xn, offs, lens, "QAM16", 1, 16)
    assert (rec["status"] == st).all()
    ok = st == 0
    assert (rec["actual_crc"][ok] == crc[ok]).all()
    for i in range(0, n, 7):  # whole result objects and bytes on a stride of the batch
        r, refpay = O.decode(c, xn[offs[i]:offs[i] + lens[i]], "QAM16", 1, False)
        ref = ref_dict(struct_to_dict(r), refpay.tobytes(), via_legacy=True)
        assert as_golden(amodem.to_reference(rec[i], pay[i].tobytes(), True)) == ref, i
    assert ((rec["flags"] & FLAG_DEMAP) != 0).sum() > 0
