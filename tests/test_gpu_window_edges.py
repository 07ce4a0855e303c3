"""Symbol windows k_demod tests with a shortcut, against the C oracle (modem.js in fp64).

k_demod decides two window facts without looking at every sample:
- constant window (all 512 samples equal: an all-zero spectrum, modem.js:431-438 and the
  demap of zero bins): one sample per lane first, all 512 only when those 64 agree;
- chunk mode's NaN/Inf samples (`x || 0` semantics, decodeChunkFrame modem.js:770-803,
  go to the exact path): read off one FFT bin pair per lane, since a non-finite input
  makes every bin of the transform non-finite.
Both must leave every record field and payload byte equal to the oracle's: windows with
NaN / +Inf / -Inf at random places (CE symbol, data symbols, the last symbol), constant
runs of zero and of a non-zero level covering whole symbols, in chunk and received mode."""
import numpy as np
import pytest

from helpers import ref_dict, struct_to_dict

import amodem
from amodem import _lib as L
from oracle import oracle as O

pytestmark = pytest.mark.gpu

FLAG_NONFINITE = 1 << 1


def as_golden(d: dict) -> dict:
    return {k: ({"hex": v.hex()} if isinstance(v, (bytes, bytearray)) else v) for k, v in d.items()}


def _frames(chunk, n, seed0):
    out = []
    for i in range(n):
        if chunk:
            case = {"config": "standard", "tx": {"kind": "chunk", "seq": i, "seed": 0x9E3779B9 ^ (5000 + i),
                                                 "len": 2048, "mod": "QPSK", "rep": 1},
                    "post": [{"op": "noise", "snr": 20, "seed": seed0 + 31 * i},
                             {"op": "slice", "start": 2205, "end": 2205 + 3 * 576 + 41 * 576}]}
        else:
            case = {"config": "standard", "tx": {"kind": "legacy", "seed": 0x9E3779B9 ^ (6000 + i), "len": 512,
                                                 "name": "e.bin", "mod": "QPSK", "rep": 1},
                    "post": [{"op": "noise", "snr": 20, "seed": seed0 + 31 * i}]}
        out.append(O.build_case(case).astype(np.float32))
    return out


def _damage(f, i, rng):
    """Frame i's edit (kind i % 8); returns whether it holds a non-finite sample."""
    n = len(f)
    kind = i % 8
    if kind == 0:
        f[rng.integers(n // 4, n)] = np.nan
    elif kind == 1:
        f[rng.integers(n // 4, n)] = np.inf
    elif kind == 2:
        f[rng.integers(0, 3 * 576)] = -np.inf       # the preamble / CE symbols
    elif kind == 3:
        f[n - 1 - rng.integers(0, 500)] = np.nan    # the last symbol
    elif kind == 4:
        a = int(rng.integers(3 * 576, n - 1300))
        f[a:a + 1300] = 0.0                          # two whole symbols of silence at least
    elif kind == 5:
        a = int(rng.integers(3 * 576, n - 1300))
        f[a:a + 1300] = np.float32(0.37)             # a constant non-zero level
    elif kind == 6:
        f[rng.integers(0, n, 3)] = [np.nan, np.inf, -np.inf]
    return kind in (0, 1, 2, 3, 6)


@pytest.mark.parametrize("chunk", [True, False], ids=["chunk", "received"])
def test_window_edges_match_oracle(chunk):
    rng = np.random.default_rng(77 if chunk else 78)
    fr = _frames(chunk, 32, 0x5EED)
    nonfinite = [_damage(f, i, rng) for i, f in enumerate(fr)]
    lens = np.array([len(f) for f in fr], np.int32)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    x = np.concatenate(fr).astype(np.float32)
    cfg = amodem.preset("standard", "QPSK", 1)
    dm = amodem.Demodulator(0)
    try:
        rec, pay = dm.decode_batch(x, offs, lens, cfg=cfg, mode=L.MODE_CHUNK if chunk else L.MODE_RECEIVED)
    finally:
        dm.close()
    c = O.cfg("standard")
    for i, f in enumerate(fr):
        r, rp = O.decode(c, f, "QPSK", 1, chunk)
        ref = ref_dict(struct_to_dict(r), rp.tobytes(), via_legacy=not chunk)
        got = as_golden(amodem.to_reference(rec[i], pay[i].tobytes(), via_legacy=not chunk))
        assert got == ref, (i, i % 8, int(rec[i]["flags"]))
    flagged = [bool(int(rec[i]["flags"]) & FLAG_NONFINITE) for i in range(len(fr))]
    # received mode: stage 0's mean sees every sample; chunk mode: only samples some symbol
    # window reads (a NaN in a cyclic prefix changes nothing, in the reference too)
    hit = sum(f for f, nf in zip(flagged, nonfinite) if nf)
    assert hit == sum(nonfinite) if not chunk else hit >= sum(nonfinite) // 2, (flagged, nonfinite)
    assert not any(f for f, nf in zip(flagged, nonfinite) if not nf)
    # the undamaged frames stay on the fast path
    for i in range(7, len(fr), 8):
        assert int(rec[i]["flags"]) & L.FLAG_EXACT == 0, i
