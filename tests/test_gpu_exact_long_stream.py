"""The exact replica's bit stream in global memory: frames whose decisions do not fit the
LDS stream area (k_decode_exact.hip: more than ~1,540 words, e.g. 8 KB QPSK legacy frames)
keep the slot's global words, ORed by L2 atomics and read back by the vote, parse, CRC and
payload rows after a workgroup barrier and an L1 invalidate. Long and short frames
alternate in one forced-exact launch with few persistent workgroups (AMOD_XSLOTS), so every
workgroup walks both paths several times over the same slot; each record and payload row
must equal the fast path's (which the parity tests pin to the oracle)."""
import numpy as np
import pytest

import amodem
from amodem import _lib as L

pytestmark = pytest.mark.gpu


def _mixed_batch(cfg):
    xs, offs, lens = [], [], []
    base = 0
    for k, plen in enumerate([8192, 512, 6000, 64, 8192, 1500] * 2):
        x, o, l = amodem.synth_legacy_batch(cfg, 1, payload_len=plen, first=k, threads=1)
        xs.append(x)
        offs.append(base + int(o[0]))
        lens.append(int(l[0]))
        base += len(x)
    return np.concatenate(xs), np.array(offs, np.int64), np.array(lens, np.int32)


def test_exact_global_stream_equals_fast(monkeypatch):
    cfg = amodem.preset("standard", "QPSK", 1)
    x, offs, lens = _mixed_batch(cfg)
    dm = amodem.Demodulator(0)
    ref, rpay = dm.decode_batch(x, offs, lens, cfg=cfg)
    dm.close()
    assert (ref["status"] == 0).all() and (ref["crc_valid"] == 1).all()
    monkeypatch.setenv("AMOD_XSLOTS", "3")  # (read when a context opens)
    dm = amodem.Demodulator(0)
    for _ in range(2):  # (the second pass finds the slots' lines from the first)
        rec, pay = dm.decode_batch(x, offs, lens, cfg=cfg, options=L.OPT_FORCE_EXACT)
        assert (rec["flags"] & L.FLAG_EXACT).all()
        for n in amodem.RESULT_DTYPE.names:
            if n in ("flags", "reserved", "coarse_idx", "fine_metric", "payload_valid"):
                continue
            assert (rec[n] == ref[n]).all(), n
        # the exact kernel stores every decoded byte, the fast one the prefix its parse
        # reads (header .. CRC): that prefix must agree
        assert (rec["payload_valid"] == rec["nbytes"]).all()
        for i in range(len(offs)):
            pv = int(ref["payload_valid"][i])
            assert pv <= int(rec["payload_valid"][i]) and np.array_equal(pay[i, :pv], rpay[i, :pv]), i
    dm.close()
