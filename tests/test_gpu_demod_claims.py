"""k_demod's claimed tail: with at least AMOD_CLAIM_MIN (4) frames per wave, the frames past
the static rounds are claimed one at a time from a counter (the youngest waves of a SIMD
get the issue slots the older ones leave, so a purely static split left them running the
kernel's tail alone). Which wave demodulates a frame must not change anything: every
record and payload byte equals the all-static decode (AMOD_DEMOD_STATIC=1) and the
reference's outcome (decodeChunkFrame, modem.js:770-803, through the C oracle) on a
sample of the frames, across repeated decodes (the counter is zeroed by k_detect /
k_chunk_prep, the decode's first launch)."""
import numpy as np
import pytest

import amodem
from amodem import _lib as L
from helpers import open_with_env
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _windows(n):
    """n short QPSK chunk frames (32 data bytes each, GPU transmitter), cut to the
    receiver's windows: pre1 .. the estimated frame end (app.js:853)."""
    cfg = amodem.preset("standard", "QPSK", 1)
    dm = amodem.Demodulator(0)
    pk = [amodem.packet_chunk(amodem.synth_payload(0xC1A1 ^ i, 32), i) for i in range(n)]
    x, offs, lens = dm.transmit_batch(cfg, pk, L.TX_CHUNK)
    dm.close()
    pre, _ = amodem.tx_silence(cfg, L.TX_CHUNK)
    win = amodem.estimate_frame_samples(32 + 11, "QPSK", 1)
    return cfg, x, offs + pre, np.full(n, win, np.int32)


def _decode_device(dm, cfg, x, offs, lens, reps):
    import torch
    dev = torch.device("cuda", 0)
    xs = torch.zeros(len(x) + 16, dtype=torch.float32, device=dev)
    xs[:len(x)].copy_(torch.from_numpy(x))
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    F, N = len(offs), int(lens.max())
    stride = amodem.payload_stride(cfg, N)
    dm.reserve(cfg, F, N)
    out = []
    for _ in range(reps):
        res = torch.zeros(F * 96, dtype=torch.uint8, device=dev)
        pay = torch.zeros(F * stride, dtype=torch.uint8, device=dev)
        dm.decode_device(cfg, L.MODE_CHUNK, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F, res.data_ptr(),
                         pay.data_ptr(), stride, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        out.append((np.frombuffer(res.cpu().numpy().tobytes(), amodem.RESULT_DTYPE), pay.cpu().numpy().reshape(F, stride)))
    return out


def test_claimed_tail_equals_static_split():
    n = 24000  # 5.9 frames per wave on 4,096 waves: the claimed tail is used
    cfg, x, offs, lens = _windows(n)
    dyn = amodem.Demodulator(0)
    got = _decode_device(dyn, cfg, x, offs, lens, reps=3)
    dyn.close()
    st = open_with_env(0, AMOD_DEMOD_STATIC=1)
    (ref, rpay), = _decode_device(st, cfg, x, offs, lens, reps=1)
    st.close()
    assert (ref["status"] == 0).all() and (ref["crc_valid"] == 1).all()
    assert (ref["seq_num"] == np.arange(n)).all()
    for rec, pay in got:
        assert rec.tobytes() == ref.tobytes()
        assert np.array_equal(pay, rpay)
    c = O.cfg("standard")
    for i in range(0, n, 997):  # the reference's outcome on a sample
        r, rp = O.decode(c, x[offs[i]:offs[i] + lens[i]], "QPSK", 1, True)
        assert r.status == 0 and r.crc_valid == 1 and r.seq_num == i and r.actual_crc == ref["actual_crc"][i], i
