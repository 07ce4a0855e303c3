"""List A's exact chain runs beside k_demod by construction.

Frames whose detection falls inside a guard band are listed by k_detect; the fp64
replica of their detection (modem.js:286-319, detectPreamble's sequential recurrence)
runs on the context's second stream, created at amod_open at the device's highest
priority, while k_demod demodulates every other frame on the launch stream. Profiled
decodes record, on the device's real-time clock, when the replica took its first listed
frame and when k_demod's last wave ended (amod_aux_overlap): every decode with a listed
frame must have started it before k_demod finished."""
import ctypes as C

import numpy as np
import pytest

import amodem
from amodem import _lib as L
from helpers import open_with_env

pytestmark = pytest.mark.gpu


def _batch(snr_db, distinct=48, copies=40, seed=7):
    """distinct acoustic BPSK rep-3 frames under AWGN, each referenced `copies` times
    (frames are slices of one buffer and may repeat): a k_demod launch of a few hundred
    microseconds with the listed frames spread over the batch."""
    cfg = amodem.preset("acoustic", "BPSK", 3)
    x, offs, lens = amodem.synth_legacy_batch(cfg, distinct, payload_len=64, threads=8)
    if snr_db is not None:
        sp = float(np.mean(x[x != 0] ** 2))
        rng = np.random.default_rng(seed)
        x = (x + rng.standard_normal(len(x)).astype(np.float32) *
             np.float32(np.sqrt(sp / 10 ** (snr_db / 10)))).astype(np.float32)
    idx = np.tile(np.arange(distinct), copies)
    return cfg, x, offs[idx], lens[idx]


def _profiled_decodes(dm, cfg, x, offs, lens, n=6):
    import torch
    dev = torch.device("cuda", 0)
    xs = torch.zeros(len(x) + 16, dtype=torch.float32, device=dev)
    xs[:len(x)].copy_(torch.from_numpy(x))
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    F, N = len(offs), int(lens.max())
    stride = amodem.payload_stride(cfg, N)
    res = torch.zeros(F * 96, dtype=torch.uint8, device=dev)
    pay = torch.zeros(F * stride, dtype=torch.uint8, device=dev)
    dm.reserve(cfg, F, N)
    lib = L.load()

    def decode():
        dm.decode_device(cfg, L.MODE_RECEIVED, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F,
                         res.data_ptr(), pay.data_ptr(), stride, stream=torch.cuda.current_stream().cuda_stream)

    decode()
    torch.cuda.synchronize()
    lib.amod_set_profiling(dm.ctx, 1)
    for _ in range(n):
        decode()
    torch.cuda.synchronize()
    ms = (C.c_double * L.STAGE_COUNT)()
    nd = C.c_int64()
    assert lib.amod_kernel_stages(dm.ctx, ms, L.STAGE_COUNT, C.byref(nd)) == 0
    lib.amod_set_profiling(dm.ctx, 0)
    listed, beside, lead = C.c_int64(), C.c_int64(), C.c_double()
    assert lib.amod_aux_overlap(dm.ctx, C.byref(listed), C.byref(beside), C.byref(lead)) == 0
    rec = np.frombuffer(res.cpu().numpy().tobytes(), amodem.RESULT_DTYPE)
    return nd.value, listed.value, beside.value, lead.value, rec, [ms[i] / max(1, nd.value) for i in range(L.STAGE_COUNT)]


def test_listed_replica_starts_before_k_demod_ends():
    cfg, x, offs, lens = _batch(8.0)
    dm = open_with_env(0, AMOD_GUARD_SCALE=50)
    try:
        nd, listed, beside, lead, rec, st = _profiled_decodes(dm, cfg, x, offs, lens)
    finally:
        dm.close()
    nlisted = int(((rec["flags"] & (L.FLAG_EXACT | L.FLAG_REPLAY)) != 0).sum())
    assert nlisted > 0, np.unique(rec["flags"])
    assert nd == 6 and listed == nd, (nd, listed)
    assert beside == listed, (beside, listed, lead, st)
    assert lead > 0.0


def test_clean_batch_lists_nothing():
    cfg, x, offs, lens = _batch(None, distinct=16, copies=16)
    dm = amodem.Demodulator(0)
    try:
        nd, listed, beside, lead, rec, _ = _profiled_decodes(dm, cfg, x, offs, lens, n=3)
    finally:
        dm.close()
    assert nd == 3 and listed == 0 and beside == 0
    assert (rec["status"] == 0).all() and (rec["crc_valid"] == 1).all()
