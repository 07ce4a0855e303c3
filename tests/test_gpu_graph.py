"""amod_decode_device captured into a hipGraph (include/amodem.h: amod_reserve, then
capture) and replayed: every replay, and an eager decode after the replays, returns the
eager decode's records and payload. Frames are listed for the exact kernel (wide guard
bands), so the exact-list counters — zeroed at the end of every decode, replayed or
eager, by its own list-B launch's last workgroup — are exercised across replays."""

import numpy as np
import pytest

import amodem
from amodem import _lib as L
from helpers import open_with_env

pytestmark = pytest.mark.gpu


def test_captured_decode_replays_equal_eager():
    import torch
    cfg = amodem.preset("acoustic", "BPSK", 3)
    x, offs, lens = amodem.synth_legacy_batch(cfg, 32, payload_len=64, threads=8)
    sp = float(np.mean(x[x != 0] ** 2))
    rng = np.random.default_rng(5)
    x = (x + rng.standard_normal(len(x)).astype(np.float32) * np.float32(np.sqrt(sp / 10 ** 0.6))).astype(np.float32)
    F, N = len(offs), int(lens.max())
    dev = torch.device("cuda", 0)
    xs = torch.zeros(len(x) + 16, dtype=torch.float32, device=dev)
    xs[:len(x)].copy_(torch.from_numpy(x))
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    stride = amodem.payload_stride(cfg, N)
    res = torch.zeros(F * 96, dtype=torch.uint8, device=dev)
    pay = torch.zeros(F * stride, dtype=torch.uint8, device=dev)

    dm = open_with_env(0, AMOD_GUARD_SCALE=50)  # knobs are read when a context opens
    dm.reserve(cfg, F, N)
    s = torch.cuda.Stream()

    def decode():
        dm.decode_device(cfg, L.MODE_RECEIVED, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F,
                         res.data_ptr(), pay.data_ptr(), stride, stream=torch.cuda.current_stream().cuda_stream)

    with torch.cuda.stream(s):
        decode()
        decode()
    torch.cuda.synchronize()
    ref_res, ref_pay = res.cpu().numpy().copy(), pay.cpu().numpy().copy()
    rec = np.frombuffer(ref_res.tobytes(), amodem.RESULT_DTYPE)
    assert ((rec["flags"] & (L.FLAG_EXACT | L.FLAG_REPLAY)) != 0).sum() > 0, np.unique(rec["flags"])

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        decode()
    torch.cuda.synchronize()
    for k in range(4):
        res.zero_()
        pay.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(res.cpu().numpy(), ref_res), k
        assert np.array_equal(pay.cpu().numpy(), ref_pay), k
    res.zero_()
    with torch.cuda.stream(s):
        decode()
    torch.cuda.synchronize()
    assert np.array_equal(res.cpu().numpy(), ref_res)
    assert np.array_equal(pay.cpu().numpy(), ref_pay)
    del g
    dm.close()


def test_replay_after_workspace_growth():
    """A captured decode replayed after the same context decoded (eagerly) a larger batch
    of longer frames, and after a larger amod_reserve, so every grow-only workspace
    buffer (counters and lists, detection records, exact-kernel scratch) was reallocated:
    the retired buffers the graph references stay alive (runtime.cpp DevBuf), so the
    replay still returns the eager records (replays must not touch freed
    memory)."""
    import torch
    dev = torch.device("cuda", 0)
    cfg = amodem.preset("standard", "QPSK", 1)
    x, offs, lens = amodem.synth_legacy_batch(cfg, 8, payload_len=200, threads=8)
    F, N = len(offs), int(lens.max())
    xs = torch.zeros(len(x) + 16, dtype=torch.float32, device=dev)
    xs[:len(x)].copy_(torch.from_numpy(x))
    d_off, d_len = torch.from_numpy(offs.astype(np.int64)).to(dev), torch.from_numpy(lens.astype(np.int32)).to(dev)
    stride = amodem.payload_stride(cfg, N)
    res = torch.zeros(F * 96, dtype=torch.uint8, device=dev)
    pay = torch.zeros(F * stride, dtype=torch.uint8, device=dev)
    dm = amodem.Demodulator(0)
    dm.reserve(cfg, F, N)
    s = torch.cuda.Stream()

    def decode():
        dm.decode_device(cfg, L.MODE_RECEIVED, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F, res.data_ptr(),
                         pay.data_ptr(), stride, stream=torch.cuda.current_stream().cuda_stream)

    with torch.cuda.stream(s):
        decode()
    torch.cuda.synchronize()
    ref_res, ref_pay = res.cpu().numpy().copy(), pay.cpu().numpy().copy()
    assert (np.frombuffer(ref_res.tobytes(), amodem.RESULT_DTYPE)["status"] == 0).all()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        decode()
    torch.cuda.synchronize()
    # a bigger eager workload on the same context: 64 frames of 4 KB payload (longer frames,
    # more of them) through the host path, then a device-path reservation for 200k samples
    xb, ob, lb = amodem.synth_legacy_batch(cfg, 64, payload_len=4096, threads=8)
    rec_b, _ = dm.decode_batch(xb, ob, lb, cfg=cfg)
    assert (rec_b["status"] == 0).all() and (rec_b["crc_valid"] == 1).all()
    dm.reserve(cfg, 4096, 200000)
    for k in range(3):
        res.zero_()
        pay.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(res.cpu().numpy(), ref_res), k
        assert np.array_equal(pay.cpu().numpy(), ref_pay), k
    del g
    dm.close()


def test_eager_decode_after_capture_before_replay():
    """amod_reserve, then capture, then an EAGER decode before the first replay,
    then replays. The captured decode's counter reset exists only in the graph, so the
    eager decode must zero the exact-list counters itself; frames are listed (wide guard
    bands) so a stale list count would put list writes out of place."""
    import torch
    cfg = amodem.preset("acoustic", "BPSK", 3)
    x, offs, lens = amodem.synth_legacy_batch(cfg, 24, payload_len=64, threads=8)
    sp = float(np.mean(x[x != 0] ** 2))
    rng = np.random.default_rng(11)
    x = (x + rng.standard_normal(len(x)).astype(np.float32) * np.float32(np.sqrt(sp / 10 ** 0.6))).astype(np.float32)
    F, N = len(offs), int(lens.max())
    dev = torch.device("cuda", 0)
    xs = torch.zeros(len(x) + 16, dtype=torch.float32, device=dev)
    xs[:len(x)].copy_(torch.from_numpy(x))
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    stride = amodem.payload_stride(cfg, N)
    res = torch.zeros(F * 96, dtype=torch.uint8, device=dev)
    pay = torch.zeros(F * stride, dtype=torch.uint8, device=dev)
    dm = open_with_env(0, AMOD_GUARD_SCALE=50)
    dm.reserve(cfg, F, N)
    s = torch.cuda.Stream()

    def decode():
        dm.decode_device(cfg, L.MODE_RECEIVED, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F,
                         res.data_ptr(), pay.data_ptr(), stride, stream=torch.cuda.current_stream().cuda_stream)

    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):  # the context's first decode is the captured one
        decode()
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        decode()  # eager, before any replay
    torch.cuda.synchronize()
    ref_res, ref_pay = res.cpu().numpy().copy(), pay.cpu().numpy().copy()
    rec = np.frombuffer(ref_res.tobytes(), amodem.RESULT_DTYPE)
    assert ((rec["flags"] & (L.FLAG_EXACT | L.FLAG_REPLAY)) != 0).sum() > 0, np.unique(rec["flags"])
    r2, p2 = dm.decode_batch(x, offs, lens, cfg=cfg, stride=stride)  # host path: a third decode
    assert np.array_equal(r2.tobytes(), ref_res.tobytes())
    for k in range(3):
        res.zero_()
        pay.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert np.array_equal(res.cpu().numpy(), ref_res), k
        assert np.array_equal(pay.cpu().numpy(), ref_pay), k
        with torch.cuda.stream(s):
            decode()  # eager between replays
        torch.cuda.synchronize()
        assert np.array_equal(res.cpu().numpy(), ref_res), k
    del g
    dm.close()
