"""Several GPUs from one process (amod_group_decode_host; decodeBatch {devices: n}): the
batch is cut into contiguous frame ranges of about equal sample counts, one per context,
decoded at once. On the one-GPU test box the group holds repeated contexts of device 0
(separate streams and workspaces, the same code path as distinct devices). Results must
equal the single-context decode frame for frame, in frame order, whatever the split."""
import numpy as np
import pytest

import amodem
from amodem import _lib as L

pytestmark = pytest.mark.gpu


def _batch():
    cfg = amodem.preset("standard", "QPSK", 1)
    xs, offs, lens = [], [], []
    base = 0
    for k, plen in enumerate([64, 1024, 300, 2000, 17, 900] * 20):
        x, o, l = amodem.synth_legacy_batch(cfg, 1, payload_len=plen, threads=1)
        xs.append(x)
        offs.append(base + int(o[0]))
        lens.append(int(l[0]))
        base += len(x)
    return cfg, np.concatenate(xs), np.array(offs, np.int64), np.array(lens, np.int32)


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_group_equals_single_context(devices):
    cfg, x, offs, lens = _batch()
    dm = amodem.Demodulator(0)
    ref, rpay = dm.decode_batch(x, offs, lens, cfg=cfg)
    dm.close()
    g = amodem.DeviceGroup(devices)
    rec, pay, split = g.decode_batch(x, offs, lens, cfg)
    # frames out of buffer order (offsets permuted): the same results at the same indices
    perm = np.random.default_rng(1).permutation(len(offs))
    rec2, pay2, _ = g.decode_batch(x, offs[perm], lens[perm], cfg)
    g.close()
    assert sum(split) == len(offs) and len(split) == len(devices)
    if len(devices) > 1:
        assert min(split) > 0
    # whole records (the engine-side fields too: a frame's route depends on the frame and on
    # the launch's own capacity, which every frame of a host launch fits) and whole rows
    inv = np.argsort(perm)
    for n in amodem.RESULT_DTYPE.names:
        if n == "reserved":
            continue
        assert (rec[n] == ref[n]).all(), n
        assert (rec2[n][inv] == ref[n]).all(), n
    assert np.array_equal(pay, rpay)
    assert np.array_equal(pay2[inv], rpay)
    assert (ref["status"] == 0).all()


@pytest.mark.parametrize("piece", [40_000, 333_333])
def test_host_pipeline_pieces(monkeypatch, piece):
    """amod_decode_host uploads the samples in pieces on its upload stream and decodes the
    frames whose samples have landed while the next piece goes up (frames in index order
    when their ends never decrease, else after the last piece). Any piece size gives the
    one-piece result: frames in order, permuted, and overlapping slices of one buffer."""
    cfg, x, offs, lens = _batch()
    dm = amodem.Demodulator(0)
    ref, rpay = dm.decode_batch(x, offs, lens, cfg=cfg)
    dm.close()
    monkeypatch.setenv("AMOD_UP_PIECE", str(piece))  # read when a context opens
    dm = amodem.Demodulator(0)
    rec, pay = dm.decode_batch(x, offs, lens, cfg=cfg)
    perm = np.random.default_rng(2).permutation(len(offs))
    rec2, pay2 = dm.decode_batch(x, offs[perm], lens[perm], cfg=cfg)
    # every frame twice, the copies interleaved (non-decreasing ends, shared samples)
    dup = np.repeat(np.arange(len(offs)), 2)
    rec3, pay3 = dm.decode_batch(x, offs[dup], lens[dup], cfg=cfg)
    dm.close()
    inv = np.argsort(perm)
    for n in amodem.RESULT_DTYPE.names:
        assert (rec[n] == ref[n]).all(), n
        assert (rec2[n][inv] == ref[n]).all(), n
        assert (rec3[n] == ref[n][dup]).all(), n
    assert np.array_equal(pay, rpay) and np.array_equal(pay2[inv], rpay)
    assert np.array_equal(pay3, rpay[dup])
    assert (ref["status"] == 0).all()


def test_host_progress_prefixes_final(monkeypatch):
    """amod_decode_host_progress: each decoded piece's records and payload rows come back
    while later pieces upload; progress(done) runs with done increasing to nframes, and
    every prefix it reports is already final (equals the returned arrays and the plain
    amod_decode_host result). In-order frames report as pieces complete; permuted ones
    only after the last piece."""
    cfg, x, offs, lens = _batch()
    dm = amodem.Demodulator(0)
    ref, rpay = dm.decode_batch(x, offs, lens, cfg=cfg)
    dm.close()
    monkeypatch.setenv("AMOD_UP_PIECE", "40000")
    dm = amodem.Demodulator(0)
    for order in (np.arange(len(offs)), np.random.default_rng(3).permutation(len(offs))):
        seen = []
        rec, pay = dm.decode_batch(x, offs[order], lens[order], cfg=cfg,
                                   progress=lambda d, r, p: seen.append((d, r[:d].copy(), p[:d].copy())))
        done = [d for d, _, _ in seen]
        assert done[-1] == len(offs) and all(a < b for a, b in zip(done, done[1:])), done
        for d, r, p in seen:
            assert r.tobytes() == rec[:d].tobytes() and np.array_equal(p, pay[:d]), d
        for n in amodem.RESULT_DTYPE.names:
            assert (rec[n] == ref[n][order]).all(), n
        assert np.array_equal(pay, rpay[order])
        if order[0] == 0 and order[-1] == len(offs) - 1:
            assert len(done) > 2, done  # in order: reported piece by piece
    dm.close()


def test_host_progress_exception_raised(monkeypatch):
    """A progress callback that raises: the decode still completes, the callback is not
    called again, and decode_batch re-raises that exception (ctypes alone would print it
    and return as if nothing failed); the Demodulator decodes normally afterwards."""
    cfg, x, offs, lens = _batch()
    monkeypatch.setenv("AMOD_UP_PIECE", "40000")
    dm = amodem.Demodulator(0)
    calls = []

    def bad(done, r, p):
        calls.append(done)
        raise KeyError("progress boom")

    with pytest.raises(KeyError, match="progress boom"):
        dm.decode_batch(x, offs, lens, cfg=cfg, progress=bad)
    assert len(calls) == 1
    rec, _ = dm.decode_batch(x, offs, lens, cfg=cfg)
    assert (rec["status"] == 0).all()
    dm.close()


def _assert_same(rec, pay, ref, rpay):
    for n in amodem.RESULT_DTYPE.names:
        if n == "reserved":
            continue
        assert (rec[n] == ref[n]).all(), n
    assert np.array_equal(pay, rpay)


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_resident_group_equals_single_context(devices):
    """amod_group_upload + amod_resident_decode: the batch resident across the group's
    members once, decoded from HBM twice (device path on every member at once, one D2H
    per member): whole records and payload rows equal the single-context decode."""
    cfg, x, offs, lens = _batch()
    dm = amodem.Demodulator(0)
    ref, rpay = dm.decode_batch(x, offs, lens, cfg=cfg)
    dm.close()
    g = amodem.DeviceGroup(devices)
    rb = g.upload(x, offs, lens, cfg)
    split = rb.frames_per_device()
    rec, pay = rb.decode(cfg)
    rec2, pay2 = rb.decode(cfg)
    rb.close()
    g.close()
    assert sum(split) == len(offs) and len(split) == len(devices)
    _assert_same(rec, pay, ref, rpay)
    _assert_same(rec2, pay2, ref, rpay)


def test_group_decode_device_torch_shards():
    """amod_group_decode_device over caller-owned device buffers (torch tensors) and a
    caller stream: member k decodes its own shard; records equal the single-context
    decode of the same frames."""
    import torch
    cfg, x, offs, lens = _batch()
    dm = amodem.Demodulator(0)
    ref, rpay = dm.decode_batch(x, offs, lens, cfg=cfg)
    dm.close()
    dev = torch.device("cuda", 0)
    stride = amodem.payload_stride(cfg, int(lens.max()))
    halves = [(0, len(offs) // 2), (len(offs) // 2, len(offs))]
    g = amodem.DeviceGroup([0, 0])
    keep, shards = [], []
    s = torch.cuda.Stream(dev)
    for k, (a, b) in enumerate(halves):
        lo = int(offs[a]) & ~3
        hi = int((offs[a:b] + lens[a:b]).max())
        xs = torch.zeros(hi - lo + 16, dtype=torch.float32, device=dev)
        xs[:hi - lo].copy_(torch.from_numpy(x[lo:hi]))
        d_off = torch.from_numpy((offs[a:b] - lo).astype(np.int64)).to(dev)
        d_len = torch.from_numpy(lens[a:b].astype(np.int32)).to(dev)
        res = torch.zeros((b - a) * 96, dtype=torch.uint8, device=dev)
        pay = torch.zeros((b - a) * stride, dtype=torch.uint8, device=dev)
        g_ctx = L.load().amod_group_context(g._h, k)
        L.check(L.load().amod_reserve(g_ctx, L.C.byref(cfg), b - a, int(lens[a:b].max())))
        keep += [xs, d_off, d_len, res, pay]
        shards.append({"samples": xs.data_ptr(), "offsets": d_off.data_ptr(), "lengths": d_len.data_ptr(),
                       "results": res.data_ptr(), "payload": pay.data_ptr(), "payload_stride": stride,
                       "nframes": b - a, "stream": s.cuda_stream if k == 0 else 0})
    torch.cuda.synchronize()
    g.decode_device(cfg, L.MODE_RECEIVED, shards)
    g.synchronize()
    s.synchronize()
    rec = np.concatenate([np.frombuffer(keep[5 * k + 3].cpu().numpy().tobytes(), amodem.RESULT_DTYPE)
                          for k in range(2)])
    pay = np.concatenate([keep[5 * k + 4].cpu().numpy().reshape(-1, stride) for k in range(2)])
    g.close()
    _assert_same(rec, pay, ref, rpay)
