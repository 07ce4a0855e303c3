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
