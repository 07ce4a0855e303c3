"""Chunk mode runs list A (frames routed to the exact kernel before any demodulation) after
k_demod on the launch stream, not beside it on the aux stream (VERDICT
r4 item 7). A device-path batch mixes short chunk windows with long ones past the fast-path
capacity of the latest amod_reserve (AMOD_FLAG_BIG: list A), in both orders and repeated:
every long window comes back from the exact kernel with the same status, bytes and CRC as
a decode whose capacity holds it (all fast), and the short ones are untouched; an empty
list A (every window short) decodes the same as before."""
import numpy as np
import pytest

import amodem
from amodem import _lib as L

pytestmark = pytest.mark.gpu


def _windows(sizes, seed):
    cfg = amodem.preset("standard", "QPSK", 1)
    dm = amodem.Demodulator(0)
    pk = [amodem.packet_chunk(amodem.synth_payload(seed ^ i, n), i) for i, n in enumerate(sizes)]
    x, offs, lens = dm.transmit_batch(cfg, pk, L.TX_CHUNK)
    dm.close()
    pre, _ = amodem.tx_silence(cfg, L.TX_CHUNK)
    wins = np.array([amodem.estimate_frame_samples(n + 11, "QPSK", 1) for n in sizes], np.int32)
    return cfg, x, offs + pre, wins


def _decode(dm, cfg, x, offs, lens, cap, reps=2):
    import torch
    dev = torch.device("cuda", 0)
    xs = torch.zeros(len(x) + 16, dtype=torch.float32, device=dev)
    xs[:len(x)].copy_(torch.from_numpy(x))
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    F, N = len(offs), int(lens.max())
    stride = amodem.payload_stride(cfg, N)
    dm.reserve(cfg, F, N)    # the exact kernel's workspace holds the longest window
    dm.reserve(cfg, F, cap)  # the fast path's capacity: the latest reservation's
    out = []
    for _ in range(reps):
        res = torch.zeros(F * 96, dtype=torch.uint8, device=dev)
        pay = torch.zeros(F * stride, dtype=torch.uint8, device=dev)
        dm.decode_device(cfg, L.MODE_CHUNK, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F, res.data_ptr(),
                         pay.data_ptr(), stride, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        out.append((np.frombuffer(res.cpu().numpy().tobytes(), amodem.RESULT_DTYPE), pay.cpu().numpy().reshape(F, stride)))
    return out


@pytest.mark.parametrize("order", ["short_first", "long_first", "interleaved"])
def test_big_windows_in_chunk_mode(order):
    short, long_ = [64] * 48, [2048] * 8
    sizes = {"short_first": short + long_, "long_first": long_ + short,
             "interleaved": [s for pair in zip(short[:8], long_) for s in pair] + short[8:]}[order]
    cfg, x, offs, lens = _windows(sizes, 0x5EED)
    cap = int(lens[np.array(sizes) == 64].max())
    big = lens > cap
    assert big.sum() == 8
    dm = amodem.Demodulator(0)
    try:
        fast = _decode(dm, cfg, x, offs, lens, int(lens.max()), reps=1)[0]
        mixed = _decode(dm, cfg, x, offs, lens, cap)
    finally:
        dm.close()
    rf, pf = fast
    assert (rf["status"] == 0).all() and (rf["crc_valid"] == 1).all()
    assert not (rf["flags"] & L.FLAG_EXACT).any()
    for rm, pm in mixed:
        assert ((rm["flags"] & L.FLAG_EXACT) != 0).tolist() == big.tolist()
        for name in ("status", "frame_type", "seq_num", "data_len", "crc_valid", "expected_crc", "actual_crc"):
            assert (rm[name] == rf[name]).all(), name
        for i in range(len(sizes)):
            n = int(rf["payload_valid"][i])
            assert np.array_equal(pm[i, :n], pf[i, :n]), i
        assert np.array_equal(rm["flags"][~big], rf["flags"][~big])
