"""amod_pipe_* (Python `Pipeline`): consecutive device decodes alternate between two
contexts so batch i + 1's detection overlaps batch i's demodulation. Overlap must not
change a result: every batch's records and payload rows equal one context's serial
decode of that batch, byte for byte, with result buffers reused two batches later (their
copies enqueued on the caller's stream between calls, and zeroed on it before each
call: the pipe's ordering makes both safe), batches of different sizes and frame contents, and received and chunk mode
in one sequence. The serial path itself is pinned to the oracle by the other GPU tests;
here a sample is checked against the C oracle (decodeReceivedSignal, modem.js:557-654)
as well."""
import numpy as np
import pytest

import amodem
from amodem import _lib as L
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _batches():
    """(cfg, mode, samples, offsets, lengths) per batch: legacy QPSK frames with different
    payload seeds and counts, and one chunk-mode batch of short windows."""
    cfg = amodem.preset("standard", "QPSK", 1)
    out = []
    for i, (n, first) in enumerate([(300, 0), (517, 1000), (64, 5000), (900, 9000), (300, 20000)]):
        x, offs, lens = amodem.synth_legacy_batch(cfg, n, 256, "p.bin", first)
        out.append((cfg, L.MODE_RECEIVED, x, offs, lens))
    dm = amodem.Demodulator(0)
    pk = [amodem.packet_chunk(amodem.synth_payload(0xB0B ^ i, 48), i) for i in range(700)]
    x, offs, lens = dm.transmit_batch(cfg, pk, L.TX_CHUNK)
    dm.close()
    pre, _ = amodem.tx_silence(cfg, L.TX_CHUNK)
    win = amodem.estimate_frame_samples(48 + 11, "QPSK", 1)
    out.insert(3, (cfg, L.MODE_CHUNK, x, offs + pre, np.full(len(offs), win, np.int32)))
    return out


def _dev(torch, b):
    cfg, mode, x, offs, lens = b
    dev = torch.device("cuda", 0)
    xs = torch.zeros(len(x) + 16, dtype=torch.float32, device=dev)
    xs[:len(x)].copy_(torch.from_numpy(x))
    return (xs, torch.from_numpy(offs.astype(np.int64)).to(dev), torch.from_numpy(lens.astype(np.int32)).to(dev))


def test_pipeline_equals_serial_decodes():
    import torch
    bs = _batches()
    F = max(len(b[3]) for b in bs)
    N = max(int(b[4].max()) for b in bs)
    cfg = bs[0][0]
    stride = amodem.payload_stride(cfg, N)
    dev = torch.device("cuda", 0)
    ins = [_dev(torch, b) for b in bs]

    # one context, serial
    ref = []
    dm = amodem.Demodulator(0)
    dm.reserve(cfg, F, N)
    for b, (xs, do, dl) in zip(bs, ins):
        n = len(b[3])
        res = torch.zeros(n * 96, dtype=torch.uint8, device=dev)
        pay = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
        dm.decode_device(cfg, b[1], xs.data_ptr(), do.data_ptr(), dl.data_ptr(), n, res.data_ptr(), pay.data_ptr(),
                         stride, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        ref.append((res.cpu().numpy().tobytes(), pay.cpu().numpy().tobytes()))

    # the pipe over dm and a second context, twice through the sequence; result buffers
    # in a ring of two, each copied out on the caller's stream after the next call
    dm2 = amodem.Demodulator(0)
    dm2.reserve(cfg, F, N)
    pipe = dm.pipeline(dm2)
    s = torch.cuda.Stream(dev)
    ring = [(torch.zeros(F * 96, dtype=torch.uint8, device=dev), torch.zeros(F * stride, dtype=torch.uint8, device=dev))
            for _ in range(2)]
    host = []
    seq = list(range(len(bs))) * 2
    with torch.cuda.stream(s):
        for j, i in enumerate(seq):
            b, (xs, do, dl) = bs[i], ins[i]
            n = len(b[3])
            res, pay = ring[j % 2]
            # (the kernels write each slot's decoded prefix only: zeroed on s, before the
            # call, as the serial reference's fresh buffers are)
            res.zero_()
            pay.zero_()
            pipe.decode_device(cfg, b[1], xs.data_ptr(), do.data_ptr(), dl.data_ptr(), n, res.data_ptr(),
                               pay.data_ptr(), stride, stream=s.cuda_stream)
            if j > 0:  # decode j - 1 is ordered on s now: copy its rows out
                pn = len(bs[seq[j - 1]][3])
                pr, pp = ring[(j - 1) % 2]
                host.append((pr[:pn * 96].to("cpu", non_blocking=False), pp[:pn * stride].to("cpu", non_blocking=False)))
        pipe.flush(s.cuda_stream)
        pn = len(bs[seq[-1]][3])
        pr, pp = ring[(len(seq) - 1) % 2]
        host.append((pr[:pn * 96].cpu(), pp[:pn * stride].cpu()))
    s.synchronize()
    assert len(host) == len(seq)
    for j, i in enumerate(seq):
        assert host[j][0].numpy().tobytes() == ref[i][0], (j, i)
        assert host[j][1].numpy().tobytes() == ref[i][1], (j, i)

    # the fast use: each batch's buffers zeroed and its rows copied out on the slot's own
    # stream (amod_pipe_next_stream), no caller stream at all
    host = []
    for j, i in enumerate(seq):
        b, (xs, do, dl) = bs[i], ins[i]
        n = len(b[3])
        res, pay = ring[j % 2]
        with torch.cuda.stream(torch.cuda.ExternalStream(pipe.next_stream(), device=dev)):
            res.zero_()
            pay.zero_()
            pipe.decode_device(cfg, b[1], xs.data_ptr(), do.data_ptr(), dl.data_ptr(), n, res.data_ptr(),
                               pay.data_ptr(), stride)
            host.append((res[:n * 96].to("cpu", non_blocking=True), pay[:n * stride].to("cpu", non_blocking=True)))
    pipe.synchronize()
    # (the pinned host copies were made on the slot streams: torch's host allocator records
    # an event on those streams when it frees them, so they go before the pipe's streams do)
    host = [(r.numpy().tobytes(), p.numpy().tobytes()) for r, p in host]
    for j, i in enumerate(seq):
        assert host[j][0] == ref[i][0], (j, i)
        assert host[j][1] == ref[i][1], (j, i)
    pipe.close()
    dm2.close()
    dm.close()

    # every frame decoded, and a sample against the C oracle
    for i, b in enumerate(bs):
        rec = np.frombuffer(ref[i][0], amodem.RESULT_DTYPE)
        assert ((rec["status"] == 0) & (rec["crc_valid"] == 1)).all(), i
    c = O.cfg("standard")
    cfg0, mode0, x, offs, lens = bs[1]
    rec = np.frombuffer(ref[1][0], amodem.RESULT_DTYPE)
    for k in range(0, len(offs), 101):
        r, _ = O.decode(c, x[offs[k]:offs[k] + lens[k]], "QPSK", 1, False)
        assert r.status == 0 and r.preamble_idx == rec["preamble_idx"][k] and r.actual_crc == rec["actual_crc"][k], k


def test_pipeline_arguments():
    a = amodem.Demodulator(0)
    with pytest.raises(RuntimeError):
        a.pipeline(a)  # two distinct contexts
    a.close()


def test_pipeline_stream_switch_and_close_order():
    """a decode issued with a caller stream is joined onto THAT stream when the
    next decode is enqueued, even if the next call passes no stream (slot mode), and a
    Demodulator closed before its Pipeline finishes and closes the pipe first."""
    import torch
    bs = _batches()[:3]
    F = max(len(b[3]) for b in bs)
    N = max(int(b[4].max()) for b in bs)
    cfg = bs[0][0]
    stride = amodem.payload_stride(cfg, N)
    dev = torch.device("cuda", 0)
    ins = [_dev(torch, b) for b in bs]
    a, b2 = amodem.Demodulator(0), amodem.Demodulator(0)
    for dm in (a, b2):
        dm.reserve(cfg, F, N)
    pipe = a.pipeline(b2)
    s = torch.cuda.Stream(dev)
    bufs = [(torch.zeros(F * 96, dtype=torch.uint8, device=dev), torch.zeros(F * stride, dtype=torch.uint8, device=dev))
            for _ in range(3)]
    # decode 0 on the caller stream s, decode 1 in slot mode (no stream): decode 0 must be
    # ordered on s after the second call
    b, (xs, do, dl) = bs[0], ins[0]
    with torch.cuda.stream(s):
        pipe.decode_device(cfg, b[1], xs.data_ptr(), do.data_ptr(), dl.data_ptr(), len(b[3]), bufs[0][0].data_ptr(),
                           bufs[0][1].data_ptr(), stride, stream=s.cuda_stream)
    b, (xs, do, dl) = bs[1], ins[1]
    pipe.decode_device(cfg, b[1], xs.data_ptr(), do.data_ptr(), dl.data_ptr(), len(b[3]), bufs[1][0].data_ptr(),
                       bufs[1][1].data_ptr(), stride)
    with torch.cuda.stream(s):
        r0 = bufs[0][0][:len(bs[0][3]) * 96].cpu().numpy()
    rec = np.frombuffer(r0.tobytes(), amodem.RESULT_DTYPE)
    assert ((rec["status"] == 0) & (rec["crc_valid"] == 1)).all()
    # a third decode in flight, then the Demodulator closed under it: the pipe goes first
    b, (xs, do, dl) = bs[2], ins[2]
    pipe.decode_device(cfg, b[1], xs.data_ptr(), do.data_ptr(), dl.data_ptr(), len(b[3]), bufs[2][0].data_ptr(),
                       bufs[2][1].data_ptr(), stride)
    a.close()
    assert pipe._h is None
    torch.cuda.synchronize()
    rec = np.frombuffer(bufs[2][0][:len(bs[2][3]) * 96].cpu().numpy().tobytes(), amodem.RESULT_DTYPE)
    assert ((rec["status"] == 0) & (rec["crc_valid"] == 1)).all()
    b2.close()
