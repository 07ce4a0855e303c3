#!/usr/bin/env python3
"""Experiments only: the C2 chain's per-stage times (amod_kernel_breakdown) for the same
10k frames decoded on the context's own stream vs on a torch stream, and for host-built
vs k_tx-built samples."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-modem_amd"))


def main():
    import torch
    import amodem
    from amodem import _lib as L
    F, N = 10000, 35874
    cfg = amodem.preset("standard", "QPSK", 1)
    x, offs, lens = amodem.synth_legacy_batch(cfg, F, threads=16)
    dev = torch.device("cuda", 0)
    xs = torch.empty(len(x) + 16, dtype=torch.float32, device=dev)
    xs[:len(x)].copy_(torch.from_numpy(x))
    d_off, d_len = torch.from_numpy(offs).to(dev), torch.from_numpy(lens).to(dev)
    stride = amodem.payload_stride(cfg, N)
    res = torch.zeros(F * 96, dtype=torch.uint8, device=dev)
    pay = torch.zeros(F * stride, dtype=torch.uint8, device=dev)
    dm = amodem.Demodulator(0)
    dm.reserve(cfg, F, N)
    lib = L.load()
    ts = torch.cuda.current_stream(dev).cuda_stream
    plan = [("own stream", 0, None), ("torch stream", ts, None), ("own stream", 0, None), ("torch stream", ts, None)]
    for c in os.environ.get("PROBE_CHUNKS", "").split(","):
        if c:
            plan += [(f"chunks={c}", ts, ("AMOD_CHUNKS", c)), ("torch stream", ts, None)]
    for c in os.environ.get("PROBE_XSLOTS", "").split(","):
        if c:
            plan += [(f"xslots={c}", ts, ("AMOD_XSLOTS", c)), ("torch stream", ts, None)]
    for label, stream, knob in plan:
        for k in ("AMOD_CHUNKS", "AMOD_XSLOTS"):
            os.environ.pop(k, None)
        if knob:
            os.environ[knob[0]] = knob[1]
        for _ in range(3):
            dm.decode_device(cfg, L.MODE_RECEIVED, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F,
                             res.data_ptr(), pay.data_ptr(), stride, stream=stream)
        torch.cuda.synchronize()
        dm.synchronize()
        lib.amod_set_profiling(dm.ctx, 1)
        for _ in range(20):
            dm.decode_device(cfg, L.MODE_RECEIVED, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F,
                             res.data_ptr(), pay.data_ptr(), stride, stream=stream)
        torch.cuda.synchronize()
        dm.synchronize()
        ms = (C.c_double * 3)()
        n = C.c_int64()
        lib.amod_kernel_breakdown(dm.ctx, ms, C.byref(n))
        lib.amod_set_profiling(dm.ctx, 0)
        print(f"{label:14s} detect {ms[0] / n.value:.4f}  demod+aux {ms[1] / n.value:.4f}  exactB {ms[2] / n.value:.4f} "
              f"total {(ms[0] + ms[1] + ms[2]) / n.value:.4f} ms", flush=True)
    dm.close()


if __name__ == "__main__":
    main()
