#!/usr/bin/env python3
"""Diagnostics: k_detect cost by stage on the C2 workload (AMOD_STOP_AFTER: 0 stream
pass + normalised sums, 10 Schmidl-Cox caps, 11 candidate compaction, 12 candidate
slide, 1 the coarse decision (k_corr_scan), 2 fine timing, unset = the full chain).
usage: python tools/stage_cost.py [STOP ...]   (each value in its own process for PMC runs)"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-modem_amd"))


def main():
    import torch
    import amodem
    from amodem import _lib as L
    F = int(os.environ.get("FRAMES", "10000"))
    cfg = amodem.preset("standard", "QPSK", 1)
    x, offs, lens = amodem.synth_legacy_batch(cfg, F, threads=16)
    dev = torch.device("cuda", 0)
    xs = torch.empty(len(x) + 16, dtype=torch.float32, device=dev)
    xs[:len(x)].copy_(torch.from_numpy(x))
    d_off, d_len = torch.from_numpy(offs).to(dev), torch.from_numpy(lens).to(dev)
    stride = amodem.payload_stride(cfg, int(lens.max()))
    res = torch.zeros(F * 96, dtype=torch.uint8, device=dev)
    pay = torch.zeros(F * stride, dtype=torch.uint8, device=dev)
    lib = L.load()
    for stop in (sys.argv[1:] or ["0", "10", "11", "12", "1", "2", "none"]):
        if stop == "none":
            os.environ.pop("AMOD_STOP_AFTER", None)
        else:
            os.environ["AMOD_STOP_AFTER"] = stop
        dm = amodem.Demodulator(0)
        dm.reserve(cfg, F, int(lens.max()))
        run = lambda: dm.decode_device(cfg, L.MODE_RECEIVED, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F,
                                       res.data_ptr(), pay.data_ptr(), stride)
        for _ in range(int(os.environ.get("WARM", "3"))):
            run()
        dm.synchronize()
        lib.amod_set_profiling(dm.ctx, 1)
        for _ in range(int(os.environ.get("REPS", "10"))):
            run()
        ms, n = (C.c_double * 3)(), C.c_int64()
        lib.amod_kernel_breakdown(dm.ctx, ms, C.byref(n))
        print(f"stop={stop:>4}  detect {ms[0] / n.value:.4f} ms  demod {ms[1] / n.value:.4f} ms", flush=True)
        dm.close()


if __name__ == "__main__":
    main()
