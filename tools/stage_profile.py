#!/usr/bin/env python3
"""Diagnostics: cost of each k_decode_fast stage on the bench workload.

AMOD_STOP_AFTER=k makes the fast kernel return after stage k (0 load+stats,
1 Schmidl-Cox, 2 fine timing, 3 FFT/demod, 99 full); the stage cost is the
difference of consecutive rows. Results are not written in cut runs."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-modem_amd"))


def main():
    import torch
    import amodem
    from amodem import _lib as L
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    cfg = amodem.preset("standard", "QPSK", 1)
    x, offs, lens = amodem.synth_legacy_batch(cfg, F, threads=16)
    dev = torch.device("cuda", 0)
    xs = torch.empty(len(x) + 16, dtype=torch.float32, device=dev)
    xs[:len(x)].copy_(torch.from_numpy(x))
    d_off, d_len = torch.from_numpy(offs).to(dev), torch.from_numpy(lens).to(dev)
    stride = amodem.payload_stride(cfg, 35874)
    res = torch.zeros(F * 96, dtype=torch.uint8, device=dev)
    pay = torch.zeros(F * stride, dtype=torch.uint8, device=dev)
    lib = L.load()
    rows = []
    for stop in [int(s) for s in os.environ.get("STAGES", "0,1,2,3,99").split(",")]:
        os.environ["AMOD_STOP_AFTER"] = str(stop)
        dm = amodem.Demodulator(0)
        dm.reserve(cfg, F, 35874)
        run = lambda: dm.decode_device(cfg, L.MODE_RECEIVED, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F,
                                       res.data_ptr(), pay.data_ptr(), stride)
        run(); dm.synchronize()
        lib.amod_set_profiling(dm.ctx, 1)
        for _ in range(5):
            run()
        fm, fn, em, en = C.c_double(), C.c_int64(), C.c_double(), C.c_int64()
        lib.amod_kernel_times(dm.ctx, C.byref(fm), C.byref(fn), C.byref(em), C.byref(en))
        ms = fm.value / fn.value
        rows.append((stop, ms))
        print(f"stop_after={stop:3d}  fast kernel {ms:8.3f} ms  ({4 * len(x) / ms / 1e6:8.1f} GB/s)", flush=True)
        dm.close()
    prev = 0.0
    for stop, ms in rows:
        print(f"  stage<= {stop:3d}: +{ms - prev:7.3f} ms")
        prev = ms


if __name__ == "__main__":
    main()
