#!/usr/bin/env python3
"""Experiments only: interleaved A/B timing of libamodem.so builds in ONE process.

  python tools/ab.py LIB_A LIB_B [...]   (paths to libamodem.so files)

Each library gets two contexts on the C2 bench workload: the full fast kernel and
k_corr_scan (AMOD_STOP_AFTER=1). Launch rounds alternate between the libraries
(A B A B ...), so GPU clock drift over the run hits every variant alike; per
variant the mean and median kernel time (HIP events, amod_kernel_times) are printed."""
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
    libs = sys.argv[1:]
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
    runs = []
    for path in libs:
        lib = C.CDLL(os.path.abspath(path))
        for name, (rt, args) in L.SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = rt, args
        stops = os.environ.get("AB_STOPS") or ("99,1" if os.environ.get("AB_SCAN") else "99")
        for stop in stops.split(","):  # 99 whole chain, 2 detection only, 1 scan only
            os.environ["AMOD_STOP_AFTER"] = stop
            h = C.c_void_p()
            L.check(lib.amod_open(0, C.byref(h)))
            L.check(lib.amod_reserve(h, C.byref(cfg), F, N))
            run = (lambda lib=lib, h=h: L.check(lib.amod_decode_device(
                h, C.byref(cfg), L.MODE_RECEIVED, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F,
                res.data_ptr(), pay.data_ptr(), stride, 0, None)))
            run()
            L.check(lib.amod_synchronize(h))
            if stop == "99":
                rec = np.frombuffer(res.cpu().numpy().tobytes(), amodem.RESULT_DTYPE)
                assert ((rec["status"] == 0) & (rec["crc_valid"] == 1)).all(), path
            runs.append((os.path.basename(os.path.dirname(path)) + {"99": "/full", "2": "/detect", "1": "/scan"}.get(stop, "/" + stop), lib, h, run))
    os.environ.pop("AMOD_STOP_AFTER", None)
    times = {name: [] for name, *_ in runs}
    for _ in range(3):  # warm-up
        for _, lib, h, run in runs:
            run()
    for rnd in range(int(os.environ.get("AB_ROUNDS", "15"))):
        for name, lib, h, run in runs:
            lib.amod_set_profiling(h, 1)
            for _ in range(3):
                run()
            fm, fn, em, en = C.c_double(), C.c_int64(), C.c_double(), C.c_int64()
            lib.amod_kernel_times(h, C.byref(fm), C.byref(fn), C.byref(em), C.byref(en))
            lib.amod_set_profiling(h, 0)
            times[name].append(fm.value / max(1, fn.value))
    for name, t in times.items():
        t = np.array(t)
        print(f"{name:28s} mean {t.mean():.4f} ms  median {np.median(t):.4f}  min {t.min():.4f}  "
              f"({4 * len(x) / np.median(t) / 1e6:.0f} GB/s at median)", flush=True)


if __name__ == "__main__":
    main()
