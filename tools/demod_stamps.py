#!/usr/bin/env python3
"""Diagnostics: s_memtime marks inside k_demod (AMOD_STAMPS=1) on the C2 workload:
job 1 of each frame (16 loaded, 17 FFT, 18 band + equalise, 19 guard + pilot
reductions, 20 demap, 21 pack) and the frame end (22 start, 23 parse_need, 24 parse,
25 CRC, 26 stores). Prints median/p10/p90 cycles between consecutive marks."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-modem_amd"))


def main():
    os.environ["AMOD_STAMPS"] = "1"
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
    dm = amodem.Demodulator(0)
    dm.reserve(cfg, F, 35874)
    for _ in range(3):
        dm.decode_device(cfg, L.MODE_RECEIVED, xs.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), F,
                         res.data_ptr(), pay.data_ptr(), stride)
    dm.synchronize()
    st = np.zeros(F * 32, dtype=np.uint64)
    n = lib.amod_debug_stamps(dm.ctx, st.ctypes.data, st.size)
    st = st[:n].reshape(F, 32).astype(np.int64)
    for seq in ([16, 17, 18, 19, 20, 21], [22, 23, 24, 25, 26]):
        for a, b in zip(seq, seq[1:]):
            ok = (st[:, a] != 0) & (st[:, b] != 0)
            d = st[ok, b] - st[ok, a]
            if ok.any():
                print(f"  {a} -> {b}  n={ok.sum():6d}  median {np.median(d):8.0f}  p10 {np.percentile(d, 10):8.0f}"
                      f"  p90 {np.percentile(d, 90):8.0f}")
    ok = (st[:, 21] != 0) & (st[:, 16] != 0)
    print("job 1 total median", np.median(st[ok, 21] - st[ok, 16]))
    ok = (st[:, 21] != 0) & (st[:, 27] != 0)
    if ok.any():
        d = st[ok, 27] - st[ok, 21]
        print(f"job 1 end -> job 2 samples ready: median {np.median(d):.0f} p10 {np.percentile(d, 10):.0f} "
              f"p90 {np.percentile(d, 90):.0f}")
    ok = (st[:, 28] != 0) & (st[:, 29] != 0)
    if ok.any():
        a, b = st[ok, 28], st[ok, 29]
        print(f"waves {ok.sum()}: lifetime median {np.median(b - a):.0f} p10 {np.percentile(b - a, 10):.0f} "
              f"p90 {np.percentile(b - a, 90):.0f}; start spread {a.max() - a.min()}, kernel span {b.max() - a.min()}")


if __name__ == "__main__":
    main()
