#!/usr/bin/env python3
"""Diagnostics: wave 0's s_memtime timeline inside k_decode_fast (AMOD_STAMPS=1).

Marks: 0 entry, 1 stream pass + block sums, 2 SC block-start metrics, 3 SC
candidates, 4 SC argmax, 5 SC plateau/decision, 6 fine timing, 7 FFT tables,
14 FFT rounds done, 15 finish. Prints the median/p10/p90 cycles between
consecutive marks (per workgroup, so it includes time shared with the other
workgroups on the CU)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-modem_amd"))
NAMES = {0: "entry", 1: "stream", 2: "sc_blocks", 3: "sc_cand", 4: "sc_argmax", 5: "sc_done", 6: "fine",
         7: "fft_tables", 8: "r1_loaded", 9: "r1_fft", 10: "r1_G", 11: "r1_band", 12: "r1_barrier",
         16: "r2_loaded", 17: "r2_fft", 18: "r2_band", 19: "r2_barrier", 14: "fft_rounds", 15: "finish"}


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
    order = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 16, 17, 18, 19, 14, 15]
    have = [k for k in order if (st[:, k] != 0).any()]
    print(f"frames {F}  marks {have}")
    prev = None
    for k in have:
        if prev is not None:
            ok = (st[:, k] != 0) & (st[:, prev] != 0)
            d = st[ok, k] - st[ok, prev]
            print(f"  {NAMES.get(prev, prev):>12s} -> {NAMES.get(k, k):<12s} n={ok.sum():6d}  median {np.median(d):9.0f}"
                  f"  p10 {np.percentile(d, 10):9.0f}  p90 {np.percentile(d, 90):9.0f} cycles")
        prev = k
    ok = (st[:, 0] != 0) & (st[:, 15] != 0)
    tot = st[ok, 15] - st[ok, 0]
    print(f"  frame total median {np.median(tot):.0f} cycles, p90 {np.percentile(tot, 90):.0f}")
    t0 = st[ok, 0] - st[ok, 0].min()
    t1 = st[ok, 15] - st[ok, 0].min()
    print(f"  span {t1.max():.0f} cycles; sum(frame)/span = {tot.sum() / t1.max():.1f} concurrent frames")
    # start-time histogram of the first 512 frames (dispatch pattern)
    print("  first frames start:", np.sort(t0)[:8], "... frame 256..263:", np.sort(t0)[256:264])
    dm.close()


if __name__ == "__main__":
    main()
