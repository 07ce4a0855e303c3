#!/usr/bin/env python3
"""Diagnostics: where the exact kernel's time goes on chunk windows it demodulates
(AMOD_STAMPS: s_memtime marks per listed frame): C5 acoustic BPSK rep3 256 B chunk windows
at noise divisor 1.5 (the soft chunk leg's batch), hard vote (DEMAP-listed frames).
8 -> 11 frame start, 11 -> 12 channel estimate + data symbols, 12 -> 17 vote, 17 -> 16 frame end."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    env = bench.Env()
    os.environ["AMOD_STAMPS"] = "1"
    wl = bench.Workload(env, "c5c", int(sys.argv[1]) if len(sys.argv) > 1 else 2000, 10 * np.log10(1.5))
    del os.environ["AMOD_STAMPS"]
    for _ in range(3):
        wl.step()
    wl.dm.synchronize()
    rec = wl.records()
    st = np.zeros(wl.F * 32, dtype=np.uint64)
    n = env.lib.amod_debug_stamps(wl.dm.ctx, st.ctypes.data, st.size)
    st = st[:n].reshape(-1, 32).astype(np.int64)
    listed = np.nonzero(rec["flags"] & env.L.FLAG_EXACT)[0]
    print(f"{wl.F} windows, {len(listed)} listed; symbols per window {(int(wl.dlens[0]) - 3 * wl.cfg.symbol_len) // wl.cfg.symbol_len}")
    for a, b, what in ((8, 11, "start"), (11, 12, "CE + symbols"), (12, 17, "vote"), (17, 16, "parse + CRC + rows"),
                       (12, 16, "vote + end"), (8, 16, "whole")):
        ok = (st[:, a] != 0) & (st[:, b] != 0) & (st[:, b] >= st[:, a])
        if ok.any():
            d = st[ok, b] - st[ok, a]
            print(f"  {what:14s} n={ok.sum():5d} median {np.median(d):10.0f} p90 {np.percentile(d, 90):10.0f} cycles")
    wl.close()


if __name__ == "__main__":
    main()
