#!/usr/bin/env python3
"""Diagnostics: k_decode_exact's stage marks (AMOD_STAMPS=1: 8 start, 9 preprocess, 10
Schmidl-Cox, 11 fine timing, 12 demodulation, 13/14 sub-marks) for the frames the fast
path lists on the bench's C5 workload at 10 dB, plus the aux-stream chain timing.
  python tools/c5_exact_marks.py [frames]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from amodem import _lib as L
    frames = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    env = bench.Env()
    wl = bench.Workload(env, "c5", frames, snr=10.0)
    for _ in range(10):
        wl.step()
    os.environ["AMOD_STAMPS"] = "1"
    wl.step()
    wl.dm.synchronize()
    del os.environ["AMOD_STAMPS"]
    st = np.zeros(wl.F * 32, dtype=np.uint64)
    n = env.lib.amod_debug_stamps(wl.dm.ctx, st.ctypes.data, st.size)
    st = st[:n].reshape(-1, 32).astype(np.int64)
    rec = wl.results() if hasattr(wl, "results") else None
    rows = np.nonzero(st[:, 8])[0]
    print(f"c5 10 dB: {wl.F} frames x {int(wl.dlens[0])} samples; {len(rows)} frames through k_decode_exact")
    for i in rows:
        m = st[i]
        marks = {f"{a}->{b}": int(m[b] - m[a]) for a, b in ((8, 13), (13, 14), (14, 9), (9, 10), (10, 15), (8, 15), (15, 11), (11, 12), (8, 12))
                 if m[a] and m[b]}
        rt = (m[2] - m[1]) / 100.0 if m[1] and m[2] else None  # s_memrealtime: 100 MHz
        print("frame", int(i), marks, "range", int(m[7]) >> 32, int(m[7]) & 0xFFFFFFFF,
              "8->15 real us", rt, "start rel us", (m[1] - st[rows, 1].min()) / 100.0)
    wl.close()


if __name__ == "__main__":
    main()
