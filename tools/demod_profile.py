#!/usr/bin/env python3
"""Diagnostics: k_demod phase marks (AMOD_STAMPS=1, s_memtime per wave) on a bench workload.

  bash tools/build_variants.sh stamps=-DAMOD_DEMOD_STAMPS
  AMODEM_LIB=audio-modem_amd/lib/variants/stamps/libamodem.so python tools/demod_profile.py [c2|c4|c5] [frames]

(the product build compiles k_demod's marks out: only the exact kernel's remain)

Job 1 of each frame: 16 samples folded -> 17 FFT -> 18 band + equalise -> 19 guards + pilot
reductions -> 20 demap + bit stream -> 21 end of job; frame end: 22 start -> 23 parse_need ->
24 parse -> 25 CRC -> 26 stores. Prints median / p10 / p90 cycles between marks, the wave
lifetime and the frames per wave."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    conf = sys.argv[1] if len(sys.argv) > 1 else "c2"
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    env = bench.Env()
    os.environ["AMOD_STAMPS"] = "1"  # (read when the workload's context opens)
    wl = bench.Workload(env, conf, frames, snr=10.0)
    del os.environ["AMOD_STAMPS"]
    for _ in range(23):
        wl.step()
    wl.dm.synchronize()
    st = np.zeros(wl.F * 32, dtype=np.uint64)
    n = env.lib.amod_debug_stamps(wl.dm.ctx, st.ctypes.data, st.size)
    st = st[:n].reshape(-1, 32).astype(np.int64)
    print(f"{conf}: {wl.F} frames x {int(wl.dlens[0])} samples")
    for seq in ([16, 17, 18, 19, 20, 21], [22, 23, 24, 25, 26], [24, 30, 31, 25]):
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
              f"p90 {np.percentile(b - a, 90):.0f}; start spread {a.max() - a.min()}, kernel span {b.max() - a.min()}; "
              f"frames per wave {wl.F / ok.sum():.2f}")
        # per wave (its first frame f = F - 1 - w, frames last-first): lifetime by the number
        # of frames it took and by XCD (blockIdx % 8) and SIMD (wave in the workgroup)
        f_idx = np.nonzero(ok)[0]
        w = wl.F - 1 - f_idx
        nw = int(ok.sum())
        life = (b - a).astype(np.float64)
        nfw = (wl.F - 1 - w) // nw + 1  # frames w, w + nw, ... below F
        for k in np.unique(nfw):
            sel = nfw == k
            print(f"  waves with {k} frames: {sel.sum()}  lifetime median {np.median(life[sel]):.0f}  "
                  f"p90 {np.percentile(life[sel], 90):.0f}  per frame {np.median(life[sel]) / k:.0f}")
        blk = w // 4
        print("  lifetime median by XCD:", [int(np.median(life[(blk % 8) == x])) for x in range(8)])
        print("  lifetime median by wave slot:", [int(np.median(life[(w % 4) == x])) for x in range(4)])
        start = a - a.min()
        print(f"  start offsets: median {np.median(start):.0f} p90 {np.percentile(start, 90):.0f} max {start.max()}")
    wl.close()


if __name__ == "__main__":
    main()
