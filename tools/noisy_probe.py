#!/usr/bin/env python3
"""Diagnostics: where a noisy C5 step goes (the exact lists' chain).

  python tools/noisy_probe.py [snr_db=7] [frames=10000]

Prints the per-stage HIP-event times of K decodes on one context (k_detect, k_demod, the
aux stream's list-A chain, the wait for it, list B), the listed frames by route (flags),
and the exact kernel's per-frame phase marks (AMOD_STAMPS: s_memtime cycles) for the
listed frames: 8 -> 13 preprocess pass 1, 13 -> 14 the mean's chain, 14 -> 9 normalise,
9 -> 10 detectPreamble, 10 -> 15 fine timing, 11 -> 12 demodulation; slot 7 = the
recurrence's range [d_lo, d_hi]."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    snr = float(sys.argv[1]) if len(sys.argv) > 1 else 7.0
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    env = bench.Env()
    L = env.L
    os.environ["AMOD_STAMPS"] = "1"  # (read when the workload's context opens)
    wl = bench.Workload(env, "c5", frames, snr=snr)
    del os.environ["AMOD_STAMPS"]
    sync = lambda: env.torch.cuda.synchronize(env.dev)  # noqa: E731
    for _ in range(5):
        wl.step()
    sync()
    env.lib.amod_set_profiling(wl.dm.ctx, 1)
    K = 10
    import time
    t0 = time.perf_counter()
    for _ in range(K):
        wl.step()
    sync()
    dt = (time.perf_counter() - t0) / K
    kms, kn = (C.c_double * L.STAGE_COUNT)(), C.c_int64()
    env.lib.amod_kernel_stages(wl.dm.ctx, kms, L.STAGE_COUNT, C.byref(kn))
    env.lib.amod_set_profiling(wl.dm.ctx, 0)
    st_ms = [kms[i] / max(1, kn.value) for i in range(L.STAGE_COUNT)]
    print(f"C5 {snr} dB, {wl.F} frames: {dt * 1e3:.3f} ms per step (one context)")
    for name, i in (("k_detect", L.STAGE_DETECT), ("k_demod", L.STAGE_DEMOD), ("list B", L.STAGE_EXACT_B),
                    ("aux (list A chain)", L.STAGE_AUX), ("join wait", L.STAGE_JOIN_WAIT),
                    ("demod path", L.STAGE_DEMOD_PATH)):
        print(f"  {name:20s} {st_ms[i]:8.3f} ms")
    rec = wl.records()
    fl = rec["flags"].astype(np.int64)
    listed = np.nonzero(fl & (L.FLAG_EXACT | L.FLAG_REPLAY))[0]
    print(f"listed frames {len(listed)}: exact {int(((fl & L.FLAG_EXACT) != 0).sum())}, "
          f"replayed {int(((fl & L.FLAG_REPLAY) != 0).sum())}")
    hist = {}
    for f in fl[listed]:
        key = "|".join(bench.FLAG_NAMES.get(b, str(b)) for b in range(16) if f & (1 << b) and b != 15) or "-"
        hist[key] = hist.get(key, 0) + 1
    print("  by flags:", dict(sorted(hist.items(), key=lambda kv: -kv[1])))
    print("  status of listed:", dict(zip(*np.unique(rec["status"][listed], return_counts=True))))
    st = np.zeros(wl.F * 32, dtype=np.uint64)
    n = env.lib.amod_debug_stamps(wl.dm.ctx, st.ctypes.data, st.size)
    st = st[:n].reshape(-1, 32)
    sti = st.astype(np.int64)
    for a, b, what in ((8, 13, "pass 1"), (13, 14, "mean chain"), (14, 9, "normalise"), (9, 10, "detectPreamble"),
                       (10, 15, "fine"), (11, 12, "demod"), (8, 12, "whole (demod frames)"),
                       (8, 15, "whole detection")):
        ok = (sti[:, a] != 0) & (sti[:, b] != 0) & (sti[:, b] >= sti[:, a])
        if ok.any():
            d = sti[ok, b] - sti[ok, a]
            print(f"  {what:22s} n={ok.sum():4d} median {np.median(d):10.0f}  p90 {np.percentile(d, 90):10.0f}  "
                  f"max {d.max():10.0f} cycles")
    rng = st[:, 7]
    ok = rng != 0
    if ok.any():
        lo = (rng[ok] >> np.uint64(32)).astype(np.int64)
        hi = (rng[ok] & np.uint64(0xFFFFFFFF)).astype(np.int64)
        span = hi - lo
        print(f"  recurrence ranges n={ok.sum()}: d_lo median {np.median(lo):.0f} (max {lo.max()}), span median "
              f"{np.median(span):.0f} p90 {np.percentile(span, 90):.0f} max {span.max()}; frame {int(wl.dlens[0])}")
        full = int((lo == 0).sum())
        print(f"  ranges starting at 0 (no hull): {full}")
    wl.close()


if __name__ == "__main__":
    main()
