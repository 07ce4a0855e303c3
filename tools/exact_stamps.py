#!/usr/bin/env python3
"""Diagnostics: s_memtime marks inside k_decode_exact (AMOD_STAMPS=1) on C5 frames
(acoustic BPSK rep3 256 B, 10 dB AWGN) forced onto the exact path: 8 start,
9 preprocess done, 10 Schmidl-Cox done, 11 fine timing done, 12 demodulation done."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-modem_amd"))


def main():
    os.environ["AMOD_STAMPS"] = "1"
    import amodem
    from amodem import _lib as L
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    cfg = amodem.preset("acoustic", "BPSK", 3)
    x, offs, lens = amodem.synth_legacy_batch(cfg, F, payload_len=256, threads=16)
    sp = float(np.mean(x[x != 0] ** 2))
    rng = np.random.default_rng(1)
    x = (x + rng.standard_normal(len(x)).astype(np.float32) * np.float32(np.sqrt(sp / 10 ** (float(os.environ.get("SNR", "10")) / 10)))).astype(np.float32)
    dm = amodem.Demodulator(0)
    if len(sys.argv) > 2:  # default routing: the frames the fast path lists
        rec, _ = dm.decode_batch(x, offs, lens, cfg=cfg)
        st = np.zeros(F * 32, dtype=np.uint64)
        n = L.load().amod_debug_stamps(dm.ctx, st.ctypes.data, st.size)
        st = st[:n].reshape(-1, 32).astype(np.int64)
        for i in np.nonzero(rec["flags"] & L.FLAG_EXACT)[0]:
            print("frame", i, "flags", hex(int(rec["flags"][i])), "coarse", int(rec["coarse_idx"][i]),
                  "marks", [int(st[i, b] - st[i, a]) if st[i, a] and st[i, b] else None for a, b in ((8, 9), (9, 10), (10, 11), (11, 12))])
        return
    for opt in (L.OPT_FORCE_EXACT, L.OPT_FORCE_EXACT):
        t = time.perf_counter()
        rec, _ = dm.decode_batch(x, offs, lens, cfg=cfg, options=opt)
        print("force-exact decode %.2f ms (host-inclusive), ok %d/%d" % (1e3 * (time.perf_counter() - t), (rec["status"] == 0).sum(), F))
    st = np.zeros(F * 32, dtype=np.uint64)
    n = L.load().amod_debug_stamps(dm.ctx, st.ctypes.data, st.size)
    st = st[:n].reshape(-1, 32).astype(np.int64)
    for a, b in ((8, 9), (9, 10), (10, 11), (11, 12), (8, 12)):
        ok = (st[:, a] != 0) & (st[:, b] != 0)
        if ok.any():
            d = st[ok, b] - st[ok, a]
            print(f"  {a} -> {b}  n={ok.sum()}  median {np.median(d):10.0f}  max {d.max():10.0f}")


if __name__ == "__main__":
    main()
