#!/usr/bin/env python3
"""Diagnostics: histogram of exact-path flags for a synthetic legacy batch.
  python tools/flags_hist.py MOD NFRAMES [PAYLOAD] [PRESET]"""
import os
import sys
from collections import Counter

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-modem_amd"))


def main():
    import amodem
    mod = sys.argv[1] if len(sys.argv) > 1 else "QAM16"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    plen = int(sys.argv[3]) if len(sys.argv) > 3 else 1024
    cfg = amodem.preset(sys.argv[4] if len(sys.argv) > 4 else "standard", mod, 1)
    x, offs, lens = amodem.synth_legacy_batch(cfg, n, payload_len=plen, threads=16)
    dm = amodem.Demodulator(0)
    rec, pay = dm.decode_batch(x, offs, lens, cfg=cfg)
    fl = rec["flags"] & ~(1 << 15)
    print(mod, n, "frames; status", Counter(rec["status"].tolist()), "crc_valid", int(rec["crc_valid"].sum()))
    print("flags", sorted(Counter(fl.tolist()).items()))
    print("preamble_idx", Counter(rec["preamble_idx"].tolist()).most_common(4))


if __name__ == "__main__":
    main()
