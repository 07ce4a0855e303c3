#!/usr/bin/env python3
"""Diagnostics: frames decoded with a valid CRC, hard vote vs AMOD_OPT_SOFT_COMBINE,
for acoustic BPSK rep3 and standard QPSK rep3 chunk frames over a sweep of noise."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-modem_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import amodem  # noqa: E402
from amodem import _lib as L  # noqa: E402
from test_gpu_soft_combine import _decode, _frames  # noqa: E402

dm = amodem.Demodulator(0)
for mod, cfgname, length, divs in (("BPSK", "acoustic", 128, (1.0, 1.5, 2.0)),
                                   ("QPSK", "standard", 256, (3.0, 5.0, 8.0))):
    cfg = amodem.preset(cfgname, mod, 3)
    for div in divs:
        x, offs, lens = _frames(64, div, 0x50F7, mod=mod, config=cfgname, length=length)
        res = []
        for opt in (0, L.OPT_SOFT_COMBINE):
            rec, _ = _decode(dm, cfg, x, offs, lens, opt)
            res.append(int(((rec["status"] == 0) & (rec["crc_valid"] == 1)).sum()))
        print(mod, "div", div, "hard", res[0], "soft", res[1], flush=True)
