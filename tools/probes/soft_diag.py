"""Experiments only: fast soft-combining decode vs the exact kernel's, per frame (first
differing payload byte, record fields)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "audio-modem_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import amodem  # noqa: E402
from amodem import _lib as L  # noqa: E402
from test_gpu_soft_combine import _frames  # noqa: E402

div = float(sys.argv[1]) if len(sys.argv) > 1 else 1.5
cfg = amodem.preset("acoustic", "BPSK", 3)
dm = amodem.Demodulator(0)
x, offs, lens = _frames(16, div, 0x5A5A + int(10 * div), rep=3, mod="BPSK", config="acoustic", length=128)
fast, fp = dm.decode_batch(x, offs, lens, cfg=cfg, mode=L.MODE_CHUNK, options=L.OPT_SOFT_COMBINE)
ex, ep = dm.decode_batch(x, offs, lens, cfg=cfg, mode=L.MODE_CHUNK, options=L.OPT_SOFT_COMBINE | L.OPT_FORCE_EXACT)
hd, hp = dm.decode_batch(x, offs, lens, cfg=cfg, mode=L.MODE_CHUNK, options=0)
for i in range(len(fast)):
    pv = min(fast["payload_valid"][i], ex["payload_valid"][i])
    a, b = fp[i, :pv], ep[i, :pv]
    d = np.nonzero(a != b)[0]
    dh = np.nonzero(hp[i, :pv] != b)[0]
    print(i, "fast", fast["status"][i], fast["crc_valid"][i], fast["flags"][i], fast["payload_valid"][i],
          "exact", ex["status"][i], ex["crc_valid"][i], ex["payload_valid"][i], "hard crc", hd["crc_valid"][i],
          "ndiff", len(d), "first", d[:4].tolist(), "xor", [int(a[k] ^ b[k]) for k in d[:4]],
          "hard-vs-exact ndiff", len(dh))
dm.close()
