import os, sys, ctypes as C
import numpy as np
os.environ["AMOD_STAMPS"] = "1"
sys.path.insert(0, "audio-modem_amd")
import amodem
from amodem import _lib as L
cfg = amodem.preset("standard", sys.argv[1], 1)
n = 64
x, offs, lens = amodem.synth_legacy_batch(cfg, n, payload_len=1024, threads=16)
dm = amodem.Demodulator(0)
rec, pay = dm.decode_batch(x, offs, lens, cfg=cfg)
st = np.zeros(n * 32, np.uint64)
L.load().amod_debug_stamps(dm.ctx, st.ctypes.data, n * 32)
st = st.reshape(n, 32)[:, 20:28]
f = lambda v: np.array([v], np.uint32).view(np.float32)[0]
for i in range(16):
    s = st[i]
    print(i, "flags", rec["flags"][i] & 0xff, "off%4", offs[i] % 4, "CB %.6f CBL %.6f CBH %.6f" % (f(s[0]), f(s[1]), f(s[2])), "U", int(s[3]), "LO", int(s[4]), "HI", int(s[5]), "ncand", int(s[6]), "errw %.3g" % f(s[7]))
