"""Diagnostics: fast vs forced-exact decode of noisy standard BPSK rep3 frames, on a
fresh context after another context's use, with k_demod stamps (AMOD_STAMPS=1)."""
import os, sys, numpy as np
os.environ["AMOD_STAMPS"] = "1"
sys.path.insert(0, 'audio-modem_amd')
import amodem
from amodem import _lib as L
cfg = amodem.preset("standard", "BPSK", 3)
x, offs, lens = amodem.synth_legacy_batch(cfg, 48, payload_len=128, threads=8)
rng = np.random.default_rng(7)
sig_pow = float(np.mean(x[x != 0] ** 2))
xn = (x + rng.standard_normal(len(x)).astype(np.float32) * np.float32(np.sqrt(sig_pow / 10 ** 0.5))).astype(np.float32)


def run(tag, d, o, l):
    r, _ = d.decode_batch(xn, o, l, cfg=cfg)
    st = np.zeros(len(o) * 32, dtype=np.uint64)
    n = L.load().amod_debug_stamps(d.ctx, st.ctypes.data, st.size)
    bad = [i for i in range(len(o)) if r["nbits"][i] == 0]
    print(tag, "unwritten", bad, "flags", np.unique(r["flags"], return_counts=True))
    if n:
        st = st[:n].reshape(-1, 32)
        for i in bad[:6]:
            print("  frame", i, "marks", [k for k in range(32) if st[i, k]])
    return r


mode = sys.argv[1] if len(sys.argv) > 1 else "seq"
if mode == "fresh":
    d = amodem.Demodulator(0)
    run("fresh48", d, offs, lens)
    run("again48", d, offs, lens)
elif mode == "seq":
    dm = amodem.Demodulator(0)
    run("dm48", dm, offs, lens)
    d1 = amodem.Demodulator(0)
    run("one", d1, offs[[38]], lens[[38]])
    d1.close()
    d2 = amodem.Demodulator(0)
    run("d2_48", d2, offs, lens)
if mode == "rec":
    d = amodem.Demodulator(0)
    r, _ = d.decode_batch(xn, offs, lens, cfg=cfg)
    e, _ = d.decode_batch(xn, offs, lens, cfg=cfg, options=L.OPT_FORCE_EXACT)
    for i in (0, 1, 3):
        print("fast ", i, {n: r[n][i] for n in r.dtype.names})
        print("exact", i, {n: e[n][i] for n in e.dtype.names})
