import sys, numpy as np
sys.path.insert(0, 'audio-modem_amd')
import amodem
dm = amodem.Demodulator(0)
for preset in ("standard", "acoustic", "narrowband"):
    cfg = amodem.preset(preset, "BPSK", 3)
    x, offs, lens = amodem.synth_legacy_batch(cfg, 48, payload_len=128, threads=8)
    sig_pow = float(np.mean(x[x != 0] ** 2))
    for snr in (5, 6, 7, 8, 10):
        rng = np.random.default_rng(7)
        xn = (x + rng.standard_normal(len(x)).astype(np.float32) * np.float32(np.sqrt(sig_pow / 10 ** (snr / 10)))).astype(np.float32)
        r, _ = dm.decode_batch(xn, offs, lens, cfg=cfg)
        print(preset, snr, "ok", int((r["status"] == 0).sum()), "detected", int((r["preamble_idx"] >= 0).sum()) , "exact", int(((r["flags"] & 0x80) != 0).sum()), np.unique(r["status"], return_counts=True))
