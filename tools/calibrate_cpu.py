#!/usr/bin/env python3
"""CPU-baseline calibration (build container only: it runs the reference modem.js).

For each bench workload, builds the same frames the bench decodes (the product's host
transmitter, the synthetic xorshift32 payloads), then times on one thread:
  * the unmodified reference modem.js (tools/time_rx.js, vm.runInThisContext),
  * the JS CPU baseline oracle/rx_cpu.js on the same frames, interleaved with it,
  * the C restatement oracle/amodem_oracle.c.
Writes profiles/cpu_calibration.json. BASELINE.md asks the JS baseline (what bench.py
times on the GPU box with one worker_thread per core) to be within +-15 % of modem.js;
`js_over_modem_js` records the measured ratio (rate / rate)."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-modem_amd"))
sys.path.insert(0, ROOT)

WORK = {
    "c2": ("standard", "QPSK", 1, 1024, False),
    "c3": ("standard", "QAM16", 1, 1024, False),
    "c4": ("standard", "QPSK", 1, 2048, True),
    "c5": ("acoustic", "BPSK", 3, 256, False),
}


def frames_for(key, n):
    import amodem
    from amodem import _lib as L
    preset, mod, rep, plen, chunk = WORK[key]
    cfg = amodem.preset(preset, mod, rep)
    sigs = []
    for i in range(n):
        data = amodem.synth_payload(0x9E3779B9 ^ i, plen)
        if chunk:
            f = amodem.build_data_chunk_frame(data, i, cfg=cfg)
            pre, _ = amodem.tx_silence(cfg, L.TX_CHUNK)
            win = amodem.estimate_frame_samples(2048 + 11, mod, rep)
            f = f[pre:pre + win]
        else:
            f = amodem.build_transmit_signal(data, file_name="f.bin", cfg=cfg)
        sigs.append(np.asarray(f, np.float32))
    return sigs


def main(nframes=40, reps=9):
    from oracle import oracle as O
    out = {"what": "single-thread ms per frame on identical frames: reference modem.js (Node, vm), the JS CPU "
                   "baseline oracle/rx_cpu.js and the C oracle (build container, idle)",
           "frames": nframes, "reps": reps, "workloads": {}}
    with tempfile.TemporaryDirectory() as tmp:
        for key, (preset, mod, rep, _, chunk) in WORK.items():
            n = nframes if key != "c5" else min(nframes, 16)
            sigs = frames_for(key, n)
            lens = np.array([len(s) for s in sigs], np.int32)
            offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
            x = np.concatenate(sigs)
            xf = os.path.join(tmp, f"{key}.f32")
            x.tofile(xf)
            spec = os.path.join(tmp, f"{key}.json")
            with open(spec, "w") as f:
                json.dump({"samples": xf, "offsets": offs.tolist(), "lengths": lens.tolist(), "preset": preset,
                           "mod": mod, "rep": rep, "chunk": chunk}, f)
            t = json.loads(subprocess.run(["node", os.path.join(ROOT, "tools", "time_rx.js"), spec, str(reps)],
                                          capture_output=True, text=True, check=True).stdout)
            c = O.cfg(preset)
            ts = []
            for _ in range(reps):
                dt, st, _ = O.bench_decode(c, x, offs, lens, mod, rep, 1, chunk=chunk)
                assert (st == 0).all(), key
                ts.append(dt / n * 1e3)
            ms_c = float(np.median(ts))
            out["node"] = t["node"]
            out["workloads"][key] = {"samples_per_frame": int(lens[0]), "modem_js_ms": t["ref_ms"],
                                     "js_baseline_ms": t["js_ms"], "oracle_c_ms": ms_c,
                                     "js_over_modem_js": t["ref_ms"] / t["js_ms"],
                                     "ratio_oracle_over_modem_js": t["ref_ms"] / ms_c}
    p = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    with open(p, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
