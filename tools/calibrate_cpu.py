#!/usr/bin/env python3
"""CPU-baseline calibration (build container only: it runs the reference modem.js).

Times the reference (tests/golden/time_reference.js: unmodified modem.js under Node,
one thread) and the C restatement oracle/amodem_oracle.c (one thread) on the same
frames of each bench workload, and writes profiles/cpu_calibration.json with the
per-workload ratio oracle_rate / modem.js_rate. bench.py's cpu_baseline divides its
measured oracle rate by this ratio to state the modem.js-equivalent rate."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-modem_amd"))
sys.path.insert(0, ROOT)


def main(nframes=40, reps=7):
    import amodem
    from amodem import _lib as L
    from oracle import oracle as O
    ref = json.loads(subprocess.run(["node", os.path.join(ROOT, "tests", "golden", "time_reference.js"), str(nframes),
                                     str(reps)], capture_output=True, text=True, check=True).stdout)
    out = {"what": "single-thread ms per frame: reference modem.js (Node, vm) vs the C oracle on identical frames",
           "node": ref["node"], "frames": nframes, "reps": reps, "workloads": {}}
    work = {
        "c2": ("standard", "QPSK", 1, 1024, False),
        "c3": ("standard", "QAM16", 1, 1024, False),
        "c4": ("standard", "QPSK", 1, 2048, True),
        "c5": ("acoustic", "BPSK", 3, 256, False),
    }
    for key, (preset, mod, rep, plen, chunk) in work.items():
        cfg = amodem.preset(preset, mod, rep)
        n = nframes if key != "c5" else min(nframes, 16)
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
            sigs.append(f)
        lens = np.array([len(s) for s in sigs], np.int32)
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        x = np.concatenate(sigs).astype(np.float32)
        c = O.cfg(preset)
        ts = []
        for _ in range(reps):
            t, st, _ = O.bench_decode(c, x, offs, lens, mod, rep, 1, chunk=chunk)
            assert (st == 0).all(), key
            ts.append(t / n * 1e3)
        ms_c = float(np.median(ts))
        out["workloads"][key] = {"samples_per_frame": int(lens[0]), "modem_js_ms": ref[key]["ms"], "oracle_c_ms": ms_c,
                                 "ratio_oracle_over_modem_js": ref[key]["ms"] / ms_c}
    p = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    with open(p, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
