#!/usr/bin/env python3
"""Diagnostics: tools/node_decode_batch.js on the C4 workload (32k chunk windows, a 3.6 GB
Float32Array), run up to N times in fresh Node processes with AMODEM_SEGV_TRACE=1 (the addon
prints its native stack on a crash); prints each run's exit code and the tail of its stderr.
  python tools/node_c4.py [runs] [config]"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    conf = sys.argv[2] if len(sys.argv) > 2 else "c4"
    env = bench.Env()
    wl = bench.Workload(env, conf)
    x = wl.xs[: wl.nsamples].cpu().numpy()
    with tempfile.TemporaryDirectory() as tmp:
        xf = os.path.join(tmp, "x.f32")
        x.tofile(xf)
        spec = os.path.join(tmp, "spec.json")
        with open(spec, "w") as f:
            json.dump({"samples": xf, "offsets": wl.doffs.tolist(), "lengths": wl.dlens.tolist(), "preset": wl.preset,
                       "mod": wl.mod, "rep": wl.cfg.repetition, "chunk": wl.chunk, "reps": 3, "device": env.local}, f)
        del x
        for k in range(runs):
            r = subprocess.run(["node", os.path.join(ROOT, "tools", "node_decode_batch.js"), spec], capture_output=True,
                               text=True, timeout=240, env=dict(os.environ, AMODEM_SEGV_TRACE="1"))
            print(f"run {k}: rc {r.returncode}", flush=True)
            print(r.stderr[-4000:], flush=True)
            if r.returncode == 0:
                print(r.stdout[:600], flush=True)


if __name__ == "__main__":
    main()
