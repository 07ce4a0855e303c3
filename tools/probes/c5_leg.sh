#!/bin/bash
# Experiments only: why the C5 10 dB leg of the default bench runs slower than a C5-only
# bench (k_demod 1.2 vs 0.8 ms). Same workload after different process histories.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/c5leg; mkdir -p $out
show() { python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for name, l in [("primary", d)] + list(d.get("legs", {}).items()):
    print(sys.argv[1].split("/")[-1], name, round(l["ms_per_step"], 3), {k: round(v, 3) for k, v in l["chain"]["kernels_ms_avg"].items()}, round(l["chain"]["aux_stream_ms_avg"], 3))
PY
}
i=0
for a in "${@:-"--config c5 --snr 10 --legs c5 --stream-chunks 0 --no-e2e --cpu-frames -1"}"; do
  i=$((i+1))
  # an argument may start with VAR=value words: the environment of that run
  envs=(); set -- $a; while [[ "$1" == *=* ]]; do envs+=("$1"); shift; done
  timeout -k 10 300 env "${envs[@]}" python3 bench.py "$@" > $out/r$i.json 2> $out/r$i.err || { echo "run $i failed"; exit 1; }
  show $out/r$i.json
done
