#!/bin/bash
# One GPU call for a change set (GPU box): the whole GPU suite, an A/B of the given
# libraries on C2/C4 (tools/ab_demod.py), the streaming receiver's host phases at C4 scale
# and the default bench line. Each step bounded; stops at the first failure.
# usage: bash tools/session_check.sh OUT LIB_A LIB_B ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
out=${1:-gpurun_out/check}; shift
mkdir -p "$out"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$out/gpu_tests.log" 2>&1
rc=$?; tail -3 "$out/gpu_tests.log"; [ $rc -eq 0 ] || { echo "GPU tests rc=$rc"; exit $rc; }
if [ $# -gt 0 ]; then
  timeout -k 10 400 python3 tools/ab_demod.py "$@" > "$out/ab.log" 2>&1 || { echo "ab rc=$?"; exit 1; }
  grep -E "^c[0-9]" "$out/ab.log"
fi
timeout -k 10 200 python3 tools/stream_diag.py 32000 > "$out/sdiag.log" 2>&1 || { echo "stream diag rc=$?"; exit 1; }
grep "\[stream\]" "$out/sdiag.log" | tail -8
timeout -k 10 400 python3 bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench rc=$?"; exit 1; }
python3 - "$out/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C2", round(d["value"] / 1e11, 3), "e11", d["ms_per_step"], "k_detect", d["roofline"]["kernel_ms_avg"],
      "chain", d["chain"]["kernels_ms_avg"])
for k, v in d["legs"].items():
    print(k, round(v["value"] / 1e11, 3), "e11", v["ms_per_step"], v["roofline"]["kernel"], round(v["roofline"]["frac"], 3))
s = d["stream"]
print("stream", s["device_resident"]["samples_per_s"], s["device_resident"]["phases_ms"], s["device_resident"]["host_share"])
print("host_api", {k: v.get("ms") for k, v in d["host_api"].items()}, "e2e", d["e2e"]["ms"])
PY
