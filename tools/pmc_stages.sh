#!/bin/bash
# VALU / SALU instruction counts of k_detect by stage (tools/stage_cost.py), and the GPU
# clock under the C2 chain (GRBM_GUI_ACTIVE over the kernel time). usage (GPU box):
#   bash tools/pmc_stages.sh OUTDIR
set -o pipefail
out=$(realpath -m "${1:-gpurun_out/pmc_stages}")
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for st in ${STAGES:-0 10 12 1 2 none}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-trace -d "$out/s_$st" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/stage_cost.py" $st > "$out/s_$st.log" 2>&1 || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d "$out/grbm" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/stage_cost.py" none > "$out/grbm.log" 2>&1
