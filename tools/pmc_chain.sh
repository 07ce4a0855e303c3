#!/bin/bash
# SQ counters of the fast-path launches (k_detect, k_demod) on the C2 workload, one
# rocprofv3 --pmc pass (8 SQ counters), kernel stats in the same directory.
# usage (GPU box): bash tools/pmc_chain.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/pmc_chain}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
BPCS=0 FRAMES=10000 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
  --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/demod_grid.py"
