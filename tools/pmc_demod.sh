#!/bin/bash
# LDS / VALU / instruction-cache counters of k_detect and k_demod on the C2 workload
# (two rocprofv3 --pmc passes). usage (GPU box): bash tools/pmc_demod.sh OUTDIR
set -o pipefail
out=${1:-gpurun_out/pmc_demod}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
BPCS=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_SCA \
  --kernel-trace -d "$GRAFT_REPO_ROOT/$out/lds" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/demod_grid.py" &&
BPCS=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT \
  --kernel-trace -d "$GRAFT_REPO_ROOT/$out/ic" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/demod_grid.py"
