# diagnostics on the GPU box: k_demod stamps and instruction-cache counters
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/diag
timeout -k 10 200 python tools/demod_stamps.py > gpurun_out/diag/stamps.txt 2>&1 && cat gpurun_out/diag/stamps.txt &&
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAIT_INST_ANY --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/diag/ic -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --cpu-frames -1 --no-e2e --stream-chunks 0 > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/diag/ic.err; echo ic rc=$?
