# diagnostics on the GPU box: k_demod stamps and SQ counters of the C2 chain
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/diag
timeout -k 10 200 python tools/demod_stamps.py > gpurun_out/diag/stamps.txt 2>&1 && cat gpurun_out/diag/stamps.txt &&
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/diag/sq -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --cpu-frames -1 --no-e2e --stream-chunks 0 > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/diag/sq.err; echo sq rc=$?
cd $GRAFT_REPO_ROOT && python tools/pmc_summary.py gpurun_out/diag/sq/run_counter_collection.csv 2>&1 | tail -20
