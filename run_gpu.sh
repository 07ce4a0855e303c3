# usage: bash run_gpu.sh <steps...>  (each step bounded; stop at first crash)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -4 gpurun_out/$name.log; echo "rc=$rc"; if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then echo "ABORT after $name"; exit $rc; fi; }
for s in "$@"; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()";;
    tests) run gpu_tests 900 python -m pytest tests -m gpu -q --timeout 600 -p no:cacheprovider;;
    bench) run bench 900 python bench.py --steps 20 --warmup 3;;
    benchc3) run bench_c3 600 python bench.py --config c3 --steps 10 --warmup 2;;
    bench2g) run bench2g 600 env AMOD_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 5 --warmup 2 --cpu-frames -1 --stream-chunks 0 --no-e2e --legs c4,c5;;
    bench2fail) echo "== bench2fail"; timeout -k 10 300 python bench.py --gpus 2 > gpurun_out/bench2fail.log 2>&1; echo "rc=$? (2 expected)"; tail -2 gpurun_out/bench2fail.log;;
    benchc4) run bench_c4 600 python bench.py --config c4 --steps 10 --warmup 2 --stream-chunks 0;;
    stamps) run stamps 300 python tools/stamps.py;;
    stages) run stages 600 env STAGES=${STAGES:-0,1,2,3,99} python tools/stage_profile.py;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv rocpd -- python bench.py --steps 20 --warmup 3 --cpu-frames -1;;
    pmc) run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --cpu-frames -1 &&
         run pmc_sq 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --kernel-trace --stats -d gpurun_out/pmc_sq -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --cpu-frames -1;;
    pmcstages) run pmc_stages 600 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --kernel-trace -d gpurun_out/pmc_stages -o run --output-format csv -- python tools/stage_profile.py;;
    variants) for v in ${VARIANTS:-w5s8}; do run bench_$v 300 env AMODEM_LIB=audio-modem_amd/lib/variants/$v/libamodem.so python bench.py --steps 20 --warmup 3 --cpu-frames -1; done;;
    pmcic) run pmc_ic 600 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_VALU SQ_WAVES --kernel-trace -d gpurun_out/pmc_ic -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --cpu-frames -1;;
    pmcstages2) run pmc_stages2 600 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LEVEL_WAVES SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM --kernel-trace -d gpurun_out/pmc_stages2 -o run --output-format csv -- python tools/stage_profile.py;;
    demodprof) run demod_c2 300 python tools/demod_profile.py c2 && run demod_c4 300 python tools/demod_profile.py c4 && run demod_c5 300 python tools/demod_profile.py c5;;
    pmcc4) run pmc_c4_sq 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --kernel-trace --stats -d gpurun_out/pmc_c4_sq -o run --output-format csv -- python bench.py --config ${PMCCFG:-c4} --legs none --stream-chunks 0 --cpu-frames -1 --no-e2e --steps 5 --warmup 2 &&
           run pmc_c4_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats -d gpurun_out/pmc_c4_fetch -o run --output-format csv -- python bench.py --config ${PMCCFG:-c4} --legs none --stream-chunks 0 --cpu-frames -1 --no-e2e --steps 5 --warmup 2;;
    streamdiag) run stream_diag 300 python tools/stream_diag.py ${NCHUNKS:-32000};;
    emasweep) for W in ${WARMS:-16 4 2 1}; do run ema_w$W 300 env AMOD_EMA_WARM=$W python tools/ema_probe.py ${NCHUNKS:-32000} || exit 1; done;;
    c5stamps) run c5stamps 300 env AMOD_STAMPS=1 python bench.py --config c5 --snr 10 --legs none --stream-chunks 0 --cpu-frames -1 --no-e2e --steps 3 --warmup 1;;
    emaprof) for W in ${WARMS:-16 4}; do mkdir -p gpurun_out/emaprof_w$W && cd gpurun_out/emaprof_w$W && AMOD_EMA_WARM=$W timeout -k 10 300 rocprofv3 --kernel-trace --stats -d . -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/ema_probe.py ${NCHUNKS:-32000} > log.txt 2>&1; rc=$?; cd $GRAFT_REPO_ROOT; echo "emaprof w$W rc=$rc"; [ $rc -eq 0 ] || exit $rc; done;;
    emapmc) mkdir -p gpurun_out/emapmc && cd gpurun_out/emapmc && AMOD_EMA_WARM=2 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_ACTIVE_INST_LDS --kernel-trace -d . -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/ema_probe.py 8000 > log.txt 2>&1; rc=$?; cd $GRAFT_REPO_ROOT; echo "emapmc rc=$rc"; [ $rc -eq 0 ] || exit $rc;;
    chunks) for C in ${CHUNKS:-1 2 4}; do run chunks_$C$BPC 300 env AMOD_CHUNKS=$C ${BPC:+AMOD_DEMOD_BPC=$BPC} python bench.py --config ${PMCCFG:-c2} --legs none --stream-chunks 0 --cpu-frames -1 --no-e2e --steps 50 --warmup 5 || exit 1; done;;
    listpc) run listpc 120 rocprofv3 -L;;
    ab) run ab 600 python tools/ab.py $(for v in ${VARIANTS}; do echo audio-modem_amd/lib/variants/$v/libamodem.so; done);;
  esac
done
