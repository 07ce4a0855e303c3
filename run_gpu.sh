# usage: bash run_gpu.sh <steps...>  (each step bounded; stop at first crash)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -4 gpurun_out/$name.log; echo "rc=$rc"; if [ $rc -ge 2 ] && [ $rc -ne 5 ]; then echo "ABORT after $name"; exit $rc; fi; }
for s in "$@"; do
  case $s in
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()";;
    tests) run gpu_tests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider;;
    bench) run bench 900 python bench.py --steps 20 --warmup 3;;
    benchc3) run bench_c3 600 python bench.py --config c3 --steps 10 --warmup 2;;
    benchc4) run bench_c4 600 python bench.py --config c4 --steps 10 --warmup 2 --stream-chunks 0;;
    bench2g) run bench2g 600 env AMOD_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 5 --warmup 2 --cpu-frames -1 --stream-chunks 0 --no-e2e --legs c4,c5;;
    bench2fail) echo "== bench2fail"; timeout -k 10 300 python bench.py --gpus 2 > gpurun_out/bench2fail.log 2>&1; echo "rc=$? (2 expected)"; tail -2 gpurun_out/bench2fail.log;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --cpu-frames -1;;
    demodprof) export AMODEM_LIB=audio-modem_amd/lib/variants/stamps/libamodem.so; run demod_c2 300 python tools/demod_profile.py c2 && run demod_c4 300 python tools/demod_profile.py c4 && run demod_c5 300 python tools/demod_profile.py c5;;
    streamdiag) run stream_diag 300 python tools/stream_diag.py ${NCHUNKS:-32000};;
    ab) run ab 600 python tools/ab_demod.py $(for v in ${VARIANTS}; do echo audio-modem_amd/lib/variants/$v/libamodem.so; done);;
  esac
done
