set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo smoke rc=$?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -30 gpurun_out/gpu_tests.log; echo tests rc=$rc
if [ $rc -le 1 ]; then timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; echo bench rc=$?; cat gpurun_out/bench.json; fi
