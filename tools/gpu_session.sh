set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash run_gpu.sh tests || exit $?
grep -q " failed" gpurun_out/gpu_tests.log && { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; exit 1; }
timeout -k 10 170 python tools/node_c4.py 3 > gpurun_out/nodec4.log 2>&1 || exit $?
grep -E "^run" gpurun_out/nodec4.log
