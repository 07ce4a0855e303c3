set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_pipe.py -m gpu > gpurun_out/pipe_tests.log 2>&1; rc=$?; tail -4 gpurun_out/pipe_tests.log; [ $rc -eq 0 ] || exit $rc
AB_CONFS=c2,c5 AB_ROUNDS=8 timeout -k 10 300 python -u tools/pipeline_ab.py > gpurun_out/pab.log 2>&1; rc=$?; grep -v Warn gpurun_out/pab.log | tail -5; exit $rc
