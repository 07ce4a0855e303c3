set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
AB_CONFS=c2,c5,c4 AB_ROUNDS=10 timeout -k 10 500 python -u tools/aux_ab.py 'split:' 'nosplit:AMOD_DEMOD_NOSPLIT=1' > gpurun_out/split_ab.log 2>&1; rc=$?; grep -v Warn gpurun_out/split_ab.log | tail -12; exit $rc
