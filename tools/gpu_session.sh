set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
AB_CONFS=c2,c4,c5 timeout -k 10 600 python -u tools/ab_demod.py audio-modem_amd/lib/variants/vmin/libamodem.so audio-modem_amd/lib/variants/live/libamodem.so > gpurun_out/live_ab.log 2>&1; rc=$?; grep -v Warn gpurun_out/live_ab.log | tail -8; exit $rc
