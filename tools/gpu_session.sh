set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash run_gpu.sh tests || exit $?
grep -q " failed" gpurun_out/gpu_tests.log && { grep -E "FAILED|Error" gpurun_out/gpu_tests.log | head -20; exit 1; }
AB_CONFS=c2,c4,c5 timeout -k 10 150 python -u tools/ab_demod.py audio-modem_amd/lib/variants/base/libamodem.so audio-modem_amd/lib/variants/rot/libamodem.so > gpurun_out/rot_ab.log 2>&1 || exit $?
grep "^c" gpurun_out/rot_ab.log
AB_CONFS=c4 bash tools/ko_counters.sh gpurun_out/rotko base rot || exit $?
