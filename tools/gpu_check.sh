# GPU check used while iterating: the GPU test suite (fail-fast), then the C5 10 dB and
# C2 bench lines (kernel breakdown), each under its own time limit
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${TESTS:-} > gpurun_out/t_gpu.log 2>&1
rc=$?; echo "tests rc $rc"; tail -3 gpurun_out/t_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python bench.py --config c5 --snr 10 --no-e2e --cpu-frames -1 > gpurun_out/c5_10.json 2>gpurun_out/c5_10.err && python3 -c "
import json; d=json.loads(open('gpurun_out/c5_10.json').read().strip().splitlines()[-1]); print('c5_10 %.3e'%d['value'], d['ms_per_step'], d['frames_ok'], d['frames_exact_fallback'], d['chain']['kernels_ms_avg'])" &&
timeout -k 10 120 python bench.py --cpu-frames -1 --no-e2e --stream-chunks 0 > gpurun_out/c2.json 2>/dev/null && python3 -c "
import json; d=json.loads(open('gpurun_out/c2.json').read().strip().splitlines()[-1]); print('c2 %.3e'%d['value'], d['ms_per_step'], d['frames_ok'], d['chain']['kernels_ms_avg'])"
