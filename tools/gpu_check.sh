# GPU box: the -m gpu suite, then (if green) a short C2 bench; usage: bash tools/gpu_check.sh [TAG]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=${1:-chk}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$tag.tests.log 2>&1; rc=$?
tail -15 gpurun_out/$tag.tests.log; echo tests rc=$rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-frames -1 --no-e2e --stream-chunks 0 > gpurun_out/$tag.bench.json 2> gpurun_out/$tag.bench.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/$tag.bench.json'));print('value',d['value'],'ms',d['ms_per_step'],'chain',d['chain']['ms_avg'],d['chain']['kernels_ms_avg'],'ok',d['frames_ok'],'fb',d['frames_exact_fallback'])"
