# chain time of the C2 bench for two-stream chunk counts (AMOD_CHUNKS) x demod grid (AMOD_DEMOD_BPC)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/chunks
for cb in ${CB:-1:0 4:1 4:2 8:1 8:2 16:1}; do
  c=${cb%%:*}; b=${cb#*:}
  if [ "$b" = 0 ]; then unset AMOD_DEMOD_BPC; else export AMOD_DEMOD_BPC=$b; fi
  AMOD_CHUNKS=$c timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-frames -1 --no-e2e --stream-chunks 0 > gpurun_out/chunks/c${c}_b$b.json 2> gpurun_out/chunks/c${c}_b$b.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/chunks/c${c}_b$b.json'));print('chunks $c bpc $b', d['ms_per_step'], d['chain']['ms_avg'], d['chain']['kernels_ms_avg'], d['frames_ok'])"
done
