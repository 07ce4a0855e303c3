#!/bin/bash
# C2 chain time under the two-stream chunked overlap (AMOD_CHUNKS) and k_demod grid
# sizes (AMOD_DEMOD_BPC). usage (GPU box): bash tools/overlap_scan.sh
q="--steps 20 --warmup 3 --cpu-frames -1 --no-e2e --stream-chunks 0"
for c in 1 2 4 8; do
  for b in 0 1 2 3; do
    if [ $b -gt 0 ]; then export AMOD_DEMOD_BPC=$b; else unset AMOD_DEMOD_BPC; fi
    r=$(AMOD_CHUNKS=$c timeout -k 10 60 python3 bench.py $q 2>/dev/null) || exit 1
    echo "chunks=$c bpc=$b $(echo "$r" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("%.3e ms %.4f" % (d["value"], d["ms_per_step"]), d["chain"]["kernels_ms_avg"])')"
  done
done
