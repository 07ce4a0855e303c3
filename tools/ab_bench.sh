#!/bin/bash
# Experiments only: interleaved A/B of libamodem variants (audio-modem_amd/lib/variants/<v>)
# on one bench config; prints ms per step, the chain's kernel times and the roofline.
#   tools/ab_bench.sh OUTDIR "BENCH ARGS" v1 v2 ... (each run twice, interleaved)
O=$1; ARGS=$2; shift 2
mkdir -p $O
for r in 1 2; do
  for v in "$@"; do
    AMODEM_LIB=audio-modem_amd/lib/variants/$v/libamodem.so timeout -k 10 150 python bench.py $ARGS \
      > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v failed"; tail -5 $O/${v}_$r.err; exit 1; }
    python - "$O/${v}_$r.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "ms/step %.4f" % d["ms_per_step"], "value %.4g" % d["value"], "chain", d.get("chain"),
      "roof %.4f" % d["roofline"]["frac"], d["roofline"].get("kernel"), "%.4f" % d["roofline"]["kernel_ms_avg"])
PY
  done
done
