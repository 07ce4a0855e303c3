#!/bin/bash
# Experiments only (GPU box): k_demod's instruction counts per knockout build (VALU, SALU,
# LDS, SMEM per launch), to apportion the per-job work by phase. Build the variants first on
# the CPU (tools/ko_variants.sh); each library runs alone under one rocprofv3 --pmc pass.
# usage: AB_CONFS=c4 bash tools/ko_insts.sh gpurun_out/koi product ko_base ko_end ...
set -o pipefail
out=$(realpath -m "${1:-gpurun_out/koi}")
shift
root="$GRAFT_REPO_ROOT"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  lib="$root/audio-modem_amd/lib/variants/$v/libamodem.so"
  [ "$v" = product ] && lib="$root/audio-modem_amd/lib/libamodem.so"
  AB_CONFS=${AB_CONFS:-c4} AB_ROUNDS=2 AB_CHECK=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES \
    SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
    --kernel-trace -d "$out/$v" -o run --output-format csv -- python3 "$root/tools/ab_demod.py" "$lib" \
    > "$out/$v.log" 2>&1 || exit $?
done
python3 - "$out" "$@" <<'PYEOF'
import collections, csv, os, sys
out = sys.argv[1]
for v in sys.argv[2:]:
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(out, v, "run_counter_collection.csv"))):
        if "k_demod" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {c: max(x) for c, x in agg.items()}  # the main launch (the replay launch is empty)
    t = [l for l in open(os.path.join(out, v + ".log")) if " demod " in l]
    print(f"{v:12s} VALU {m.get('SQ_INSTS_VALU', 0):12.0f} SALU {m.get('SQ_INSTS_SALU', 0):12.0f} "
          f"LDS {m.get('SQ_INSTS_LDS', 0):11.0f} SMEM {m.get('SQ_INSTS_SMEM', 0):10.0f} "
          f"waitinst/wave {m.get('SQ_WAIT_INST_ANY', 0) / max(1, m.get('SQ_WAVE_CYCLES', 1)):.3f} "
          f"activeVALU/wave {m.get('SQ_ACTIVE_INST_VALU', 0) / max(1, m.get('SQ_WAVE_CYCLES', 1)):.3f} | "
          + (t[-1].strip() if t else ""))
PYEOF
