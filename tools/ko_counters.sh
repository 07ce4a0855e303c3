#!/bin/bash
# Experiments only (GPU box): k_demod's LDS counters per knockout build, to see which phase
# its bank conflicts come from. Build the variants first on the CPU (tools/ko_variants.sh);
# each library runs alone under one rocprofv3 --pmc pass (tools/ab_demod.py, C4, no check).
# usage: bash tools/ko_counters.sh gpurun_out/ko [lib dirs under audio-modem_amd/lib/variants]
set -o pipefail
out=$(realpath -m "${1:-gpurun_out/ko}")
shift
root="$GRAFT_REPO_ROOT"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  lib="$root/audio-modem_amd/lib/variants/$v/libamodem.so"
  [ "$v" = product ] && lib="$root/audio-modem_amd/lib/libamodem.so"
  AB_CONFS=${AB_CONFS:-c4} AB_ROUNDS=2 AB_CHECK=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES \
    SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
    --kernel-trace -d "$out/$v" -o run --output-format csv -- python3 "$root/tools/ab_demod.py" "$lib" \
    > "$out/$v.log" 2>&1 || exit $?
done
python3 - "$out" "$@" <<'EOF'
import collections, csv, os, sys
out = sys.argv[1]
for v in sys.argv[2:]:
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(out, v, "run_counter_collection.csv"))):
        if "k_demod" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {c: max(x) for c, x in agg.items()}  # the main launch (the replay launch is empty)
    lds = m.get("SQ_ACTIVE_INST_LDS", 0) or 1
    print(f"{v:12s} LDS insts {m.get('SQ_INSTS_LDS', 0):12.0f}  active {lds:12.0f}  conflicts "
          f"{m.get('SQ_LDS_BANK_CONFLICT', 0):12.0f} ({m.get('SQ_LDS_BANK_CONFLICT', 0) / lds:.3f})  "
          f"WAIT_ANY/WAVE_CYCLES {m.get('SQ_WAIT_ANY', 0) / max(1, m.get('SQ_WAVE_CYCLES', 1)):.3f}")
EOF
