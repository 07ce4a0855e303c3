# Experiments only: kernel times and SQ counters of the streaming receiver's kernels on the
# 32k-chunk stream (tools/ema_probe.py: three device-resident receives)
cd /tmp && export TMPDIR=/tmp
o=$GRAFT_REPO_ROOT/gpurun_out/emaprof
mkdir -p $o
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ema_probe.py 32000 > $o/kt.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --kernel-trace -d $o/sq -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ema_probe.py 32000 > $o/sq.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $o/fetch -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ema_probe.py 32000 > $o/fetch.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob, collections
o = "gpurun_out/emaprof"
import os; os.chdir(os.environ.get("GRAFT_REPO_ROOT", "."))
for r in csv.DictReader(open(glob.glob(o + "/kt/**/run_kernel_stats.csv", recursive=True)[0])):
    print("%-40s %5s calls  avg %9.1f us" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(o + "/sq/**/run_counter_collection.csv", recursive=True) + glob.glob(o + "/fetch/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][-30:]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "ema" in k or "k_sc" in k or "k_fine" in k or "gap" in k:
        print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
