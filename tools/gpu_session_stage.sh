set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=$(realpath -m gpurun_out/s32); mkdir -p $O
timeout -k 10 300 python3 tools/stage_cost.py > $O/stage.log 2>&1 || { tail -5 $O/stage.log; exit 1; }
cat $O/stage.log | grep stop
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVES --kernel-trace -d $O/pmc -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/stage_cost.py > /dev/null 2> $O/pmc.err || exit $?
python3 - <<PY
import csv, collections
rows = [r for r in csv.DictReader(open("$O/pmc/run_counter_collection.csv")) if ("k_detect" in r["Kernel_Name"] or "k_corr_scan" in r["Kernel_Name"])]
by = collections.OrderedDict()
for r in rows:
    by.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
ids = list(by)
stops = ["0", "10", "11", "12", "1", "2", "none"]
per = len(ids) // len(stops)
for k, s in enumerate(stops):
    grp = [by[i] for i in ids[k * per:(k + 1) * per]][3:]
    avg = {c: sum(g.get(c, 0) for g in grp) / max(1, len(grp)) for c in grp[0]}
    print("stop", s, {c: round(v / 1e6, 2) for c, v in sorted(avg.items())})
PY
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/stream_diag.py 32000 > $O/sd.json 2> $O/sd.err || { tail -5 $O/sd.err; exit 1; }
grep -h "decode_dispatch of 32000\|launches:\|sparse copy" $O/sd.err
