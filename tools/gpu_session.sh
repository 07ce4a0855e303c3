set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 150 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_stream_sharded.py -m gpu > gpurun_out/ts.log 2>&1; rc=$?; tail -2 gpurun_out/ts.log; [ $rc -le 1 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 170 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/sprof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/tools/stream_diag.py" 32000 > "$GRAFT_REPO_ROOT/gpurun_out/sprof.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
python3 - <<'PY'
import csv,re,collections
d=collections.defaultdict(list)
for r in csv.DictReader(open('gpurun_out/sprof/run_kernel_trace.csv')):
    m=re.search(r'(k_\w+)',r['Kernel_Name'])
    if m: d[m.group(1)].append((int(r['Start_Timestamp']),(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3))
for k in ('k_gap_scan','k_fine','k_sc_blocks','k_ema_out','k_window'):
    print(k, [round(x[1],1) for x in sorted(d[k])][-4:])
PY
