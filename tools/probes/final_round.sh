# The round's last profile set: C2 profile round (bench line with every leg and the graph
# object), C5 at 20 and 10 dB bench lines
cd $GRAFT_REPO_ROOT
bash tools/profile_round.sh gpurun_out/r03/c2 c2 || exit 1
timeout -k 10 300 python3 bench.py --config c5 --snr 20 --legs none --stream-chunks 0 --no-e2e --cpu-frames -1 > gpurun_out/r03/c5_20db.json 2> gpurun_out/r03/c5_20db.err || exit 1
timeout -k 10 300 python3 bench.py --config c5 --snr 10 --legs none --stream-chunks 0 --no-e2e --cpu-frames -1 > gpurun_out/r03/c5_10db.json 2> gpurun_out/r03/c5_10db.err || exit 1
python3 - <<'PY'
import json
for f in ("c2/bench.json", "c5_20db.json", "c5_10db.json"):
    d = json.loads(open("gpurun_out/r03/" + f).read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("graph"))
PY
