# Experiments only: k_ema_out output chunks per lane x warm-up chunks, 32k-chunk stream
cd $GRAFT_REPO_ROOT
for PW in 4:4 8:4 4:2 8:2; do
  P=${PW%%:*}; W=${PW##*:}
  AMOD_EMA_PER=$P AMOD_EMA_WARM=$W timeout -k 10 200 python3 tools/ema_probe.py 32000 > gpurun_out/ep_${P}_${W}.log 2>&1 || { echo "p$P w$W failed"; exit 1; }
  python3 -c "
import json
runs=[json.loads(l) for l in open('gpurun_out/ep_${P}_${W}.log') if l.startswith('{\"seconds')]
print('per $P warm $W', [(round(r['t_ema_ms'],2), r['fixed'], r['file_ok'], round(r['seconds']*1e3,1)) for r in runs])"
done
