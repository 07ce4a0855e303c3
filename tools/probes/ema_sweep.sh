cd $GRAFT_REPO_ROOT
for W in 4 2 1 8; do
  AMOD_EMA_WARM=$W timeout -k 10 200 python3 tools/stream_diag.py 32000 > gpurun_out/sd_w$W.log 2>&1 || { echo "w$W failed"; exit 1; }
  python3 -c "
import json;t=open('gpurun_out/sd_w$W.log').read();i=t.index('{');d=json.loads(t[i:]);r=d['device_resident'];print('warm $W', round(r['samples_per_s']/1e9,2), r['phases_ms'], r['file_ok'])"
done
