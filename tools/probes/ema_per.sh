cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_stream_ema.py tests/test_gpu_stream.py tests/test_gpu_stream_sharded.py 2>&1 | tail -2
for P in 1 2 4; do
  AMOD_EMA_PER=$P timeout -k 10 200 python3 tools/stream_diag.py 32000 > gpurun_out/sd_p$P.log 2>&1 || { echo "p$P failed"; exit 1; }
  python3 -c "
import json;t=open('gpurun_out/sd_p$P.log').read();i=t.index('{');d=json.loads(t[i:]);r=d['device_resident'];print('per $P', round(r['samples_per_s']/1e9,2), r['phases_ms'], r['file_ok'])"
done
