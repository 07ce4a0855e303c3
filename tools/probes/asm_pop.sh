# Experiments only: the streaming receiver with and without the assembler arena's
# background population (32k-chunk stream, device-resident host phases)
cd $GRAFT_REPO_ROOT
for V in 0 1; do
  if [ $V = 1 ]; then export AMOD_ASM_NO_POPULATE=1; fi
  timeout -k 10 200 python3 tools/stream_diag.py 32000 > gpurun_out/ap_$V.log 2>&1 || { echo "v$V failed"; exit 1; }
  grep "\[stream\]" gpurun_out/ap_$V.log | grep -v "thread [0-9]" | tail -5
  python3 -c "
import json;t=open('gpurun_out/ap_$V.log').read();i=t.index('{');d=json.loads(t[i:]);r=d['device_resident'];print('no_populate=$V', round(r['samples_per_s']/1e9,2), r['phases_ms'], r['file_ok'])"
done
