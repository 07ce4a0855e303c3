cd $GRAFT_REPO_ROOT
for v in base fine8; do
  AMODEM_LIB=audio-modem_amd/lib/variants/$v/libamodem.so timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD --kernel-trace -d gpurun_out/pmcv_$v -o run --output-format csv -- python tools/stage_profile.py > gpurun_out/pmcv_$v.log 2>&1 || exit 1
done
