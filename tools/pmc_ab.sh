#!/bin/bash
# Experiments only: per-variant SQ counters over tools/ab.py (one library per pass).
# usage (GPU box): VARIANTS="a b" bash tools/pmc_ab.sh ; summaries under gpurun_out/pmcab_<v>/
cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-base}; do
  AB_ROUNDS=2 timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/pmcab_$v -o run --output-format csv -- python tools/ab.py audio-modem_amd/lib/variants/$v/libamodem.so > gpurun_out/pmcab_$v.log 2>&1 || exit 1
done
echo ok
