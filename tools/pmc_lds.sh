#!/bin/bash
# Experiments only: LDS / issue counters of one variant over tools/ab.py.
cd "$GRAFT_REPO_ROOT"
v=${VARIANT:-pk}
AB_ROUNDS=2 timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmclds_$v -o run --output-format csv -- python tools/ab.py audio-modem_amd/lib/variants/$v/libamodem.so > gpurun_out/pmclds_$v.log 2>&1 || exit 1
AB_ROUNDS=2 timeout -s KILL 180 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_LEVEL_VMEM --kernel-trace -d gpurun_out/pmcwait_$v -o run --output-format csv -- python tools/ab.py audio-modem_amd/lib/variants/$v/libamodem.so > gpurun_out/pmcwait_$v.log 2>&1 || exit 1
echo ok
