set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
AB_CONFS=c5 AB_ROUNDS=12 timeout -k 10 500 python -u tools/aux_ab.py 'all:' 'p1:AMOD_YIELD_PER=1' 'p2:AMOD_YIELD_PER=2' 'p4:AMOD_YIELD_PER=4' > gpurun_out/yield_ab.log 2>&1; rc=$?; grep -v Warn gpurun_out/yield_ab.log | tail -12; exit $rc
