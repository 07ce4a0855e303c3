set -o pipefail
cd "$GRAFT_REPO_ROOT"
AB_ROUNDS=16 AB_CONFS=${CONFS:-c2,c4,c5} timeout -k 10 170 python -u tools/aux_ab.py d: bal:AMOD_DEMOD_BALANCE=1 > gpurun_out/bal.log 2>&1 || exit $?
grep "^c" gpurun_out/bal.log
