set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in own ctx hi; do
  AMOD_PIPE_STREAMS=$v AB_CONFS=c2,c5,c3 AB_ROUNDS=6 timeout -k 10 300 python -u tools/pipeline_ab.py > gpurun_out/pab_$v.log 2>&1 || exit $?
  echo "== $v"; grep -v Warn gpurun_out/pab_$v.log | grep ms/step
done
