set -o pipefail
cd "$GRAFT_REPO_ROOT"
for c in ${CONFS:-c2 c4}; do
  extra=""; [ "$c" = c5 ] && extra="--snr 10"
  echo "== profile $c"; bash tools/profile_round.sh gpurun_out/r04/$c $c $extra || exit $?
  ls gpurun_out/r04/$c
done
