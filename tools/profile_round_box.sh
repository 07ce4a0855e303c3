#!/bin/bash
# GPU box: tools/profile_round.sh for each workload, summarised there (profile_summary.py),
# keeping only the summaries under gpurun_out/<tag>/ (the raw traces exceed what gpurun
# brings back).  usage: bash tools/profile_round_box.sh r06 c2 c4 ...
set -o pipefail
tag=$1; shift
root="$GRAFT_REPO_ROOT"
for c in "$@"; do
  raw=/tmp/prof_$tag/$c
  extra=""; [ "$c" = c5 ] && extra="--snr 10" # (the default run's C5 leg)
  bash "$root/tools/profile_round.sh" "$raw" "$c" $extra || exit $?
  python3 "$root/tools/profile_summary.py" "$raw" "$root/gpurun_out/$tag/$c" || exit $?
  for f in bench.err ktrace.err; do [ -f "$raw/$f" ] && cp "$raw/$f" "$root/gpurun_out/$tag/$c/"; done
  echo "profiled $c"
done
