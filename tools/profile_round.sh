#!/bin/bash
# A round's judged profile set for one workload (GPU box): the bench line, rocprofv3 kernel
# stats and per-dispatch trace of the same command, FETCH_SIZE and WRITE_SIZE passes (one
# TCC counter group each) and two SQ passes; for c2 the full default bench line (every
# leg) and the stream leg's kernel stats as well.
# usage: bash tools/profile_round.sh gpurun_out/r03/c2 c2 [extra bench args]
#        (then python tools/profile_summary.py gpurun_out/r03/c2 profiles/r03/c2)
set -o pipefail
out=$(realpath -m "${1:-gpurun_out/r03/c2}")
conf=${2:-c2}
shift 2 2>/dev/null
extra="$*"
mkdir -p "$out"
root="$GRAFT_REPO_ROOT"
B="$root/bench.py"
one="--config $conf --legs none --cpu-frames -1 --no-e2e --stream-chunks 0 $extra"
cd /tmp && export TMPDIR=/tmp
if [ "$conf" = c2 ]; then
  timeout -k 10 420 python3 "$B" > "$out/bench.json" 2> "$out/bench.err" || exit $?
else
  timeout -k 10 240 python3 "$B" $one --steps 20 --warmup 5 > "$out/bench.json" 2> "$out/bench.err" || exit $?
fi
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$out/ktrace" -o run --output-format csv -- python3 "$B" $one --steps 20 --warmup 3 > "$out/bench_under_rocprof.json" 2> "$out/ktrace.err" &&
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$out/fetch" -o run --output-format csv -- python3 "$B" $one --steps 5 --warmup 1 > /dev/null 2> "$out/fetch.err" &&
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$out/write" -o run --output-format csv -- python3 "$B" $one --steps 5 --warmup 1 > /dev/null 2> "$out/write.err" &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
  --kernel-trace -d "$out/sq" -o run --output-format csv -- python3 "$B" $one --steps 5 --warmup 1 > /dev/null 2> "$out/sq.err" &&
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_SCA \
  --kernel-trace -d "$out/sq2" -o run --output-format csv -- python3 "$B" $one --steps 5 --warmup 1 > /dev/null 2> "$out/sq2.err" || exit $?
if [ "$conf" = c2 ]; then
  # the streaming receiver's kernels (the bench's stream leg alone: C4-shaped 32k-chunk stream)
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/ktrace_stream" -o run --output-format csv -- python3 "$B" --legs none --steps 2 --warmup 1 --cpu-frames -1 --no-e2e > "$out/bench_stream_under_rocprof.json" 2> "$out/ktrace_stream.err"
fi
