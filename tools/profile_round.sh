#!/bin/bash
# The round's judged profile set (GPU box): the C2 bench line, rocprofv3 kernel stats
# and per-dispatch trace of the same command, FETCH_SIZE and WRITE_SIZE passes (one
# TCC counter group each), an SQ pass, and the C5 lines at 10 and 20 dB.
# usage: bash tools/profile_round.sh gpurun_out/r02   (then tools/profile_summary.py)
set -o pipefail
out=$(realpath -m "${1:-gpurun_out/r02}")
mkdir -p "$out"
root="$GRAFT_REPO_ROOT"
B="$root/bench.py"
quick="--steps 20 --warmup 3 --cpu-frames -1 --no-e2e --stream-chunks 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 python3 "$B" > "$out/bench.json" 2> "$out/bench.err" &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$out/ktrace" -o run --output-format csv -- python3 "$B" $quick > "$out/bench_under_rocprof.json" 2> "$out/ktrace.err" &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$out/fetch" -o run --output-format csv -- python3 "$B" --steps 5 --warmup 1 --cpu-frames -1 --no-e2e --stream-chunks 0 > /dev/null 2> "$out/fetch.err" &&
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$out/write" -o run --output-format csv -- python3 "$B" --steps 5 --warmup 1 --cpu-frames -1 --no-e2e --stream-chunks 0 > /dev/null 2> "$out/write.err" &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
  --kernel-trace -d "$out/sq" -o run --output-format csv -- python3 "$B" --steps 5 --warmup 1 --cpu-frames -1 --no-e2e --stream-chunks 0 > /dev/null 2> "$out/sq.err" &&
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_SCA \
  --kernel-trace -d "$out/sq2" -o run --output-format csv -- python3 "$B" --steps 5 --warmup 1 --cpu-frames -1 --no-e2e --stream-chunks 0 > /dev/null 2> "$out/sq2.err" &&
timeout -k 10 240 python3 "$B" --config c5 --snr 20 --no-e2e > "$out/bench_c5_20db.json" 2> "$out/c5_20.err" &&
timeout -k 10 240 python3 "$B" --config c5 --snr 10 --soft --no-e2e > "$out/bench_c5_10db.json" 2> "$out/c5_10.err" &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$out/ktrace_c5" -o run --output-format csv -- python3 "$B" --config c5 --snr 10 $quick > /dev/null 2> "$out/ktrace_c5.err"
# the streaming receiver's kernels (the bench's stream leg: C4-shaped 2000-chunk stream)
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$out/ktrace_stream" -o run --output-format csv -- python3 "$B" --steps 2 --warmup 1 --cpu-frames -1 --no-e2e > "$out/bench_stream_under_rocprof.json" 2> "$out/ktrace_stream.err"
