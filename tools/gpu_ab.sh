# GPU box: the -m gpu suite on the in-tree build, then an interleaved A/B of libamodem variants
# usage: bash tools/gpu_ab.sh TAG VARIANT...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
tag=$1; shift
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/$tag.tests.log 2>&1; rc=$?
tail -3 gpurun_out/$tag.tests.log; echo tests rc=$rc
[ $rc -eq 0 ] || exit $rc
libs=""; for v in "$@"; do libs="$libs audio-modem_amd/lib/variants/$v/libamodem.so"; done
timeout -k 10 300 python tools/ab.py $libs
