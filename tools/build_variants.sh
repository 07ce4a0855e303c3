#!/bin/bash
# Experiments only: libamodem.so variants of the fast kernel, each NAME=FLAGS
# (extra hipcc flags for k_decode_fast.hip, e.g. base= or w6=-DAMOD_WPE=6),
# under audio-modem_amd/lib/variants/<name>/ (git-ignored; travels with gpurun).
# The other objects come from the current in-tree build (make -C audio-modem_amd/csrc).
set -e
cd "$(dirname "$0")/../audio-modem_amd/csrc"
HIPCC=/opt/rocm/bin/hipcc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -I."
OBJS="../lib/k_decode_exact.o ../lib/k_tx.o ../lib/k_stream.o ../lib/stream.o ../lib/runtime.o ../lib/assembler.o ../lib/group.o ../lib/pipe.o"
for v in "$@"; do
  name=${v%%=*}; extra=${v#*=}
  out=../lib/variants/$name; mkdir -p $out
  src=k_decode_fast.hip
  [ -n "$SRC_DIR" ] && src=$SRC_DIR/k_decode_fast.hip
  $HIPCC $FLAGS $extra -c $src -o $out/k_decode_fast.o
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $out/libamodem.so $out/k_decode_fast.o $OBJS -Wl,-soname,libamodem.so -lpthread
  echo built $out
done
