#!/bin/bash
# Experiments only: libamodem.so variants of the exact kernel, each NAME=FLAGS (extra hipcc
# flags for k_decode_exact.hip, e.g. q8=-DAMOD_SC_CQ=8), under audio-modem_amd/lib/variants/
# <name>/ (git-ignored; travels with gpurun). The other objects come from the in-tree build.
set -e
cd "$(dirname "$0")/../audio-modem_amd/csrc"
HIPCC=/opt/rocm/bin/hipcc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -I. -ffp-contract=off"
OBJS="../lib/k_decode_fast.o ../lib/k_tx.o ../lib/k_stream.o ../lib/stream.o ../lib/runtime.o ../lib/assembler.o ../lib/group.o ../lib/pipe.o"
for v in "$@"; do
  name=${v%%=*}; extra=${v#*=}
  out=../lib/variants/$name; mkdir -p $out
  $HIPCC $FLAGS $extra -c k_decode_exact.hip -o $out/k_decode_exact.o
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $out/libamodem.so $out/k_decode_exact.o $OBJS -Wl,-soname,libamodem.so -lpthread
  echo built $out
done
