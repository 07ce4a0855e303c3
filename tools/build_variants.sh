#!/bin/bash
# Experiments only: libamodem.so variants of the fast kernel (waves-per-EU x stream batch)
# under audio-modem_amd/lib/variants/<name>/ (git-ignored; travels with gpurun).
set -e
cd "$(dirname "$0")/../audio-modem_amd/csrc"
HIPCC=/opt/rocm/bin/hipcc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -I."
for v in "$@"; do
  wpe=${v%x*}; sb=${v#*x}
  out=../lib/variants/w${wpe}s${sb}; mkdir -p $out
  $HIPCC $FLAGS -DAMOD_WPE=$wpe -DAMOD_SB=$sb -c k_decode_fast.hip -o $out/k_decode_fast.o
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $out/libamodem.so $out/k_decode_fast.o ../lib/k_decode_exact.o ../lib/runtime.o -Wl,-soname,libamodem.so
  echo built $out
done
