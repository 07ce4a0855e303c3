#!/bin/bash
# Experiments only: libamodem.so variants of the fast kernel: <wpe>x<sb>[t0|t1]
# (waves-per-EU, stream batch, twiddles in LDS)
# under audio-modem_amd/lib/variants/<name>/ (git-ignored; travels with gpurun).
set -e
cd "$(dirname "$0")/../audio-modem_amd/csrc"
HIPCC=/opt/rocm/bin/hipcc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../../include -I."
for v in "$@"; do
  wpe=${v%%x*}; rest=${v#*x}; sb=${rest%%t*}; tw=1; case $rest in *t0) tw=0;; esac
  out=../lib/variants/w${wpe}s${sb}t${tw}; mkdir -p $out
  $HIPCC $FLAGS -DAMOD_WPE=$wpe -DAMOD_SB=$sb -DAMOD_TW_LDS=$tw -c k_decode_fast.hip -o $out/k_decode_fast.o
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o $out/libamodem.so $out/k_decode_fast.o ../lib/k_decode_exact.o ../lib/runtime.o -Wl,-soname,libamodem.so
  echo built $out
done
