#!/bin/bash
# Experiments only: k_demod knockout builds (AMOD_KO, k_decode_fast.hip) under
# audio-modem_amd/lib/variants/ko_*; time them with
#   AB_CHECK=0 python tools/ab_demod.py audio-modem_amd/lib/variants/ko_*/libamodem.so
set -e
cd "$(dirname "$0")"
for v in ${KO_LIST:-ko_base=0x100 ko_crc=0x101 ko_demap=0x102 ko_pilot=0x104 ko_chk=0x108 ko_fft=0x110 ko_demaplds=0x140 ko_fftlds=0x180}; do
  bash build_variants.sh "${v%%=*}=-DAMOD_KO=${v#*=}" > /dev/null &
done
wait
ls ../audio-modem_amd/lib/variants/
