#!/bin/bash
# Static instruction mix of one kernel in a hipcc object (gfx950): whole-kernel counts of the
# classes that matter for k_demod's job loop (VALU moves, lane reads/writes, s_nop, ...).
# usage: tools/isa_stats.sh <object.o> [kernel-symbol-regex]   (default: QPSK k_demod, NS 4)
set -e
obj=$1; pat=${2:-_ZN4amod12_GLOBAL__N_17k_demodILi1ELi4EEEvNS_6DevCfgENS_7DevWorkE}
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
B=/opt/rocm/lib/llvm/bin
$B/llvm-objcopy --dump-section=.hip_fatbin="$tmp/fat.bin" "$obj"
$B/clang-offload-bundler --unbundle --type=o --input="$tmp/fat.bin" --output="$tmp/co.elf" \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950
$B/llvm-objdump -d --no-show-raw-insn "$tmp/co.elf" > "$tmp/all.s"
awk -v pat="<$pat>:" 'index($0, pat) {on=1; next} /^[0-9a-f]+ <.*>:$/ {on=0} on && NF {print $1}' "$tmp/all.s" > "$tmp/k.txt"
printf "%-8s total %5d  v_mov %4d  v_readlane %3d  v_writelane %3d  v_cndmask %4d  s_nop %4d  s_and_b64 %4d  valu %5d  salu %5d\n" \
  "$(basename $(dirname $obj))" "$(wc -l < $tmp/k.txt)" "$(grep -c '^v_mov' $tmp/k.txt)" "$(grep -c '^v_readlane' $tmp/k.txt)" \
  "$(grep -c '^v_writelane' $tmp/k.txt)" "$(grep -c '^v_cndmask' $tmp/k.txt)" "$(grep -c '^s_nop' $tmp/k.txt)" \
  "$(grep -c '^s_and_b64' $tmp/k.txt)" "$(grep -c '^v_' $tmp/k.txt)" "$(grep -Ec '^s_(add|sub|mul|and|or|xor|andn2|orn2|cselect|mov|cmp|lshl|lshr|ashr|bcnt|min|max|not|bfe|ff1)' $tmp/k.txt)"
