#!/bin/bash
# usage: tools/kernel_resources.sh <object.o> [kernel-name-regex]
# VGPR / SGPR / scratch / LDS of every gfx950 kernel in a hipcc object (code-object notes).
set -e
obj=$1; pat=${2:-.}
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
B=/opt/rocm/lib/llvm/bin
$B/llvm-objcopy --dump-section=.hip_fatbin="$tmp/fat.bin" "$obj"
$B/clang-offload-bundler --unbundle --type=o --input="$tmp/fat.bin" --output="$tmp/co.elf" \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950
$B/llvm-readelf --notes "$tmp/co.elf" | python3 -c '
import re, sys
txt = sys.stdin.read()
pat = re.compile(sys.argv[1])
for blk in txt.split("  - .agpr_count")[1:]:
    g = lambda k: (re.search(r"\.%s:\s+(\S+)" % k, blk) or [None, "?"])[1]
    name = g("name")
    if not pat.search(name):
        continue
    print("%-60s vgpr %4s agpr %3s sgpr %3s scratch %5s lds %6s" % (name[:60], g("vgpr_count"),
          (re.match(r"\s*:\s*(\d+)", blk) or [None, "?"])[1], g("sgpr_count"), g("private_segment_fixed_size"),
          g("group_segment_fixed_size")))
' "$pat"
