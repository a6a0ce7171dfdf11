#!/bin/bash
# Register / LDS / scratch use of the gfx950 kernels in a built library (no GPU needed):
#   tools/kernel_regs.sh [lib] [name-regex]
LIB=${1:-nart_amd/lib/libnart_hip.so}; PAT=${2:-k_render}
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section .hip_fatbin=$T/fb.bin "$LIB" || exit 1
/opt/rocm/lib/llvm/bin/clang-offload-bundler --type=o --input=$T/fb.bin --unbundle \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co || exit 1
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/k.co | python3 -c '
import sys, re
txt = sys.stdin.read()
pat = re.compile(sys.argv[1])
for blk in txt.split("  - .agpr_count")[1:]:
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    name = g("name")
    if pat.search(name):
        print("%-70s vgpr %s agpr %s spill v %s s %s lds %s scratch %s" % (name[:70], g("vgpr_count"), blk.split()[0],
              g("vgpr_spill_count"), g("sgpr_spill_count"), g("group_segment_fixed_size"), g("private_segment_fixed_size")))
' "$PAT"
rm -rf $T
