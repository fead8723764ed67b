#!/bin/bash
# VGPR count / spills of the kernels in one built object: bash profiles/kregs.sh <obj.o> [kernel-regex]
B=/opt/rocm/llvm/bin
T=$(mktemp -d)
objcopy -O binary --only-section=.hip_fatbin "$1" $T/fat.bin
$B/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
$B/llvm-readelf --notes $T/k.co | grep -E "\.name:|\.vgpr_count|\.vgpr_spill|\.sgpr_spill|agpr_count" | paste - - - - - \
  | sed -E 's/ +/ /g; s/\.agpr_count: [0-9]+//' | grep -E "${2:-.}"
rm -rf $T
