#!/bin/bash
# Register / scratch usage of the kernels in a built object (the code object's metadata):
#   tools/kernel_regs.sh auction-gym_amd/build/ag_sim_p2.o [name-regex]
set -e
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$B/llvm-objcopy --dump-section .hip_fatbin=$T/fat.bin "$1"
TGT=$($B/clang-offload-bundler --list --type=o --input=$T/fat.bin | grep gfx950 | head -1)
$B/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin --targets="$TGT" --output=$T/dev.co
$B/llvm-readelf --notes $T/dev.co | grep -E "^ +\.name:|\.vgpr_count:|\.sgpr_count:|\.private_segment_fixed_size:|vgpr_spill_count|sgpr_spill_count" \
  | paste - - - - - - | sed -E 's/ +/ /g' | grep -E "${2:-.}" || true
rm -rf $T
