#!/bin/bash
# Print VGPR / SGPR / spill / LDS / scratch usage of the gfx950 kernels in a HIP object or shared library.
# Usage: tools/kernel_resources.sh <file.o|file.so> [kernel-regex]
set -eo pipefail
F=$1; RE=${2:-.}
L=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$L/llvm-objcopy --dump-section=.hip_fatbin=$T/fb.bin "$F" "$T/dummy" 2>/dev/null || $L/llvm-objcopy -O binary --only-section=.hip_fatbin "$F" $T/fb.bin
$L/clang-offload-bundler --unbundle --type=o --input=$T/fb.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
$L/llvm-readelf --notes $T/k.co | grep -E "^ +\.name:|\.vgpr_count|\.sgpr_count|private_segment_fixed_size|group_segment_fixed_size|vgpr_spill_count" \
  | awk '{printf "%s ", $0} /\.vgpr_spill_count/ {print ""}' | sed 's/  */ /g; s/\.group_segment_fixed_size/lds/; s/\.private_segment_fixed_size/scratch/' | grep -E "$RE"
rm -rf $T
