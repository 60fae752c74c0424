#!/bin/bash
# Register / scratch / LDS use of every kernel in the built library (code-object notes).
# Usage: tools/kernel_resources.sh [pattern]      (no GPU needed)
set -e
LIB=${USV_LIB_PATH:-$(dirname "$0")/../gym-usv_amd/gym_usv_amd/libusvhip.so}
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$LIB"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
  --input=$T/fat.bin --output=$T/k.co
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $T/k.co |
  grep -E "^\s+\.name:|private_segment_fixed_size|\.vgpr_count|\.sgpr_count|group_segment_fixed_size" |
  paste - - - - - | sed 's/\s\+/ /g; s/\.group_segment_fixed_size/lds/; s/\.private_segment_fixed_size/scratch/' |
  grep -E "${1:-.}" || true
rm -rf $T
