#!/bin/bash
# Disassemble the gfx950 code object of a built library (no GPU needed).
#   bash tools/disasm.sh [lib.so] > out.s
set -e
LIB=${1:-$(dirname "$0")/../gym-usv_amd/gym_usv_amd/libusvhip.so}
T=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$LIB"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 \
  --input=$T/fat.bin --output=$T/k.co
/opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn $T/k.co
rm -rf $T
