#!/bin/bash
# A/B build of the product source with extra defines (never the product): diagbuild/NAME.so
#   bash tools/build_variant.sh NAME -DUSV_ROW_STORE=0 ...
set -e
cd "$(dirname "$0")/.."
mkdir -p diagbuild
n=$1; shift
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -mllvm -amdgpu-atomic-optimizer-strategy=None \
  -Iinclude "$@" -o diagbuild/$n.so gym-usv_amd/csrc/usv_kernels.hip
