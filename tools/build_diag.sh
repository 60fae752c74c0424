# Diagnostic builds of the step library (never the product): clock stamps / section counters.
#   bash tools/build_diag.sh STAMPS QPROF PROF   -> diagbuild/stamps.so, diagbuild/qprof.so, diagbuild/prof.so (travels with gpurun)
# Each defines USV_DIAG (csrc/usv_diag.hpp is included only then) plus USV_DIAG_<X>.
set -e
cd "$(dirname "$0")/.."
mkdir -p diagbuild
for x in "$@"; do
  lc=$(echo $x | tr A-Z a-z)
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -mllvm -amdgpu-atomic-optimizer-strategy=None \
    -Iinclude -DUSV_DIAG -DUSV_DIAG_$x -o diagbuild/$lc.so gym-usv_amd/csrc/usv_kernels.hip &
done
wait
ls -la diagbuild
