# Diagnostic builds of the step library (never the product): ablations and per-wave stamps.
#   bash tools/build_diag.sh NOLIDAR NOSTORE NODYN STAMPS ...   -> diag/abl_<X>.so / diag/stamps.so
set -e
cd "$(dirname "$0")/.."
mkdir -p diag
for x in "$@"; do
  if [ "$x" = STAMPS ]; then def=-DUSV_DIAG_STAMPS; out=diag/stamps.so; else def=-DUSV_ABL_$x; out=diag/abl_$x.so; fi
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -mllvm -amdgpu-atomic-optimizer-strategy=None -Iinclude $def -o $out gym-usv_amd/csrc/usv_kernels.hip &
done
wait
ls -la diag
