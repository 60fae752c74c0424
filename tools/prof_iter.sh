# per-wave cycle breakdown for a few variants (diagnostic build)
set -e
cd $GRAFT_REPO_ROOT
hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -Iinclude -DUSV_DIAG_PROF -o /tmp/libprof.so gym-usv_amd/csrc/usv_kernels.hip
for v in ${VARIANTS:-64,7,1 32,7,1 16,7,2}; do
  USV_LIB_PATH=/tmp/libprof.so timeout -k 10 120 python tools/prof_waves.py --variant $v 2>/dev/null
done
