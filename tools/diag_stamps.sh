set -e
cd $GRAFT_REPO_ROOT
hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -Iinclude -DUSV_DIAG_STAMPS -o /tmp/libdiag.so gym-usv_amd/csrc/usv_kernels.hip
for v in 32,7 16,7; do
USV_LIB_PATH=/tmp/libdiag.so timeout -k 10 120 python tools/stamps.py --variant $v 2>/dev/null
done
