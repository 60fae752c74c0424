set -e
cd $GRAFT_REPO_ROOT
H="hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -Iinclude"
$H -DUSV_DIAG_NOLIDAR -o /tmp/libusv_nolidar.so gym-usv_amd/csrc/usv_kernels.hip &
$H -DUSV_DIAG_NODYN -o /tmp/libusv_nodyn.so gym-usv_amd/csrc/usv_kernels.hip &
$H -DUSV_DIAG_NOLIDAR -DUSV_DIAG_NODYN -o /tmp/libusv_none.so gym-usv_amd/csrc/usv_kernels.hip &
wait
for lib in gym-usv_amd/gym_usv_amd/libusvhip.so /tmp/libusv_nolidar.so /tmp/libusv_nodyn.so /tmp/libusv_none.so; do
  for n in 16384 65536 262144; do
    echo "$lib $n $(USV_LIB_PATH=$lib timeout -k 10 120 python tools/sweep_variants.py --envs $n --steps 200 --variants '32,7' 2>/dev/null | grep variant)"
  done
done
