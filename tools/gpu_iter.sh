# one GPU iteration: parity suite, variant sweep, phase stamps, workload stats
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-x}
timeout -k 10 600 python -m pytest tests -m gpu -q -s -p no:cacheprovider > gpurun_out/pytest_gpu_$tag.log 2>&1 || { echo "pytest FAILED"; grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu_$tag.log | head -30; exit 1; }
tail -1 gpurun_out/pytest_gpu_$tag.log
timeout -k 10 300 python tools/sweep_variants.py --variants "${VARIANTS:-16,7 32,7 16,7,1 32,7,1 64,7,1}" 2>/dev/null | grep variant | cut -c1-140
if [ -n "$STAMPS" ]; then
hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -Iinclude -DUSV_DIAG_STAMPS -o /tmp/libdiag.so gym-usv_amd/csrc/usv_kernels.hip
USV_LIB_PATH=/tmp/libdiag.so timeout -k 10 120 python tools/stamps.py --variant $STAMPS 2>/dev/null | python -c "import json,sys; d=json.load(sys.stdin); print({k:(v['mean'] if isinstance(v,dict) else v) for k,v in d.items()})"
fi
if [ -n "$PRIO" ]; then
hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -Iinclude -DUSV_WAVE_PRIO -o /tmp/libprio.so gym-usv_amd/csrc/usv_kernels.hip
echo "with s_setprio ramp:"
USV_LIB_PATH=/tmp/libprio.so timeout -k 10 300 python tools/sweep_variants.py --variants "$PRIO" 2>/dev/null | grep variant | cut -c1-140
fi
