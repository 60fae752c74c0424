set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_full.log 2>&1 || { echo "pytest FAILED"; grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_gpu_full.log | head -20; exit 1; }
tail -2 gpurun_out/pytest_gpu_full.log
timeout -k 10 200 python bench.py --env-id usv-asmc-simple > gpurun_out/bench_asmc_simple.json 2> gpurun_out/bench_asmc_simple.err
tail -1 gpurun_out/bench_asmc_simple.json
