set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider -k "asmc and not v0" > gpurun_out/asmc_tests.log 2>&1 || { echo "pytest FAILED"; grep -E "^(FAILED|ERROR)|Error|assert|golden|round" gpurun_out/asmc_tests.log | tail -30; exit 1; }
grep -E "golden|round|PASS" gpurun_out/asmc_tests.log | tail -30
timeout -k 10 150 python tools/sweep_variants.py --env-id usv-asmc-simple --variants "128,7,4 16,7,2" --steps 1000 2>/dev/null | grep variant
