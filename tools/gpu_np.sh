set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -v -s --timeout 200 --timeout-method thread -p no:cacheprovider -k "np_reset or v0 or legacy" > gpurun_out/np_tests.log 2>&1 || { echo "pytest FAILED"; grep -E "^(FAILED|ERROR)|Error|assert|np-reset|Mismatch|Max abs|x:|y:" gpurun_out/np_tests.log | head -40; exit 1; }
grep -E "np-reset|PASS" gpurun_out/np_tests.log | tail -20
