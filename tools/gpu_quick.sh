# Quick GPU check after a kernel change: the parity tests that exercise the step kernels, then the
# default step timing (sweep) and the bench line.  Usage: bash tools/gpu_quick.sh TAG
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-q}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "variants or lidar or golden or ragged or c3 or single_step or sharding" > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest FAILED"; grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_$T.log | head -30; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_$T.log | tail -1
timeout -k 10 120 python tools/sweep_variants.py --variants "128,7,5" --steps 2000 2>/dev/null | grep variant
