# Round-2 GPU check: full -m gpu suite (verbose, printed errors kept), smoke, a short bench and a
# kernel-trace profile.  Stops at the first failing step.  Usage: bash tools/gpu_r02.sh TAG [pytest -k expr]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r02}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "$K" > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest FAILED"; grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_$T.log | head -30; exit 1; }
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest FAILED"; grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_$T.log | head -30; exit 1; }
fi
grep -E "passed|failed" gpurun_out/pytest_$T.log | tail -2
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 300 python bench.py --steps 2000 --warmup 100 --no-cpu-baseline > gpurun_out/bench_$T.json
tail -1 gpurun_out/bench_$T.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$T -o kt --output-format csv -- python3 bench.py --steps 2000 --warmup 100 --no-cpu-baseline > gpurun_out/prof_$T.log 2>&1
find gpurun_out/prof_$T -name "*kernel_stats.csv" -exec head -5 {} \;
