# Round-2 GPU check: full -m gpu suite, smoke, public-API throughput at 4096 envs, bench line.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r02b}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$T.log 2>&1 || { echo "pytest FAILED"; grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_$T.log | head -30; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_$T.log | tail -1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 300 python tools/api_throughput.py --envs 4096 --steps 2000 > gpurun_out/api_$T.json
cat gpurun_out/api_$T.json
timeout -k 10 300 python bench.py --steps 5000 --warmup 200 --no-cpu-baseline > gpurun_out/bench_$T.json
tail -1 gpurun_out/bench_$T.json
