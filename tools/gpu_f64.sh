# f64 path check: variant bit-identity (window vs brute), golden replays, lidar scenes, single steps;
# then the f64 bench line at 65536 envs (window and brute).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "f64 or variants or lidar_scenes or safe_vmcnt" > gpurun_out/pytest_f64.log 2>&1 || { echo "pytest FAILED"; grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/pytest_f64.log | head -30; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_f64.log | tail -1
for lid in window brute; do
  timeout -k 10 300 python bench.py --precision f64 --lidar $lid --steps 1000 --warmup 50 --no-cpu-baseline > gpurun_out/bench_f64_$lid.json
  tail -1 gpurun_out/bench_f64_$lid.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lid', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
