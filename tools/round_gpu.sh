# GPU parity suite, then the round profile (bench JSON, kernel stats, FETCH/WRITE passes).
# Stops at the first failing step.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${1:-r01}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$R.log 2>&1 || { echo "pytest FAILED"; grep -E "^(FAILED|ERROR)|Error" gpurun_out/pytest_gpu_$R.log | head -20; exit 1; }
tail -2 gpurun_out/pytest_gpu_$R.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
bash tools/profile_round.sh $R
