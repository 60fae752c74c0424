set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
tag=${1:-x}
timeout -k 10 300 python tools/sweep_variants.py --variants "${VARIANTS:-32,3 16,7 32,7 64,7}" > gpurun_out/sweep_$tag.log 2>&1
grep variant gpurun_out/sweep_$tag.log
for n in 16384 262144 1048576; do
  timeout -k 10 120 python tools/sweep_variants.py --envs $n --steps 200 --variants '32,7' 2>/dev/null | grep variant
done
timeout -k 10 600 python -m pytest tests -m gpu -q -s -p no:cacheprovider > gpurun_out/pytest_gpu_$tag.log 2>&1 || { echo "pytest FAILED"; grep -E "^(FAILED|ERROR)|Error" gpurun_out/pytest_gpu_$tag.log | head -20; exit 1; }
tail -2 gpurun_out/pytest_gpu_$tag.log
