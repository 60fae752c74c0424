set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 150 python tools/sweep_variants.py --env-id usv-asmc-simple --variants "16,7,2 128,7,4 128,7,5 64,7,4 64,7,5 256,7,4" --steps 1000 2>/dev/null | grep variant
for id in usv-pid-v0 usv-asmc-ye-int-v0; do
  timeout -k 10 200 python bench.py --env-id $id --cpu-seconds 5 > gpurun_out/bench_$id.json 2> gpurun_out/bench_$id.err
  tail -1 gpurun_out/bench_$id.json
done
