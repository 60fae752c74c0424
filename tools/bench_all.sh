# bench.py lines of every env id at 65536 envs (f32), no CPU leg: profiles/r02_bench_<id>.json
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ball
for id in usv-asmc-simple usv-asmc-v0 usv-pid-v0 usv-asmc-ye-int-v0; do
  timeout -k 10 300 python bench.py --env-id $id --steps 2000 --warmup 100 --no-cpu-baseline > gpurun_out/ball/$id.json
  tail -1 gpurun_out/ball/$id.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$id', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
