#!/bin/bash
# One bench line per (env id, precision, env count) given as id:prec:envs; summary to stdout.
#   bash tools/bench_matrix.sh usv-asmc-v0:f32:65536 usv-simple:f64:65536
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/matrix
for c in "$@"; do
  IFS=: read id prec n <<< "$c"
  out=gpurun_out/matrix/$id.$prec.$n.json
  timeout -k 10 150 python3 bench.py --no-cpu-baseline --api-steps 0 --steps ${STEPS:-2000} --warmup 100 --env-id $id --precision $prec --envs $n > $out
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], 'value %.4g' % d['value'], 'step_us', round(r['kernel_ms']*1e3, 2), 'wall_us', round(d['ms_per_step']*1e3, 2), 'frac', r['frac'])" $out $c
done
