#!/bin/bash
# Event-timed step (bench.py roofline.kernel_ms: every kernel of a step plus the gaps) for each
# library given, interleaved over two rounds.   ARGS="--env-id usv-asmc-simple" bash tools/exp_step_ab.sh a.so b.so
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/stepab
for round in 1 2; do
  for lib in "$@"; do
    t=$(basename $lib .so)
    USV_LIB_PATH=$lib timeout -k 10 120 python3 bench.py --no-cpu-baseline --api-steps 0 --steps 3000 --warmup 50 $ARGS > gpurun_out/stepab/$t.$round.json
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'round', sys.argv[3], 'step_us', round(d['roofline']['kernel_ms']*1e3, 2), 'wall_us', round(d['ms_per_step']*1e3, 2))" gpurun_out/stepab/$t.$round.json $t $round
  done
done
