#!/bin/bash
# Round-end check on the GPU box: every -m gpu test, the smoke, the driver's bench command, and a
# kernel-trace profile of usv-asmc-simple (the secondary config) -> gpurun_out/final_$1/
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/final_${1:-r03}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/asmc_kt -o kt --output-format csv -- python3 bench.py --env-id usv-asmc-simple --no-cpu-baseline --api-steps 0 --steps 2000 --warmup 100 > $O/bench_asmc.json 2> $O/bench_asmc.err
tail -1 $O/pytest_gpu.log; tail -1 $O/smoke.log; tail -1 $O/bench.json | cut -c1-300
