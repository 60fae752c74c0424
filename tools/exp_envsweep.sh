#!/bin/bash
# Per-kernel rocprof averages of one library over env counts.   ARGS="--env-id usv-asmc-simple" bash tools/exp_envsweep.sh 32768 65536 131072
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/envsweep
for n in "$@"; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/envsweep/n$n -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --api-steps 0 --steps 300 --warmup 20 --clock-warmup 0.2 --envs $n $ARGS > gpurun_out/envsweep/n$n.log 2>&1
  echo "== $n envs"
  find gpurun_out/envsweep/n$n -name "*kernel_stats.csv" -exec python3 -c "
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'usv::' in r['Name'] and int(r['Calls']) > 10: print('   ', r['Name'].split('(')[0][:60], r['Calls'], round(float(r['AverageNs'])/1000, 2), 'us')
" {} \;
done
