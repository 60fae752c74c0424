# Per-kernel average durations (rocprofv3 kernel trace) of a bench run for each library given.
#   ARGS="--env-id usv-asmc-simple" bash tools/exp_kernel_times.sh lib1.so lib2.so ...
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ktimes
for lib in "$@"; do
  t=$(basename $lib .so)
  USV_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/ktimes/$t -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --api-steps 0 --steps 300 --warmup 20 --clock-warmup 0.2 $ARGS > gpurun_out/ktimes/$t.log 2>&1
  echo "== $t"
  find gpurun_out/ktimes/$t -name "*kernel_stats.csv" -exec python3 -c "
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'usv::' in r['Name'] and int(r['Calls']) > 10: print('   ', r['Name'].split('(')[0][:60], r['Calls'], round(float(r['AverageNs'])/1000, 2), 'us')
" {} \;
done
