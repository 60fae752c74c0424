#!/bin/bash
# WRITE_SIZE / FETCH_SIZE per step-kernel launch and event-timed step of library builds, at ENVS envs
# (default 524288, beyond the Infinity Cache).   ENVS=65536 bash tools/exp_write_ab.sh a.so b.so
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ENVS=${ENVS:-524288}
O=gpurun_out/writeab_$ENVS
mkdir -p $O
B="python3 bench.py --envs $ENVS --no-cpu-baseline --api-steps 0 --clock-warmup 0 $ARGS"
for lib in "$@"; do
  t=$(basename $lib .so)
  USV_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/$t/write -o write --output-format csv -- $B --steps 40 --warmup 10 > $O/$t.write.log 2>&1
  USV_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/$t/fetch -o fetch --output-format csv -- $B --steps 40 --warmup 10 > $O/$t.fetch.log 2>&1
  python3 - $O/$t <<'PY'
import csv, glob, sys, re
d = sys.argv[1]
for c in ("write", "fetch"):
    v = [float(r["Counter_Value"]) for f in glob.glob(f"{d}/{c}/**/*counter_collection.csv", recursive=True)
         for r in csv.DictReader(open(f)) if re.search(r"usv::step\w*_kernel", r["Kernel_Name"])]
    v = v[5:] or v
    print(d, c, "KiB/launch", round(sum(v) / max(1, len(v)), 1), "samples", len(v))
PY
done
for round in 1 2; do
  for lib in "$@"; do
    t=$(basename $lib .so)
    USV_LIB_PATH=$lib timeout -k 10 120 python3 bench.py --envs $ENVS --no-cpu-baseline --api-steps 0 --steps 1000 --warmup 50 $ARGS > $O/$t.$round.json
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'round', sys.argv[3], 'step_us', round(d['roofline']['kernel_ms']*1e3, 2), 'wall_us', round(d['ms_per_step']*1e3, 2), 'frac', d['roofline']['frac'])" $O/$t.$round.json $t $round
  done
done
