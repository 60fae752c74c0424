# Round profile: bench JSON, rocprofv3 kernel-trace stats, FETCH_SIZE and WRITE_SIZE passes
# (separate runs, no tracing domains combined with --pmc), summary into profiles/.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${1:-r01}
ENVS=${ENVS:-65536}
OUT=gpurun_out/prof_$R
mkdir -p $OUT profiles
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --envs $ENVS --steps 2000 --warmup 100 --no-cpu-baseline > $OUT/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 bench.py --envs $ENVS --steps 40 --warmup 10 --no-cpu-baseline > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 bench.py --envs $ENVS --steps 40 --warmup 10 --no-cpu-baseline > $OUT/write.log 2>&1
python3 tools/pmc_summary.py --kt $OUT/kt --fetch $OUT/fetch --write $OUT/write --key usv-simple/$ENVS/f32/window --round $R --out $OUT/profiles
# bench last: it reads roofline.traffic from the PMC summary just written
timeout -k 10 300 python bench.py --pmc $OUT/profiles/pmc_summary.json > $OUT/bench.json 2> $OUT/bench.err
tail -1 $OUT/bench.json
cp $OUT/kt/kt/*kernel_stats.csv $OUT/profiles/${R}_kernel_stats.csv 2>/dev/null || find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/profiles/${R}_kernel_stats.csv \;
