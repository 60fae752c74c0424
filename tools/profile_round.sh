# Round profile of the headline step kernel at ENVS envs (default 65536; 524288 defeats the 256 MB
# Infinity Cache): rocprofv3 kernel-trace stats, FETCH_SIZE / WRITE_SIZE passes, three SQ counter
# passes (one rocprofv3 --pmc run each, no tracing domains combined), the summary (traffic and
# VALU / SALU instruction counts per launch) into $OUT/profiles, then the bench line that reads it.
#   bash tools/profile_round.sh TAG        (on the GPU box, via gpurun)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
R=${1:-r03}
ENVS=${ENVS:-65536}
ENV_ID=${ENV_ID:-usv-simple}
PREC=${PREC:-f32}
KERNELS=${KERNELS:-}        # regex of every kernel of a step (usv-asmc-simple: "usv::(step_q_kernel|asmc_chain_kernel)")
OUT=gpurun_out/prof_$R
mkdir -p $OUT
KT_STEPS=${KT_STEPS:-2000}
B="python3 bench.py --envs $ENVS --env-id $ENV_ID --precision $PREC --no-cpu-baseline --api-steps 0 --f64-steps 0"
P="$B --clock-warmup 0 --steady-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- $B --steps $KT_STEPS --warmup 100 > $OUT/kt.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- $P --steps 40 --warmup 10 > $OUT/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- $P --steps 40 --warmup 10 > $OUT/write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT/sq/p1 -o p1 --output-format csv -- $P --steps 30 --warmup 5 > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY -d $OUT/sq/p2 -o p2 --output-format csv -- $P --steps 30 --warmup 5 > $OUT/p2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_LDS_UNALIGNED_STALL SQ_IFETCH -d $OUT/sq/p3 -o p3 --output-format csv -- $P --steps 30 --warmup 5 > $OUT/p3.log 2>&1
python3 tools/pmc_all.py $OUT/sq --envs $ENVS > $OUT/sq_counters.txt
python3 tools/pmc_all.py $OUT --envs $ENVS > $OUT/all_counters.txt
cat $OUT/sq_counters.txt
cp profiles/pmc_summary.json $OUT/pmc_summary_prev.json 2>/dev/null || true
mkdir -p $OUT/profiles
cp profiles/pmc_summary.json $OUT/profiles/pmc_summary.json 2>/dev/null || true
python3 tools/pmc_summary.py --kt $OUT/kt --fetch $OUT/fetch --write $OUT/write --sq $OUT/sq --envs $ENVS \
  --key $ENV_ID/$ENVS/$PREC/window --round $R --out $OUT/profiles ${KERNELS:+--kernels "$KERNELS"}
find $OUT/kt -name "*kernel_stats.csv" -exec cp {} $OUT/profiles/${R}_kernel_stats.csv \;
# bench last, with the default CPU leg at 65 536 envs: it reads roofline.traffic / valu_frac from the summary
timeout -k 10 300 python bench.py --envs $ENVS --env-id $ENV_ID --precision $PREC --pmc $OUT/profiles/pmc_summary.json $([ "$ENVS" != 65536 ] && echo --no-cpu-baseline) > $OUT/bench.json 2> $OUT/bench.err
tail -1 $OUT/bench.json
