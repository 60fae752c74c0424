# Kernel trace + two SQ counter passes of one step variant at 65 536 envs (no tracing domains with --pmc).
#   PREC=f64 ENV_ID=usv-asmc-simple bash tools/pmc_variant.sh TAG [epb,lid,kind]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_${1:-x}
mkdir -p $O
B="python3 bench.py --precision ${PREC:-f32} --env-id ${ENV_ID:-usv-simple} --steps 40 --warmup 5 --clock-warmup 0 --api-steps 0 --no-cpu-baseline ${2:+--variant $2}"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- $B > $O/kt.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/sq/p1 -o p1 --output-format csv -- $B > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY -d $O/sq/p2 -o p2 --output-format csv -- $B > $O/p2.log 2>&1
find $O/kt -name "*kernel_stats.csv" -exec cat {} \;
python3 tools/pmc_all.py $O/sq --envs 65536
