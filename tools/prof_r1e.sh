set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_e
for n in 16384 65536 262144 1048576; do
  timeout -k 10 120 python tools/sweep_variants.py --envs $n --steps 200 --variants "32,7 16,7 64,7" 2>/dev/null | grep variant
done
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/prof_e/p1 -o p1 --output-format csv -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/prof_e/p1.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY -d gpurun_out/prof_e/p2 -o p2 --output-format csv -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/prof_e/p2.log 2>&1
echo done
