set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/kt -o kt --output-format csv -- python bench.py --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/prof/kt.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d gpurun_out/prof/pmc1 -o pmc1 --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof/pmc1.log 2>&1
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/pmc2 -o pmc2 --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof/pmc2.log 2>&1
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof/pmc3 -o pmc3 --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/prof/pmc3.log 2>&1
ls -R gpurun_out/prof | head -40
