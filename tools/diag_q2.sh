# Block-queue step diagnostics: ablation timings (diag/abl_*.so, results invalid by design), the
# per-wave stamp timeline (diag/stamps.so), SQ counters and FETCH/WRITE of the product kernel.
# Build first: bash tools/build_diag.sh NOLIDAR NOSTORE NODYN STAMPS; the diag/ directory must not be
# in .gpurunignore for the run.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-q2}
O=gpurun_out/diag_$T
mkdir -p $O
for f in full NOLIDAR NOSTORE NODYN; do
  lib=gym-usv_amd/gym_usv_amd/libusvhip.so; [ $f != full ] && lib=diag/abl_$f.so
  echo -n "$f: "
  USV_LIB_PATH=$lib timeout -k 10 120 python tools/sweep_variants.py --variants "128,7,5" --steps 500 2>/dev/null | grep variant | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1000, 'us')"
done
USV_LIB_PATH=diag/stamps.so timeout -k 10 120 python tools/wave_timeline.py --variant 128,7,5 > $O/timeline.json 2> $O/timeline.err
cat $O/timeline.json
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c -d $O/$c -o $c --output-format csv -- python3 bench.py --steps 40 --warmup 10 --no-cpu-baseline > $O/$c.log 2>&1
done
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/p1 -o p1 --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/p1.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY -d $O/p2 -o p2 --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/p2.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_LDS_UNALIGNED_STALL SQ_IFETCH -d $O/p3 -o p3 --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/p3.log 2>&1
python3 tools/pmc_all.py $O
