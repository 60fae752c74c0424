set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_${1:-x}
mkdir -p $O
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/p1 -o p1 --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/p1.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY -d $O/p2 -o p2 --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/p2.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_LDS_UNALIGNED_STALL SQ_IFETCH -d $O/p3 -o p3 --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/p3.log 2>&1 || true
python3 - <<'PY'
import csv, collections, glob, sys
for f in sorted(glob.glob("gpurun_out/pmc_*/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        if "step_kernel" in row["Kernel_Name"] or "step_q_kernel" in row["Kernel_Name"]:
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, v in acc.items():
        v = v[5:] or v
        print(f"{k:26s} {sum(v)/len(v):16.0f}")
PY
