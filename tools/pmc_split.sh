# kernel trace + VALU/LDS/wait counters for one step variant: bash tools/pmc_split.sh TAG [epb,lid,kind]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_${1:-x}
mkdir -p $O
B="python3 bench.py --steps 40 --warmup 5 --clock-warmup 0 --api-steps 0 --no-cpu-baseline ${2:+--variant $2}"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- $B > $O/kt.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $O/p1 -o p1 --output-format csv -- $B > $O/p1.log 2>&1
timeout -k 10 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA -d $O/p2 -o p2 --output-format csv -- $B > $O/p2.log 2>&1
python3 - "$O" <<'PY'
import csv, collections, glob, sys
O = sys.argv[1]
for f in glob.glob(f"{O}/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:60]:60s} calls {r['Calls']:>6s} avg_ns {float(r['AverageNs']):10.0f}")
for f in sorted(glob.glob(f"{O}/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for row in csv.DictReader(open(f)):
        acc[row["Kernel_Name"][:40]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for kname, d in acc.items():
        for k, v in d.items():
            v = v[5:] or v
            print(f"{kname:40s} {k:24s} {sum(v)/len(v):16.0f}")
PY
