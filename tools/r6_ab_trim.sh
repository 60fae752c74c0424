# Round 6: the trimmed pair-row DMA (USV_DMA_TRIM, ab/trim.so) against the product library:
# bit-identity (parity subsets), step time at 65 536 / 524 288 envs, FETCH_SIZE at 524 288.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6b}; mkdir -p $O
L=${LIB:-ab/trim.so}
USV_LIB_PATH=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_r5.py tests/test_gpu_parity.py tests/test_gpu_r2.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/lib_pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 $O/lib_pytest.log; [ $rc = 0 ] || exit $rc
O=$O/ab LIBS="gym-usv_amd/gym_usv_amd/libusvhip.so $L" ROUNDS=3 bash tools/ab_libs.sh || exit $?
O=$O/ab ENVS=524288 STEPS=400 LIBS="gym-usv_amd/gym_usv_amd/libusvhip.so $L" ROUNDS=2 bash tools/ab_libs.sh || exit $?
for lib in gym-usv_amd/gym_usv_amd/libusvhip.so $L; do
  b=$(basename $lib .so)
  USV_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$b -o fetch --output-format csv -- python3 bench.py --envs 524288 --no-cpu-baseline --api-steps 0 --f64-steps 0 --clock-warmup 0 --steady-steps 0 --steps 40 --warmup 10 > $O/fetch_$b.log 2>&1 || exit $?
  USV_LIB_PATH=$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write_$b -o write --output-format csv -- python3 bench.py --envs 524288 --no-cpu-baseline --api-steps 0 --f64-steps 0 --clock-warmup 0 --steady-steps 0 --steps 40 --warmup 10 > $O/write_$b.log 2>&1 || exit $?
done
python3 - $O <<'PY'
import csv, glob, sys, statistics
O = sys.argv[1]
for f in sorted(glob.glob(f"{O}/*/**/*counter_collection.csv", recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if "step_q_kernel" in r.get("Kernel_Name", "")]
    vals = [float(r["Counter_Value"]) for r in rows]
    if vals:
        print(f.split("/")[-4] if "/" in f else f, rows[0]["Counter_Name"], "median KiB per launch", statistics.median(vals), "n", len(vals))
PY
