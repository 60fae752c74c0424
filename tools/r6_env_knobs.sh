# Round 6: runtime environment knobs vs the driver's short bench command (wall ms_per_step, event kernel time).
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r6i}; mkdir -p $O
run() {  # name, env assignments...
  n=$1; shift
  for r in 1 2; do
    env "$@" timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --api-steps 0 --f64-steps 0 > $O/$n.$r.json 2> $O/$n.$r.err || return $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roofline']['kernel_ms'], round(d['value']/1e9,3))" $O/$n.$r.json $n
  done
}
run default X=1 || exit $?
run devkernarg1 HIP_FORCE_DEV_KERNARG=1 || exit $?
run devkernarg0 HIP_FORCE_DEV_KERNARG=0 || exit $?
run nointr HSA_ENABLE_INTERRUPT=0 || exit $?
run default_b X=1 || exit $?
