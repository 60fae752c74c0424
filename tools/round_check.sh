# Round-end check on the GPU box (the tree as committed): every -m gpu test, the smoke, the driver's
# bench command twice, the headline and usv-asmc-simple profiles (profiles/${TAG}_*), the reset rate
# and the API throughput; FULL=1 adds the f64, f64 usv-asmc-simple and 524 288-env profiles and the
# stamps-build wave timeline.  Stops at the first step that faults, aborts or times out.
#   gpurun -- 'TAG=r05c bash tools/round_check.sh'
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-rXX}
O=gpurun_out/check_$TAG
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stopping after rc $1"; exit $1;; esac; }
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 $O/pytest_gpu.log; stop $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc $rc"; tail -2 $O/smoke.log; stop $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.$i.json 2> $O/bench_driver.$i.err
  rc=$?; echo "bench $i rc $rc"; stop $rc
done
bash tools/profile_round.sh $TAG > $O/prof.log 2>&1
rc=$?; echo "prof rc $rc"; stop $rc
ENV_ID=usv-asmc-simple KERNELS="usv::(step_q_kernel|asmc_chain_kernel)" bash tools/profile_round.sh ${TAG}_asmc > $O/prof_asmc.log 2>&1
rc=$?; echo "prof asmc rc $rc"; stop $rc
timeout -k 10 300 python tools/done_rate.py > $O/done_rate.json 2>&1
rc=$?; echo "done rate rc $rc"; stop $rc
timeout -k 10 200 python tools/api_throughput.py --envs 4096 > $O/api_4096.json 2>&1
rc=$?; echo "api rc $rc"; stop $rc
[ -n "$FULL" ] || exit 0
PREC=f64 bash tools/profile_round.sh ${TAG}_f64 > $O/prof_f64.log 2>&1
rc=$?; echo "prof f64 rc $rc"; stop $rc
PREC=f64 ENV_ID=usv-asmc-simple KERNELS="usv::(dyn_kernel|scan_kernel)" bash tools/profile_round.sh ${TAG}_f64asmc > $O/prof_f64asmc.log 2>&1
rc=$?; echo "prof f64 asmc rc $rc"; stop $rc
ENVS=524288 KT_STEPS=400 bash tools/profile_round.sh ${TAG}_524k > $O/prof_524k.log 2>&1
rc=$?; echo "prof 524k rc $rc"; stop $rc
if [ -f diagbuild/stamps.so ]; then
  USV_LIB_PATH=diagbuild/stamps.so timeout -k 10 200 python tools/wave_timeline.py --envs 65536 --variant 128,7,5 > $O/timeline.json 2> $O/timeline.err
  rc=$?; echo "timeline rc $rc"; stop $rc
fi
