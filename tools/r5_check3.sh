# Round-5 final check on the GPU box (the tree as committed): every -m gpu test, the smoke, the
# driver's bench command twice, and the headline profile again (profiles/r05b_*).  Stops at the
# first step that faults, aborts or times out.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5z
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
bash tools/profile_round.sh r05b > $O/prof_r05b.log 2>&1
rc=$?; echo "prof rc $rc"; stop $rc
ENV_ID=usv-asmc-simple KERNELS="usv::(step_q_kernel|asmc_chain_kernel)" bash tools/profile_round.sh r05b_asmc > $O/prof_r05b_asmc.log 2>&1
rc=$?; echo "prof asmc rc $rc"; stop $rc
timeout -k 10 300 python tools/done_rate.py > $O/done_rate.json 2>&1
rc=$?; echo "done rate rc $rc"; stop $rc
timeout -k 10 200 python tools/api_throughput.py --envs 4096 > $O/api_4096.json 2>&1
rc=$?; echo "api rc $rc"; stop $rc
