# Round-5 check on the GPU box: every -m gpu test, the smoke, the driver's bench command, and the
# round profiles of the headline (usv-simple f32, C3) and usv-asmc-simple.  Stops at the first step
# that faults, aborts or times out (a plain test failure does not stop the profiles).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5j
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stopping after rc $1"; exit $1;; esac; }
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 $O/pytest_gpu.log; stop $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc $rc"; tail -2 $O/smoke.log; stop $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
rc=$?; echo "bench rc $rc"; stop $rc
bash tools/profile_round.sh r05 > $O/prof_r05.log 2>&1
rc=$?; echo "prof rc $rc"; stop $rc
ENV_ID=usv-asmc-simple KERNELS="usv::(step_q_kernel|asmc_chain_kernel)" bash tools/profile_round.sh r05_asmc > $O/prof_r05_asmc.log 2>&1
rc=$?; echo "prof asmc rc $rc"; stop $rc
