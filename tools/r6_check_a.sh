cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -5 $O/pytest.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
tail -c 600 $O/bench.json
O=$O/ab LIBS="ab/base.so gym-usv_amd/gym_usv_amd/libusvhip.so" ROUNDS=2 bash tools/ab_libs.sh
