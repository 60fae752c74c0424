# Round 6: f64 constant divisions (div_const): GPU tests, then the f64 kernels against the round-5 library.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6c}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc $rc"; tail -3 $O/pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
O=$O/ab PREC=f64 ENV_ID=usv-asmc-simple STEPS=1000 LIBS="ab/base.so gym-usv_amd/gym_usv_amd/libusvhip.so" ROUNDS=2 bash tools/ab_libs.sh || exit $?
O=$O/ab PREC=f64 STEPS=1000 LIBS="ab/base.so gym-usv_amd/gym_usv_amd/libusvhip.so" ROUNDS=2 bash tools/ab_libs.sh || exit $?
