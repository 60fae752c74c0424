# Round 6 A/B of library builds: bit-identity of $TESTLIB (parity subsets), then LIBS interleaved at
# 65 536 envs (ROUNDS) and 524 288 envs (ROUNDS_DRAM).
#   TAG=r6d TESTLIB=ab/x.so LIBS="ab/prod.so ab/x.so" bash tools/r6_ab.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r6x}; mkdir -p $O
if [ -n "$TESTLIB" ]; then
  for L in $TESTLIB; do
    USV_LIB_PATH=$L timeout -k 10 600 python -u -m pytest tests/test_gpu_r5.py tests/test_gpu_parity.py tests/test_gpu_r2.py ${TESTS:-} -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_$(basename $L .so).log 2>&1
    rc=$?; echo "pytest $L rc $rc"; tail -2 $O/pytest_$(basename $L .so).log; [ $rc = 0 ] || exit $rc
  done
fi
O=$O/ab ROUNDS=${ROUNDS:-3} bash tools/ab_libs.sh || exit $?
[ "${ROUNDS_DRAM:-1}" = 0 ] || O=$O/ab ENVS=524288 STEPS=400 ROUNDS=${ROUNDS_DRAM:-1} bash tools/ab_libs.sh || exit $?
