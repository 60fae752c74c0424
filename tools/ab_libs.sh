#!/bin/bash
# Same-box A/B of library builds (product and diagbuild/*.so from other commits or defines):
# usv-simple at 65 536 envs for each, ROUNDS times interleaved, then optional extra lines.
#   O=gpurun_out/x LIBS="a.so b.so" ROUNDS=2 bash tools/ab_libs.sh
# Prints "<lib> <envs> <env_id> <kernel us> <frac>" per run (bench.py's event time of the step kernels).
cd "${GRAFT_REPO_ROOT:-.}"
O=${O:-gpurun_out/ab}
ROUNDS=${ROUNDS:-2}
ENVS=${ENVS:-65536}
ENV_ID=${ENV_ID:-usv-simple}
VARIANT=${VARIANT:-}
PREC=${PREC:-f32}
mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for L in $LIBS; do
    b=$(basename $L .so)
    f=$O/b_${b}_${ENV_ID}_${PREC}_${ENVS}${VARIANT:+_$VARIANT}.$r.json
    USV_LIB_PATH=$L timeout -k 10 180 python bench.py --envs $ENVS --env-id $ENV_ID --precision $PREC --no-cpu-baseline --api-steps 0 \
      --f64-steps 0 --steady-steps 0 \
      --steps ${STEPS:-2000} --warmup 100 ${VARIANT:+--variant $VARIANT} > $f 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], sys.argv[3], sys.argv[4], sys.argv[6], sys.argv[5], round(r['kernel_ms']*1e3, 2), round(r['frac'], 4))" $f $b $ENVS $ENV_ID "${VARIANT:-default}" $PREC
  done
done
