# Interleaved A/B step timing of library builds (sweep_variants: events around back-to-back launches,
# boundaries included).  Usage: bash tools/exp_ab.sh lib1.so lib2.so ...   (R rounds, default 3)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in $(seq ${R:-3}); do
  for lib in "$@"; do
    echo -n "$lib: "
    USV_LIB_PATH=$lib timeout -k 10 120 python tools/sweep_variants.py --envs ${ENVS:-65536} --variants "${VAR:-128,7,5}" --steps ${STEPS:-3000} 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1000, 2), 'us')"
  done
done
