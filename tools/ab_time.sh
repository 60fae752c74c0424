# A/B step timing of diagnostic builds diagbuild/abl_<X>.so, interleaved R rounds (default 3), 2000 launches
# each.  Usage: bash tools/ab_time.sh X Y ...   (diagbuild/ travels with gpurun)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in $(seq ${R:-3}); do
  for f in "$@"; do
    echo -n "$f: "
    USV_LIB_PATH=diagbuild/abl_$f.so timeout -k 10 120 python tools/sweep_variants.py --envs ${ENVS:-65536} --variants "${VAR:-128,7,5}" --steps 2000 2>/dev/null | grep variant | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1000, 'us', d['bit_identical_to_first'])"
  done
done
