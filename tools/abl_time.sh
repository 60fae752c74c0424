# Step time of the default build against diagnostic builds diag/abl_<X>.so (ablations: results
# invalid by design).  Usage: bash tools/abl_time.sh X[:epb,lid,kind] ...  (diag/ must not be gpurun-ignored)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for a in full "$@" full; do
  f=${a%%:*}; v=128,7,5; [ "$a" != "$f" ] && v=${a#*:}
  lib=gym-usv_amd/gym_usv_amd/libusvhip.so; [ $f != full ] && lib=diag/abl_$f.so
  echo -n "$f ($v): "
  USV_LIB_PATH=$lib timeout -k 10 120 python tools/sweep_variants.py --envs ${ENVS:-65536} --variants "$v" --steps 2000 2>/dev/null | grep variant | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1000, 'us')"
done
