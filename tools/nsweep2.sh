# Step time of the two block-queue shapes (128 envs x 16 waves, 16 envs x 8 waves) over env counts.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for n in ${NS:-1024 4096 16384 32768 49152 65536}; do
  for v in 128,7,5 16,7,5; do
    echo -n "envs $n variant $v: "
    timeout -k 10 100 python tools/sweep_variants.py --envs $n --variants "$v" --steps ${STEPS:-1000} 2>/dev/null | grep variant | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1000,2), 'us', d.get('env_steps_per_s'))"
  done
done
