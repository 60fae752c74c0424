# Step time of the default build over env counts (blocks per CU: N / 128 / 256).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for n in ${NS:-16384 32768 49152 65536 98304 131072 262144}; do
  echo -n "envs $n: "
  timeout -k 10 100 python tools/sweep_variants.py --envs $n --variants "128,7,5" --steps ${STEPS:-1000} 2>/dev/null | grep variant | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1000,2), 'us', d.get('env_steps_per_s'))"
done
