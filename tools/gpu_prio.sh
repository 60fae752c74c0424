set -e
cd $GRAFT_REPO_ROOT
for pr in 0 1 2 0; do
  echo -n "prio $pr: "
  USV_PRIO=$pr timeout -k 10 100 python tools/sweep_variants.py --variants "128,7,5" --steps 3000 2>/dev/null | grep variant | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1000, 'us')"
done
for n in 16384 262144 524288 1048576; do
  echo -n "envs $n: "
  timeout -k 10 100 python tools/sweep_variants.py --envs $n --variants "128,7,5" --steps 300 2>/dev/null | grep variant | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1000, 'us', d['env_steps_per_s'])"
done
