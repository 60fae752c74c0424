# Step time of the default build under the USV_PRIO tuning modes of the block-queue step.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for pr in 0 1 3 0 1 3; do
  echo -n "prio $pr: "
  USV_PRIO=$pr timeout -k 10 100 python tools/sweep_variants.py --variants "128,7,5" --steps 2000 2>/dev/null | grep variant | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1000, 'us')"
done
