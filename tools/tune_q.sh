# Timings of the block-queue step under the wave-priority policies (USV_PRIO) and the split variant.
set -e
cd $GRAFT_REPO_ROOT
for cfg in "0 128,7,5" "1 128,7,5" "3 128,7,5" "0 128,7,4" "1 128,7,4"; do
  set -- $cfg
  echo -n "prio $1 variant $2: "
  USV_PRIO=$1 timeout -k 10 120 python tools/sweep_variants.py --variants "$2" --steps 1000 2>/dev/null | grep variant | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step']*1000, 2), 'us')"
done
