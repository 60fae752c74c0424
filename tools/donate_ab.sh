# A/B of the block-queue step with and without work donation (USV_DONATE=0), interleaved.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for r in 1 2 3; do
  for d in 1 0; do
    echo -n "donate $d: "
    USV_DONATE=$d timeout -k 10 120 python tools/sweep_variants.py --variants "128,7,5" --steps 2000 2>/dev/null | grep variant | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1000, 'us')"
  done
done
