# Diagnostics in one GPU call: ablation timings (prebuilt diag/*.so), per-wave cycle profile,
# SQ counter passes.  Ablated builds time the kernel with parts removed (results not valid).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
V=${VARIANT:-16,7,1}
O=gpurun_out/diag
mkdir -p $O
for f in "" nolidar nodyn nostore none3; do
  lib=gym-usv_amd/gym_usv_amd/libusvhip.so; [ -n "$f" ] && lib=diag/$f.so
  echo -n "${f:-full}: "
  USV_LIB_PATH=$lib timeout -k 10 120 python tools/sweep_variants.py --variants "$V" --steps 500 2>/dev/null | grep variant | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1000, 'us')"
done
USV_LIB_PATH=diag/prof.so timeout -k 10 120 python tools/prof_waves.py --variant $V > $O/prof_waves.json 2> $O/prof_waves.err
cat $O/prof_waves.json
timeout -k 10 400 bash tools/pmc_iter.sh diag 2>&1 | tail -30
