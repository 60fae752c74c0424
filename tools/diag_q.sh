# Block-queue step (kind 5) diagnostics: ablation timings (diag/abl_*.so, results not valid) and
# the per-wave stamp timeline (diag/stamps.so).  Build the libraries on the CPU side first, and take
# ./diag out of .gpurunignore for the run (it is kept off routine GPU pushes).
set -e
cd $GRAFT_REPO_ROOT
V=${VARIANT:-128,7,5}
O=gpurun_out/diag_q
mkdir -p $O
for f in full NOLIDAR NOSTORE; do
  lib=gym-usv_amd/gym_usv_amd/libusvhip.so; [ $f != full ] && lib=diag/abl_$f.so
  echo -n "$f: "
  USV_LIB_PATH=$lib timeout -k 10 120 python tools/sweep_variants.py --variants "$V" --steps 500 2>/dev/null | grep variant | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1000, 'us')"
done
USV_LIB_PATH=diag/stamps.so timeout -k 10 120 python tools/wave_timeline.py --variant $V > $O/timeline.json 2> $O/timeline.err
cat $O/timeline.json
