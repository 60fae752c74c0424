# Ablation timings (diag/abl_*.so, results invalid by design) and the per-wave stamp timeline of the
# block-queue step.  Build first: bash tools/build_diag.sh NOLIDAR NOSTORE NODYN STAMPS (diag/ must not
# be in .gpurunignore for the run).  Usage: bash tools/diag_q3.sh TAG
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-q3}
O=gpurun_out/diag_$T
mkdir -p $O
for f in full NOLIDAR NOSTORE NODYN; do
  lib=gym-usv_amd/gym_usv_amd/libusvhip.so; [ $f != full ] && lib=diag/abl_$f.so
  echo -n "$f: "
  USV_LIB_PATH=$lib timeout -k 10 120 python tools/sweep_variants.py --variants "128,7,5" --steps 1000 2>/dev/null | grep variant | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1000, 'us')"
done
USV_LIB_PATH=diag/stamps.so timeout -k 10 120 python tools/wave_timeline.py --variant 128,7,5 > $O/timeline.json 2> $O/timeline.err
cat $O/timeline.json
