set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/exp1
for r in 1 2; do
  USV_LIB_PATH=diagbuild/stamps.so timeout -k 10 120 python tools/wave_timeline.py --variant 128,7,5 > gpurun_out/exp1/tl$r.json 2> gpurun_out/exp1/tl$r.err
done
for r in 1 2 3; do
  for lib in gym-usv_amd/gym_usv_amd/libusvhip.so diagbuild/out1.so diagbuild/out2.so; do
    echo -n "$lib: "
    USV_LIB_PATH=$lib timeout -k 10 120 python tools/sweep_variants.py --envs 65536 --variants "128,7,5" --steps 3000 2>/dev/null | tail -1
  done
done
