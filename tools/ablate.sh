# diagnostic ablations of the fused step kernel: time with parts removed (results not valid)
set -e
cd $GRAFT_REPO_ROOT
V=${VARIANT:-64,7,1}
for f in NONE USV_ABL_NOLIDAR USV_ABL_NODYN USV_ABL_NOSTORE "USV_ABL_NOLIDAR -DUSV_ABL_NODYN" "USV_ABL_NOLIDAR -DUSV_ABL_NOSTORE" "USV_ABL_NOLIDAR -DUSV_ABL_NODYN -DUSV_ABL_NOSTORE"; do
  hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -shared -Iinclude -D$f -o /tmp/libabl.so gym-usv_amd/csrc/usv_kernels.hip
  echo -n "$f: "
  USV_LIB_PATH=/tmp/libabl.so timeout -k 10 120 python tools/sweep_variants.py --variants "$V" --steps 500 2>/dev/null | grep variant | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']*1000, 'us')"
done
