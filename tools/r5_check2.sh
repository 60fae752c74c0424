# Round-5 profiles, second batch: the reference precision (f64 usv-simple kind 3 and f64
# usv-asmc-simple kind 2), the DRAM-resident size (524 288 envs), the per-wave timeline of the
# headline kernel (stamps build) and the API / SB3 throughput at 4 096 envs.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5k
mkdir -p $O
stop() { case $1 in 124|134|137|139) echo "stopping after rc $1"; exit $1;; esac; }
PREC=f64 bash tools/profile_round.sh r05_f64 > $O/prof_f64.log 2>&1
rc=$?; echo "prof f64 rc $rc"; stop $rc
PREC=f64 ENV_ID=usv-asmc-simple KERNELS="usv::(dyn_kernel|scan_kernel)" bash tools/profile_round.sh r05_f64asmc > $O/prof_f64asmc.log 2>&1
rc=$?; echo "prof f64 asmc rc $rc"; stop $rc
ENVS=524288 KT_STEPS=400 bash tools/profile_round.sh r05_524k > $O/prof_524k.log 2>&1
rc=$?; echo "prof 524k rc $rc"; stop $rc
[ -f diagbuild/stamps.so ] && USV_LIB_PATH=diagbuild/stamps.so timeout -k 10 200 python tools/wave_timeline.py --envs 65536 --variant 128,7,5 > $O/timeline.json 2> $O/timeline.err
rc=$?; echo "timeline rc $rc"; stop $rc
timeout -k 10 200 python tools/api_throughput.py --envs 4096 > $O/api_4096.json 2>&1
rc=$?; echo "api rc $rc"; stop $rc
