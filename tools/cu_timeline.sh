# Per-CU timeline of the block-queue step (diagbuild/stamps.so): which CUs end the launch, and whether
# their end follows their dispatch time.  Build first: bash tools/build_diag.sh STAMPS.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/cutl
for r in 1 2; do
  USV_LIB_PATH=${LIB:-diagbuild/stamps.so} timeout -k 10 120 python tools/wave_timeline.py --variant 128,7,5 > gpurun_out/cutl/run$r.json 2> gpurun_out/cutl/run$r.err
done
python -c "
import json
for r in (1, 2):
    d = json.load(open('gpurun_out/cutl/run%d.json' % r))
    print({k: d[k] for k in ('event_us', 'span_us', 'cu_start_us', 'cu_end_us', 'cu_busy_us', 'corr_cu_start_end', 'cu_end_by_xcc', 'cu_start_by_xcc', 'cu_busy_by_xcc', 'older_busy_by_xcc', 'cu_end_by_se_mean', 'older_block_start_end_us', 'younger_block_start_end_us', 'pairs_per_wave', 'slowest_cus')})
"
