# Per-wave stamp timelines of the block-queue step under USV_PRIO 0 and 1 (diag/stamps.so).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
for pr in 0 1; do
  USV_PRIO=$pr USV_LIB_PATH=diag/stamps.so timeout -k 10 120 python tools/wave_timeline.py --variant 128,7,5 > gpurun_out/tl/prio$pr.json 2> gpurun_out/tl/prio$pr.err
  python -c "import json; d=json.load(open('gpurun_out/tl/prio$pr.json')); print('prio $pr', {k: d[k] for k in ('event_us','span_us','block_end_us','older_block_start_end_us','younger_block_start_end_us','alive_waves_over_time')})"
done
