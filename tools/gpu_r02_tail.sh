# Strong-scaling rehearsal on one MI355X: the per-rank share of the 32.7M-row
# table at N = 2, 4, 8 (55 / 28 / 14 batches of 300k rows) scanned alone, with
# the default launch shapes and with stage A forced to 2 rows per thread
# (shorter launches, better tail), then e2e repeat runs (bimodality), the
# optimized CPU baseline on the box's cores.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -30 $O/$name.log; exit 1; }; tail -1 $O/$name.log | cut -c1-200; }
cd $R
B="python bench.py --no-cpu-baseline --no-e2e --no-layout-probe --steps 10 --warmup 3"
for rows in 4200000 8400000 16500000 32700000; do
  step tail_${rows}_s4 300 $B --rows $rows
  CUDASP_ROWS_A_FORCE=2 step tail_${rows}_s4_ra2 300 $B --rows $rows
  step tail_${rows}_s8 300 $B --rows $rows --streams 8
done
for i in 1 2 3 4 5 6; do
  GPU_MAX_HW_QUEUES=16 CUDASP_FB_BITS=26 step e2e_rep_$i 120 tools/host_e2e 32700000 8 300000 0 2 rows
done
step bench_cpu 600 python bench.py --steps 3 --no-e2e --no-layout-probe
echo all-done
