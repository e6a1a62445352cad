# Tail launch shapes (bench.py --tail-rows-a/-b: the last round of launches,
# one per stream, with fewer rows per thread) at the per-rank shares of the
# 32.7M-row table for N = 8 (14 batches) and N = 4 (28), and at N = 1 (109).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -30 $O/$name.log; exit 1; }; tail -1 $O/$name.log | cut -c1-150; }
cd $R
B="python bench.py --no-cpu-baseline --no-e2e --no-layout-probe --steps 10 --warmup 3"
for round in 1 2; do
for rows in 4200000 8400000; do
  for t in "0 0" "1 0" "2 0" "1 2" "2 2"; do
    set -- $t
    step tail2_${rows}_a$1_b$2_r$round 300 $B --rows $rows --tail-rows-a $1 --tail-rows-b $2
  done
done
done
for t in "0 0" "1 2" "2 0"; do
  set -- $t
  step tail2_32700000_a$1_b$2 300 $B --tail-rows-a $1 --tail-rows-b $2
done
echo all-done
