# PinnedTable throughput (tools/pinned_bench.py): config 4 (32.7M rows, 0 labels,
# 2 outputs), config 3 (9.4M rows, 1 label), config 2 (1M rows); each table
# pinned once, then scanned in place 3 times.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_pinned; mkdir -p $O; cd $R
for cfg in "1000000 0" "9400000 1" "32700000 0"; do
  set -- $cfg
  timeout -k 10 600 python -u tools/pinned_bench.py --rows $1 --labels $2 --reps 3 > $O/pinned_$1.json 2> $O/pinned_$1.err || { echo "pinned $1 failed"; tail -20 $O/pinned_$1.err; exit 1; }
  cat $O/pinned_$1.json
done
