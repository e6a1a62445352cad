# PinnedTable throughput (tools/pinned_bench.py): config 4 (32.7M rows, 0 labels,
# 2 outputs), config 3 (9.4M rows, 1 label), config 2 (1M rows); each table
# pinned once, then scanned in place 3 times.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_pinned; mkdir -p $O; cd $R
for cfg in "1000000 0" "9400000 1" "32700000 0"; do
  set -- $cfg
  timeout -k 10 600 python -u tools/pinned_bench.py --rows $1 --labels $2 --reps 3 > $O/pinned_$1.json 2> $O/pinned_$1.err || { echo "pinned $1 failed"; tail -20 $O/pinned_$1.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('pinned', sys.argv[2], '%.1f M exact %s pin %.2f s' % (d['tx_per_s']/1e6, d['exact'], d['pin_s']))" $O/pinned_$1.json $1
done
# the same tables through the table-function host (copies into slots), warm
# queries on the same box, for the comparison
python3 -c "import bench; open('$O/labels1.bin','wb').write(b''.join(bench.label_keys(1)))"
for cfg in "1000000 0" "9400000 1" "32700000 0"; do
  set -- $cfg
  lf=""; [ $2 -gt 0 ] && lf="--labels-file $O/labels1.bin"
  timeout -k 10 300 tools/host_e2e --rows $1 --threads 8 --batch 300000 --labels $2 $lf --outputs 2 --reps 3 --warm-reps 3 > $O/e2e_$1.json 2> $O/e2e_$1.err || { echo "e2e $1 failed"; tail -5 $O/e2e_$1.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('host e2e', sys.argv[2], 'cold %.1f M warm %.1f M exact %s' % (d['tx_per_s']/1e6, d['warm_tx_per_s']/1e6, d['emitted_equal_planted']))" $O/e2e_$1.json $1
done
