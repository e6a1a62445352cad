# Host end-to-end and the bench with GPU_MAX_HW_QUEUES = 4 (the box default),
# 8 and 16: rows mode, 8 threads, batch 300k and 75k; 2 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
rm -f $O/hwq.log
for round in 1 2; do
for Q in 4 8 16; do
for B in 300000 75000; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 120 ./tools/host_e2e 32700000 8 $B 0 2 rows >> $O/hwq.log 2> $O/hwq_err.log || { echo "host_e2e failed Q=$Q B=$B"; tail -20 $O/hwq_err.log; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('e2e', sys.argv[2], 'Q', sys.argv[3], d['batch_size'], round(d['tx_per_s']/1e6,1), d['matches'])" $O/hwq.log $round $Q
done
GPU_MAX_HW_QUEUES=$Q timeout -k 10 200 python bench.py --steps 4 --no-cpu-baseline --no-layout-probe > $O/hwq_bench.log 2>&1 || { tail -5 $O/hwq_bench.log; exit 1; }
python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print('bench', sys.argv[2], 'Q', sys.argv[3], round(d['value']/1e6,1), d['matches']['found'])" $O/hwq_bench.log $round $Q
done
done
