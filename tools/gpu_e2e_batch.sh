# Host end-to-end (PCIe-inclusive) at several batch sizes, rows and Arrow
# columns, 8 threads, 3 rounds interleaved (the run-to-run spread is ~±8%).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
rm -f $O/e2e_batch.log
for round in 1 2 3; do
for mode in rows columns; do
for B in ${E2E_BATCHES:-300000 150000 75000}; do
  timeout -k 10 120 ./tools/host_e2e 32700000 8 $B 0 2 $mode >> $O/e2e_batch.log 2> $O/e2e_batch_err.log || { echo "host_e2e failed B=$B $mode"; tail -20 $O/e2e_batch_err.log; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], d['input'], d['batch_size'], round(d['tx_per_s']/1e6,1), d['matches'], d['planted'])" $O/e2e_batch.log $round
done
done
done
