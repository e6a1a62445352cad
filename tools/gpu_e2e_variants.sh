# Host end-to-end (PCIe-inclusive) for rows and Arrow columns, then the bench
# with the protocol variants (K = 2; 1 label with negation).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
rm -f $O/e2e.log
for mode in rows columns; do
for T in 8 16; do
  timeout -k 10 300 ./tools/host_e2e 32700000 $T 300000 0 2 $mode >> $O/e2e.log 2> $O/e2e_err.log || { echo "host_e2e failed T=$T $mode"; tail -20 $O/e2e_err.log; exit 1; }
  tail -1 $O/e2e.log | cut -c1-400
done
done
timeout -k 10 300 python bench.py --steps 2 --output-count 2 --cpu-rows 300000 > $O/bench_k2.log 2>&1 || { tail -20 $O/bench_k2.log; exit 1; }
tail -1 $O/bench_k2.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 2 --rows 9400000 --labels 1 --label-negation --cpu-rows 300000 > $O/bench_neg.log 2>&1 || { tail -20 $O/bench_neg.log; exit 1; }
tail -1 $O/bench_neg.log | cut -c1-200
