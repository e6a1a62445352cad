# End-to-end (PCIe-inclusive) rate of the table-function host against the
# executor thread count (DuckDB's default is one thread per core; the box's
# CPU share is 16) at the bench's shape, 16 hardware queues, two rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
export CUDASP_FB_BITS=26 GPU_MAX_HW_QUEUES=16
for round in 1 2; do
for t in 8 12 16 4; do
  timeout -k 10 200 tools/host_e2e 32700000 $t 300000 0 2 rows > $O/e2e_t.log 2>&1 || { echo "e2e failed t=$t"; tail -20 $O/e2e_t.log; exit 1; }
  echo "threads $t $(tail -1 $O/e2e_t.log | cut -c1-220)" | tee -a $O/e2e_threads.txt
done
done
echo all-done
