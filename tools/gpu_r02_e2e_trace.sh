# Kernel + memory-copy traces of the end-to-end host (tools/host_e2e, 32.7M
# rows, 300k batches; executor threads per run from E2E_THREADS, default "8 8") for tools/timeline.py: how long the GPU waits
# for the first batches, and the drain at the end of the query.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
export CUDASP_FB_BITS=26 GPU_MAX_HW_QUEUES=${E2E_HWQ:-16}  # rocprofv3 initialises HIP before host_e2e can set it
i=0
for t in ${E2E_THREADS:-8 8}; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/e2etr_$i -o t -- $R/tools/host_e2e ${E2E_ROWS:-32700000} $t ${E2E_BATCH:-300000} 0 2 rows > $O/e2etr_$i.log 2>&1 || { echo run $i failed; tail $O/e2etr_$i.log; exit 1; }
  echo "threads $t"; tail -1 $O/e2etr_$i.log | cut -c1-400
  K=$(ls $O/e2etr_$i/*kernel_trace.csv $O/e2etr_$i/*/*kernel_trace.csv 2>/dev/null | head -1)
  C=$(ls $O/e2etr_$i/*memory_copy_trace.csv $O/e2etr_$i/*/*memory_copy_trace.csv 2>/dev/null | head -1)
  python3 $R/tools/timeline.py "$K" --copies "$C" > $O/e2etr_$i.txt && cat $O/e2etr_$i.txt
done
