# Aggregated launches in the table-function host (CUDASP_TF_AGGREGATE, default
# on): the GPU tests of the host paths, then the host end-to-end leg A/B
# (tools/host_e2e via bench.py's e2e leg; device legs skipped where possible).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests/test_sql_cases_gpu.py tests/test_arrow_gpu.py tests/test_variants_gpu.py tests/test_labels16_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/agg_tests.log 2>&1 || { echo tests failed; tail -30 $O/agg_tests.log; exit 1; }
tail -1 $O/agg_tests.log
E=tools/host_e2e
for rep in 1 2 3; do
  for agg in 1 0; do
    CUDASP_TF_AGGREGATE=$agg CUDASP_FB_BITS=26 GPU_MAX_HW_QUEUES=16 timeout -k 10 300 $E 32700000 8 300000 0 2 rows > $O/agg_e2e.log 2>&1 || { echo "e2e agg=$agg failed"; tail -20 $O/agg_e2e.log; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('agg=%s %.1f M tx/s matches %d/%d done %.4f-%.4f s' % (sys.argv[2], d['tx_per_s']/1e6, d['matches'], d['planted'], d['thread_done_s_min'], d['thread_done_s_max']))" $O/agg_e2e.log $agg
  done
done
echo all-done
