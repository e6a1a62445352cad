# Row-major tweaks read by the fused single-batch launch in the table-function (a build since reverted;
# host (no k_rows_to_cols dispatch) vs the transpose (CUDASP_TF_TRANSPOSE=1):
# the host's GPU tests under both, then end to end at 8 threads, 3 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_sql_cases_gpu.py tests/test_arrow_gpu.py tests/test_labels16_gpu.py -x -q --timeout 120 --timeout-method thread > $O/rm_tests.log 2>&1 || { echo tests failed; tail -30 $O/rm_tests.log; exit 1; }
tail -1 $O/rm_tests.log
CUDASP_TF_TRANSPOSE=1 timeout -k 10 300 python -u -m pytest tests/test_sql_cases_gpu.py -x -q --timeout 120 --timeout-method thread > $O/rm_tests2.log 2>&1 || { echo tests2 failed; tail -30 $O/rm_tests2.log; exit 1; }
tail -1 $O/rm_tests2.log
export CUDASP_FB_BITS=26 GPU_MAX_HW_QUEUES=16
for round in 1 2 3; do
for v in rows transpose; do
  if [ $v = transpose ]; then export CUDASP_TF_TRANSPOSE=1; else unset CUDASP_TF_TRANSPOSE; fi
  timeout -k 10 200 tools/host_e2e 32700000 8 300000 0 2 rows > $O/e2e_rm.log 2>&1 || { echo "e2e failed $v"; tail -20 $O/e2e_rm.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('$O/e2e_rm.log').read().strip().splitlines()[-1]);print(sys.argv[1], round(d['tx_per_s']/1e6,2), 'M tx/s', d['seconds'], 's', d['matches'], d['planted'])" $v | tee -a $O/rowmajor_ab.txt
done
done
echo all-done
