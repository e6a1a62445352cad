# Per-device in-flight cap of the table-function host (CUDASP_TF_INFLIGHT; a build since reverted)
# A/B: end-to-end rate at 8 and 16 executor threads, cap unset / 4 / 6 / 8;
# first the table-function GPU tests under the cap.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
CUDASP_TF_INFLIGHT=2 timeout -k 10 300 python -u -m pytest tests/test_sql_cases_gpu.py tests/test_arrow_gpu.py -x -q --timeout 120 --timeout-method thread > $O/inflight_tests.log 2>&1 || { echo tests failed; tail -30 $O/inflight_tests.log; exit 1; }
tail -1 $O/inflight_tests.log
export CUDASP_FB_BITS=26 GPU_MAX_HW_QUEUES=16
for round in 1 2; do
for t in 8 16; do
for cap in 0 4 6 8; do
  CUDASP_TF_INFLIGHT=$cap timeout -k 10 200 tools/host_e2e 32700000 $t 300000 0 2 rows > $O/e2e_i.log 2>&1 || { echo "e2e failed t=$t cap=$cap"; tail -20 $O/e2e_i.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('$O/e2e_i.log').read().strip().splitlines()[-1]);print('threads', sys.argv[1], 'cap', sys.argv[2], round(d['tx_per_s']/1e6,2), 'M tx/s', d['seconds'], 's', d['matches'], d['planted'])" $t $cap | tee -a $O/inflight_ab.txt
done
done
done
echo all-done
