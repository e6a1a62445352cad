# Host end-to-end with per-thread timings (time inside the table-function
# calls, inside final, thread end times): rows mode, 8 threads, batch 300k
# and 75k, 4 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
rm -f $O/e2e_thr.log
for round in 1 2 3 4; do
for B in 300000 75000; do
  timeout -k 10 120 ./tools/host_e2e 32700000 8 $B 0 2 rows >> $O/e2e_thr.log 2> $O/e2e_thr_err.log || { echo "host_e2e failed B=$B"; tail -20 $O/e2e_thr_err.log; exit 1; }
  python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(d['batch_size'], round(d['tx_per_s']/1e6,1), 'total', d['seconds'], 'calls', d['thread_call_s_mean'], 'long', d['thread_long_call_s_mean'], 'final', d['thread_final_s_mean'], 'done', d['thread_done_s_min'], d['thread_done_s_max'])" $O/e2e_thr.log
done
done
