# End-to-end A/B of the batch ramp (CUDASP_TF_RAMP halvings of a thread's first
# batch, cudasp_host.cpp batch_trigger): tools/host_e2e, 32.7M rows, 8 threads,
# 300k batches, interleaved rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
export CUDASP_FB_BITS=26
for round in $(seq ${AB_ROUNDS:-3}); do
for ramp in ${RAMPS:-0 3 2 4}; do
  CUDASP_TF_RAMP=$ramp timeout -k 10 120 ./tools/host_e2e 32700000 8 300000 0 2 ${MODE:-rows} > $O/ramp.log 2> $O/ramp_err.log || { echo "failed ramp $ramp"; tail -5 $O/ramp_err.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('$O/ramp.log').read().strip().splitlines()[-1]);print('ramp', sys.argv[1], round(d['tx_per_s']/1e6,2), 'M tx/s', d['matches'], d['planted'], 'done', d['thread_done_s_min'], d['thread_done_s_max'])" $ramp | tee -a $O/ramp_ab.txt
done
done
