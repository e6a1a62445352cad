# Fused single-batch k_scan_multi launches (the per-batch path: bench --launch batches, the
# table-function host) with adaptive piece sizing on the same grid (CUDASP_FUSED_ADAPT=1)
# vs one 4-row piece per wave (0): GPU tests under it, then interleaved rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
CUDASP_FUSED_ADAPT=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "multi or sql or parity or label" --timeout 300 --timeout-method thread > $O/fa_tests.log 2>&1 || { echo tests failed; tail -30 $O/fa_tests.log; exit 1; }
tail -1 $O/fa_tests.log
export CUDASP_FB_BITS=26
for round in $(seq ${AB_ROUNDS:-3}); do
for a in 1 0; do
  export CUDASP_FUSED_ADAPT=$a
  timeout -k 10 300 python bench.py --launch batches --no-cpu-baseline --no-e2e --no-layout-probe --exclusive-batches 0 --steps 5 --warmup 2 > $O/fa_b.log 2>&1 || { echo "bench failed $a"; tail -20 $O/fa_b.log; exit 1; }
  timeout -k 10 120 ./tools/host_e2e 32700000 8 300000 0 2 rows > $O/fa_e.log 2> $O/fa_e_err.log || { echo "e2e failed $a"; tail -5 $O/fa_e_err.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('$O/fa_b.log') if l.startswith('{\"metric')][-1]); e=json.loads(open('$O/fa_e.log').read().strip().splitlines()[-1])
print('fused_adapt', sys.argv[1], 'batches', round(d['value']/1e6,2), 'M tx/s', d['matches']['found'], '| e2e', round(e['tx_per_s']/1e6,2), 'M tx/s', e['matches'], e['planted'], 'done', e['thread_done_s_min'], e['thread_done_s_max'])" $a | tee -a $O/fused_adapt_ab.txt
done
done
