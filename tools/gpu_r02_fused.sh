# Fused single-batch launches (CUDASP_FUSED_SINGLE=1: cudasp_scan_device runs
# both stages in one k_scan_multi launch, 4 rows per thread): the whole GPU test
# suite under it, then bench --launch batches and the host end-to-end leg A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
CUDASP_FUSED_SINGLE=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/fused_tests.log 2>&1 || { echo tests failed; tail -30 $O/fused_tests.log; exit 1; }
tail -1 $O/fused_tests.log
one() { local name=$1; shift; timeout -k 10 400 python bench.py --no-cpu-baseline --no-layout-probe "$@" > $O/fused.log 2>&1 || { echo "$name failed"; tail -20 $O/fused.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); m=d['matches']
print('%-14s %.1f M tx/s e2e %s found %d/%d' % (sys.argv[2], d['value']/1e6, d.get('e2e_tx_s'), m['found'], m['expected_planted']))" $O/fused.log $name; }
for rep in 1 2; do
  CUDASP_FUSED_SINGLE=1 one fused_$rep --launch batches --steps 5 --warmup 2
  one split_$rep --launch batches --steps 5 --warmup 2
done
echo all-done
