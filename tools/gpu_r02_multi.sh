# Multi-batch persistent scan (cudasp_scan_device_batches / k_scan_multi):
# its GPU tests, then bench A/B of --launch multi vs --launch batches at the
# full table and at one rank's share of N = 8 (14 batches).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_multi_batch_gpu.py -x -v --timeout 300 --timeout-method thread > $O/multi_tests.log 2>&1 || { echo tests failed; grep -E "PASS|FAIL|Error" $O/multi_tests.log | tail -20; tail -30 $O/multi_tests.log; exit 1; }
tail -1 $O/multi_tests.log
one() { local name=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-layout-probe "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -20 $O/$name.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; m=d['matches']
print('%-12s %.1f M tx/s %.2f ms/step kernel %s %.3f ms found %d/%d/%d' % (sys.argv[2], d['value']/1e6, d['ms_per_step'], r['kernel'], r['kernel_ms'], m['found'], m['flagged'], m['expected_planted']))" $O/$name.log $name; }
for rep in 1 2; do
  one multi_full_$rep --steps 5 --warmup 2 --launch multi
  one batch_full_$rep --steps 5 --warmup 2 --launch batches
  one multi_s8_$rep --rows 4200000 --steps 10 --warmup 2 --launch multi
  one batch_s8_$rep --rows 4200000 --steps 10 --warmup 2 --launch batches
done
one multi_L16 --rows 6000000 --labels 16 --outputs-max 15 --steps 3 --launch multi
one batch_L16 --rows 6000000 --labels 16 --outputs-max 15 --steps 3 --launch batches
echo all-done
