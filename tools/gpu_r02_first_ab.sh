# First piece of the adaptive k_scan_multi sizing: senior waves (the first block on each CU)
# start with the plain rule's piece (CUDASP_MULTI_FIRST=2, default) vs every wave with one
# wave-row (1): multi-batch GPU tests, then bench shapes, interleaved rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_multi_batch_gpu.py -x -q --timeout 300 --timeout-method thread > $O/first_tests.log 2>&1 || { echo tests failed; tail -30 $O/first_tests.log; exit 1; }
tail -1 $O/first_tests.log
B="python bench.py --no-cpu-baseline --no-e2e --no-layout-probe --exclusive-batches 0"
IFS=',' read -r -a SH <<< "${SHAPES:-32700000,8400000,4200000,9400000 --labels 1}"
for round in $(seq ${AB_ROUNDS:-3}); do
for f in 2 1; do
for rows in "${SH[@]}"; do
  CUDASP_MULTI_FIRST=$f timeout -k 10 300 $B --rows $rows --steps 5 --warmup 2 > $O/first_b.log 2>&1 || { echo "bench failed $f"; tail -20 $O/first_b.log; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('$O/first_b.log') if l.startswith('{\"metric')][-1]);print('first', sys.argv[1], 'rows', sys.argv[2], round(d['value']/1e6,2), 'M tx/s', round(d['ms_per_step'],2), 'ms', d['matches']['found'], d['matches']['expected_planted'])" $f "$rows" | tee -a $O/first_ab.txt
done
done
done
