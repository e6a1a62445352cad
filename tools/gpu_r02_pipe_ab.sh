# Pipelined k_scan_multi schedule (one inversion per piece, CUDASP_MULTI_PIPE=1, the default)
# vs two (three with labels) inversions per piece (CUDASP_MULTI_PIPE=0): multi-batch GPU tests,
# then the default bench, a rank's N = 8 share and 1- / 16-label shapes, interleaved rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_multi_batch_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pipe_tests.log 2>&1 || { echo tests failed; tail -30 $O/pipe_tests.log; exit 1; }
tail -1 $O/pipe_tests.log
B="python bench.py --no-cpu-baseline --no-e2e --no-layout-probe --exclusive-batches 0"
for round in $(seq ${AB_ROUNDS:-3}); do
for pipe in 1 0; do
for shape in "32700000" "4200000" "9400000 --labels 1" "9400000 --labels 16 --outputs-max 15"; do
  CUDASP_MULTI_PIPE=$pipe timeout -k 10 300 $B --rows $shape --steps 5 --warmup 2 > $O/pipe_b.log 2>&1 || { echo "bench failed pipe $pipe"; tail -20 $O/pipe_b.log; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('$O/pipe_b.log') if l.startswith('{\"metric')][-1]);print('pipe', sys.argv[1], 'rows', sys.argv[2], round(d['value']/1e6,2), 'M tx/s', round(d['ms_per_step'],2), 'ms', d['matches']['found'], d['matches']['expected_planted'])" $pipe "$shape" | tee -a $O/pipe_ab.txt
done
done
done
