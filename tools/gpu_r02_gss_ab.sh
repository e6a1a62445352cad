# Guided self-scheduling rule (pieces of rem / waves rows, 1..6; the in-tree build = build_variants/gss)
# vs the earlier step rule (6 rows above 4 x waves wave-rows left, 2 above 1.5 x, then 1;
# build_variants/r6): multi-batch GPU tests, per-wave traces (trace builds), bench shapes.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_multi_batch_gpu.py -x -q --timeout 300 --timeout-method thread > $O/gss_tests.log 2>&1 || { echo tests failed; tail -30 $O/gss_tests.log; exit 1; }
tail -1 $O/gss_tests.log
for v in trace trace_gss; do for r in 4200000 8400000 32700000; do
  CUDASP_LIB=$R/build_variants/$v/libcudasp_amd.so timeout -k 10 200 python tools/multi_trace.py --rows $r > $O/gss_tr.log 2>&1 || { echo "trace failed $v"; tail -5 $O/gss_tr.log; exit 1; }
  echo "$v $(tail -1 $O/gss_tr.log)" | tee -a $O/gss_trace.txt
done; done
B="python bench.py --no-cpu-baseline --no-e2e --no-layout-probe --exclusive-batches 0"
IFS=',' read -r -a SH <<< "${SHAPES:-32700000,16500000,8400000,4200000,9400000 --labels 1,9400000 --labels 16 --outputs-max 15}"
for round in $(seq ${AB_ROUNDS:-2}); do
for v in gss r6; do
for rows in "${SH[@]}"; do
  CUDASP_LIB=$R/build_variants/$v/libcudasp_amd.so timeout -k 10 300 $B --rows $rows --steps 5 --warmup 2 > $O/gss_b.log 2>&1 || { echo "bench failed $v"; tail -20 $O/gss_b.log; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('$O/gss_b.log') if l.startswith('{\"metric')][-1]);print(sys.argv[1], 'rows', sys.argv[2], round(d['value']/1e6,2), 'M tx/s', round(d['ms_per_step'],2), 'ms', d['matches']['found'], d['matches']['expected_planted'])" $v "$rows" | tee -a $O/gss_ab.txt
done
done
done
