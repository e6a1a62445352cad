# Adaptive piece sizing of k_scan_multi (each wave's share of the work done; the in-tree default)
# vs the plain guided rule (CUDASP_MULTI_ADAPT=0) and the earlier step rule (build_variants/r6):
# multi-batch GPU tests, per-wave traces (build_variants/trace_adapt), bench shapes.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_multi_batch_gpu.py -x -q --timeout 300 --timeout-method thread > $O/adapt_tests.log 2>&1 || { echo tests failed; tail -30 $O/adapt_tests.log; exit 1; }
tail -1 $O/adapt_tests.log
for a in 1 0; do for r in 4200000 32700000; do
  CUDASP_MULTI_ADAPT=$a CUDASP_LIB=$R/build_variants/trace_adapt/libcudasp_amd.so timeout -k 10 200 python tools/multi_trace.py --rows $r --out $O/adapt_tr_${a}_$r > $O/adapt_tr.log 2>&1 || { echo "trace failed $a"; tail -5 $O/adapt_tr.log; exit 1; }
  echo "adapt=$a $(tail -1 $O/adapt_tr.log)" | tee -a $O/adapt_trace.txt
done; done
B="python bench.py --no-cpu-baseline --no-e2e --no-layout-probe --exclusive-batches 0"
IFS=',' read -r -a SH <<< "${SHAPES:-32700000,16500000,8400000,4200000,9400000 --labels 1,9400000 --labels 16 --outputs-max 15}"
for round in $(seq ${AB_ROUNDS:-2}); do
for v in adapt plain r6; do
for rows in "${SH[@]}"; do
  lib=$R/duckdb-cudasp-extension_amd/libcudasp_amd.so; a=1
  [ $v = plain ] && a=0
  [ $v = r6 ] && lib=$R/build_variants/r6/libcudasp_amd.so
  CUDASP_MULTI_ADAPT=$a CUDASP_LIB=$lib timeout -k 10 300 $B --rows $rows --steps 5 --warmup 2 > $O/adapt_b.log 2>&1 || { echo "bench failed $v"; tail -20 $O/adapt_b.log; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('$O/adapt_b.log') if l.startswith('{\"metric')][-1]);print(sys.argv[1], 'rows', sys.argv[2], round(d['value']/1e6,2), 'M tx/s', round(d['ms_per_step'],2), 'ms', d['matches']['found'], d['matches']['expected_planted'])" $v "$rows" | tee -a $O/adapt_ab.txt
done
done
done
