# k_scan_multi drain A/B: the youngest waves' claim rule (CUDASP_MULTI_YOUNG) x
# the end-game wave priority (CUDASP_MULTI_ENDGAME), device-resident bench steps
# at 1M, the N = 8 share of config 4 and config 4, interleaved, two passes; then
# per-SIMD traces of the default and of both off.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_drain; mkdir -p $O; cd $R
for pass in 1 2; do
  for rows in 1000000 4087500 32700000; do
    for v in 00 10 01 11; do
      y=${v:0:1}; e=${v:1:1}
      steps=10; [ $rows -le 4087500 ] && steps=20
      CUDASP_MULTI_YOUNG=$y CUDASP_MULTI_ENDGAME=$e timeout -k 10 300 python -u bench.py --rows $rows --steps $steps --warmup 3 --no-cpu-baseline --no-e2e --no-layout-probe --idle-samples 0 > $O/r${rows}_y${y}e${e}_$pass.json 2> $O/r${rows}_y${y}e${e}_$pass.err || { echo "bench failed"; tail -20 $O/r${rows}_y${y}e${e}_$pass.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1].ljust(28), 'M tx/s %7.2f' % (d['value']/1e6), 'kernel_ms %8.3f' % d['roofline']['kernel_ms'], 'found', d['matches']['found'], 'of', d['matches']['expected_planted'])" $O/r${rows}_y${y}e${e}_$pass.json
    done
  done
done
for rows in 1000000 4087500; do
  for v in 00 11 10; do
    y=${v:0:1}; e=${v:1:1}
    CUDASP_MULTI_YOUNG=$y CUDASP_MULTI_ENDGAME=$e CUDASP_LIB=build_variants/trace/libcudasp_amd.so timeout -k 10 300 python -u tools/multi_trace.py --rows $rows --prior 3 > $O/trace_${rows}_y${y}e${e}.json 2> $O/trace_${rows}_y${y}e${e}.err || { echo "trace failed"; tail -20 $O/trace_${rows}_y${y}e${e}.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], 'span', d['span_ms'], 'simd_idle', d['simd_idle_fraction_drain'], 'out', d['counter_out_ms'], 'rank_end', d['end_ms_mean_by_rank'], 'rows_share', d['rows_share_by_rank'])" $O/trace_${rows}_y${y}e${e}.json
  done
done
