# Shader clock of a k_scan_multi launch against the host gap before it (trace
# build): queued right behind the previous launches (-1), after a synchronize
# (0), after 1 / 10 / 100 ms of sleep.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_clockgap; mkdir -p $O; cd $R
for rows in ${ROWS:-1000000 4087500}; do
  for gap in -1 0 1 10 100; do
    CUDASP_LIB=build_variants/trace/libcudasp_amd.so timeout -k 10 300 python -u tools/multi_trace.py --rows $rows --gap-ms $gap --prior 3 > $O/gap_${rows}_$gap.json 2> $O/gap_${rows}_$gap.err || { echo "gap $rows $gap failed"; tail -20 $O/gap_${rows}_$gap.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['rows'], d['gap_ms'], 'span', d['span_ms'], 'clock', d['shader_clock_mhz_p1_p50_p99'], 'simd_idle', d['simd_idle_fraction_drain'])" $O/gap_${rows}_$gap.json
  done
done
