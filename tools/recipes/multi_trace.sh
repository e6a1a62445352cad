# Per-wave / per-SIMD timeline of k_scan_multi launches (trace build in
# build_variants/trace, -DCUDASP_MULTI_TRACE=1) at the given row counts.
#   ROWS="1000000 4087500 32700000" (default), MEASURE_TAG names the output directory
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_trace; mkdir -p $O; cd $R
for rows in ${ROWS:-1000000 4087500 32700000}; do
  CUDASP_LIB=build_variants/trace/libcudasp_amd.so timeout -k 10 300 python -u tools/multi_trace.py --rows $rows --out $O/trace_$rows.npz > $O/trace_$rows.json 2> $O/trace_$rows.err || { echo "trace $rows failed"; tail -20 $O/trace_$rows.err; exit 1; }
  cat $O/trace_$rows.json
done
