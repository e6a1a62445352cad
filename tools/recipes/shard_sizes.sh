# Device-only bench at each GPU's share of config 4 for N = 1, 2, 4, 8 (the rows
# one GPU scans in the driver's SCALE run), same box, two interleaved passes.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_shards; mkdir -p $O; cd $R
for pass in 1 2; do
  for rows in 4087500 8175000 16350000 32700000; do
    timeout -k 10 300 python -u bench.py --rows $rows --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-layout-probe --no-cold-start --idle-samples 0 > $O/rows_${rows}_$pass.json 2> $O/rows_${rows}_$pass.err || { echo "bench $rows failed"; tail -20 $O/rows_${rows}_$pass.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], 'value %.2f M' % (d['value']/1e6), 'kernel_ms %.3f' % d['roofline']['kernel_ms'], 'batches', d['config'].get('batches_rank0'))" $O/rows_${rows}_$pass.json $rows $pass
  done
done
# per-wave timeline of one launch at the N = 8 and N = 1 shares (trace build, if present)
if [ -f build_variants/trace/libcudasp_amd.so ]; then
  for rows in 4087500 32700000; do
    CUDASP_LIB=build_variants/trace/libcudasp_amd.so timeout -k 10 300 python -u tools/multi_trace.py --rows $rows > $O/trace_$rows.json 2> $O/trace_$rows.err || { echo "trace $rows failed"; tail -20 $O/trace_$rows.err; exit 1; }
    cat $O/trace_$rows.json
  done
fi
