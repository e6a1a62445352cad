# A/B of library builds in build_variants/: field-op parity per build, then
# isolated stage timing (2 rounds).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
rm -f gpurun_out/variants.log gpurun_out/field_variants.log
for lib in build_variants/*.so; do
  CUDASP_LIB=$R/$lib timeout -k 10 300 python -m pytest tests/test_gpu_field.py -x -q >> gpurun_out/field_variants.log 2>&1 || { echo "field test failed for $lib"; tail -20 gpurun_out/field_variants.log; exit 1; }
done
echo "field tests ok for all variants"
for round in 1 2; do
for lib in build_variants/*.so; do
  CUDASP_LIB=$R/$lib timeout -k 10 120 python tools/stage_timing.py 300000 0 >> gpurun_out/variants.log 2>&1 || { echo "variant $lib failed"; tail -5 gpurun_out/variants.log; exit 1; }
done
done
grep "rows/s" gpurun_out/variants.log
