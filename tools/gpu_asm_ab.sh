# GPU check of the asm field ops: field tests, full GPU suite, stage A/B timing
# of variant 1 (C) vs variant 3 (asm), then the default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -m pytest tests/test_gpu_field.py -x -q > gpurun_out/field.log 2>&1 || { tail -30 gpurun_out/field.log; exit 1; }
tail -2 gpurun_out/field.log
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
rm -f gpurun_out/variants.log
for round in 1 2; do
for lib in build_variants/*.so; do
  CUDASP_LIB=$R/$lib timeout -k 10 120 python tools/stage_timing.py 300000 0 >> gpurun_out/variants.log 2>&1 || { echo "variant $lib failed"; tail -5 gpurun_out/variants.log; exit 1; }
done
done
grep "rows/s" gpurun_out/variants.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
