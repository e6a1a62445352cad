# GPU suite with the default build, then A/B of fixed-base window widths
# (asymptotic 3M-row stage timing).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
rm -f gpurun_out/variants.log
for round in 1 2; do
for lib in build_variants/*.so; do
  CUDASP_LIB=$R/$lib timeout -k 10 200 python tools/stage_timing.py 3000000 0 5 >> gpurun_out/variants.log 2>&1 || { echo "variant $lib failed"; tail -5 gpurun_out/variants.log; exit 1; }
done
done
grep "rows/s" gpurun_out/variants.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-300
