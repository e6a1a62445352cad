# Full GPU suite for every build in build_variants/ (via CUDASP_LIB), then the
# A/B stage timing and bench of each.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for lib in build_variants/*.so; do
  CUDASP_LIB=$R/$lib timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests_$(basename $lib .so).log 2>&1 || { echo "GPU tests failed for $lib"; tail -30 gpurun_out/gpu_tests_$(basename $lib .so).log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/gpu_tests_$(basename $lib .so).log)"
done
bash tools/gpu_ab_timing.sh || exit 1
AB_STEPS=5 bash tools/gpu_ab_bench_only.sh
