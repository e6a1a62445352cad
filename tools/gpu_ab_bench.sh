# GPU suite with the default build, A/B stage timing of build_variants/*.so, then
# the default bench with each variant (value, kernel_ms).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
bash tools/gpu_ab_timing.sh || exit 1
for lib in build_variants/*.so; do
  CUDASP_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_ab.log 2>&1 || { tail -5 gpurun_out/bench_ab.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/bench_ab.log').read().strip().splitlines()[-1]);print(sys.argv[1], round(d['value']/1e6,2), 'M tx/s', d['matches'])" $lib
done
