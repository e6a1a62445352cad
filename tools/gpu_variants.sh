set -o pipefail
mkdir -p gpurun_out
for round in 1 2; do
for lib in build_variants/*.so; do
  CUDASP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 python tools/stage_timing.py 300000 0 >> gpurun_out/variants.log 2>&1 || { echo "variant $lib failed"; tail -5 gpurun_out/variants.log; exit 1; }
done
done
grep "rows/s" gpurun_out/variants.log
