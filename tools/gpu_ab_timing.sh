# A/B of the library builds in build_variants/ (asymptotic 3M-row stage timing, 2 rounds).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
rm -f gpurun_out/variants.log
for round in 1 2; do
for lib in build_variants/*.so; do
  CUDASP_LIB=$R/$lib timeout -k 10 200 python tools/stage_timing.py ${AB_ROWS:-3000000} ${AB_LABELS:-0} 5 >> gpurun_out/variants.log 2>&1 || { echo "variant $lib failed"; tail -5 gpurun_out/variants.log; exit 1; }
done
done
grep "rows/s" gpurun_out/variants.log
