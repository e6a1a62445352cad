# Scratch-traffic A/B: product build vs CUDASP_AB_SCRATCH_ALIAS
# = 1024 / 65536 / 131072 slots (per-row scratch folded into a 1.7 MB / 111 MB /
# 222 MB region: L2- / MALL-resident; timing only) vs stage A at 2 waves per
# SIMD (2/3 of the resident threads' scratch).  Asymptotic 3M-row stage timing,
# 2 rounds, then the device-resident bench (4 streams) for each build.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -30 $O/$name.log; exit 1; }; tail -1 $O/$name.log | cut -c1-220; }
cd $R
for round in 1 2; do
  for lib in build_variants/*.so; do
    v=$(basename $lib .so)
    CUDASP_LIB=$R/$lib step st_${v}_$round 200 python tools/stage_timing.py 3000000 0 5
  done
done
for lib in build_variants/*.so; do
  v=$(basename $lib .so)
  CUDASP_LIB=$R/$lib step bench_$v 300 python bench.py --no-cpu-baseline --no-e2e --no-layout-probe --steps 5 --warmup 2
done
echo all-done
