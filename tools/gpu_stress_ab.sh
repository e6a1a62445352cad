# Two processes sharing the GPU, small launches, per library variant; then the
# isolated stage timing of each variant.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
ITERS=${ITERS:-2000}
for lib in build_variants/*.so; do
  v=$(basename $lib .so)
  CUDASP_LIB=$R/$lib timeout -k 10 240 python -u tools/stress_values.py --iters $ITERS --seed 2 --tag $v-p0 > $O/sab_${v}_p0.log 2>&1 &
  P0=$!
  CUDASP_LIB=$R/$lib timeout -k 10 240 python -u tools/stress_values.py --iters $ITERS --seed 3 --tag $v-p1 > $O/sab_${v}_p1.log 2>&1 &
  P1=$!
  wait $P0; r0=$?; wait $P1; r1=$?
  tail -qn1 $O/sab_${v}_p0.log $O/sab_${v}_p1.log
  [ $r0 = 0 ] && [ $r1 = 0 ] || { echo "stress failed for $v ($r0 $r1)"; exit 1; }
done
for lib in build_variants/*.so; do
  CUDASP_LIB=$R/$lib timeout -k 10 120 python tools/stage_timing.py 3000000 0 2>&1 | tail -1 || exit 1
done
