# k_scan_multi tuning: rows per thread while much work remains (RMAX 4 / 6 /
# 8 / 12, build_variants/rmax*.so; 6 is the default build) and the guided
# thresholds (CUDASP_MULTI_G1 / G2, hundredths of the grid's waves), at the
# full table and one rank's N = 8 share.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
one() { local name=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-layout-probe --exclusive-batches 0 "$@" > $O/tune.log 2>&1 || { echo "$name failed"; tail -20 $O/tune.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); m=d['matches']
print('%-22s %.1f M tx/s %.2f ms/step found %d/%d' % (sys.argv[2], d['value']/1e6, d['ms_per_step'], m['found'], m['expected_planted']))" $O/tune.log $name; }
for rep in 1 2; do
  for lib in rmax4 rmax8 rmax12; do
    CUDASP_LIB=$R/build_variants/$lib.so one ${lib}_full --steps 4 --warmup 1
    CUDASP_LIB=$R/build_variants/$lib.so one ${lib}_s8 --rows 4200000 --steps 8 --warmup 2
  done
  for g in "150 400" "100 300" "200 600" "50 200" "300 800" "0 0"; do
    set -- $g
    CUDASP_MULTI_G1=$1 CUDASP_MULTI_G2=$2 one "g${1}_${2}_full" --steps 4 --warmup 1
    CUDASP_MULTI_G1=$1 CUDASP_MULTI_G2=$2 one "g${1}_${2}_s8" --rows 4200000 --steps 8 --warmup 2
  done
done
echo all-done
