# A/B of build_variants/*.so: isolated stage timing at 0, 1 and 16 labels,
# then the bench at config-3 shape (1 label) and the default (0 labels).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
rm -f $O/ab_labels.log
for L in 0 1 16; do
for lib in build_variants/*.so; do
  CUDASP_LIB=$R/$lib timeout -k 10 200 python tools/stage_timing.py 3000000 $L 5 >> $O/ab_labels.log 2>&1 || { echo "variant $lib failed"; tail -5 $O/ab_labels.log; exit 1; }
done
done
grep "rows/s" $O/ab_labels.log
for lib in build_variants/*.so; do
  CUDASP_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-layout-probe --rows 9400000 --labels 1 --steps 4 > $O/bench_ab.log 2>&1 || { tail -5 $O/bench_ab.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('$O/bench_ab.log').read().strip().splitlines()[-1]);print(sys.argv[1], 'L1', round(d['value']/1e6,2), 'M tx/s', d['matches'])" $lib
  CUDASP_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-layout-probe --steps 4 > $O/bench_ab.log 2>&1 || { tail -5 $O/bench_ab.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('$O/bench_ab.log').read().strip().splitlines()[-1]);print(sys.argv[1], 'L0', round(d['value']/1e6,2), 'M tx/s', d['matches'])" $lib
done
