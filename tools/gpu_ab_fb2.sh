# Fixed-base window width A/B: scanner creation (table build) time, isolated
# stage timing and the bench, per build_variants/*.so, 2 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for lib in build_variants/*.so; do
  CUDASP_LIB=$R/$lib timeout -k 10 200 python tools/quick_timing.py 300000 0 > $O/qt.log 2>&1 || exit 1; echo "$lib $(grep -a "scanner create" $O/qt.log)"
done
for round in 1 2; do
for lib in build_variants/*.so; do
  CUDASP_LIB=$R/$lib timeout -k 10 200 python tools/stage_timing.py 3000000 0 5 2>&1 | tail -1 || exit 1
  CUDASP_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-layout-probe --steps 6 > $O/bench_ab.log 2>&1 || { tail -5 $O/bench_ab.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('$O/bench_ab.log').read().strip().splitlines()[-1]);print(sys.argv[1], round(d['value']/1e6,2), 'M tx/s', d['matches']['found'], d['setup_s'])" $lib
done
done
