# Bench (default workload, more steps) with each build_variants/*.so, 2 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for round in 1 2; do
for lib in build_variants/*.so; do
  CUDASP_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${AB_STEPS:-8} > gpurun_out/bench_ab.log 2>&1 || { tail -5 gpurun_out/bench_ab.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/bench_ab.log').read().strip().splitlines()[-1]);print(sys.argv[1], round(d['value']/1e6,2), 'M tx/s', d['matches']['found'])" $lib
done
done
