# Bench (default workload) at several stream counts, 2 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for round in 1 2; do
for S in 3 4 5 6 8; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-layout-probe --steps 6 --streams $S > $O/bench_streams.log 2>&1 || { tail -5 $O/bench_streams.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('$O/bench_streams.log').read().strip().splitlines()[-1]);print('streams', sys.argv[1], round(d['value']/1e6,2), 'M tx/s', d['matches']['found'])" $S
done
done
