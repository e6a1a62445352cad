set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_quick; mkdir -p $O; cd $R
timeout -k 10 600 python -u bench.py --rows 3000000 --labels 16 --outputs-max 15 --steps 2 --warmup 1 --cpu-rows 50000 --no-e2e > $O/q16.json 2> $O/q16.err || { tail -20 $O/q16.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/q16.json').read().strip().splitlines()[-1]); print(d['value']/1e6, d['planted_oracle_check'], d['cpu_baseline']['flags_match_gpu'], d['matches'])"
