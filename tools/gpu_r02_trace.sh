# Kernel traces of one rank's share of N = 8 (4.2M rows, 14 batches) under
# several launch schedules, for tools/timeline.py (fill / drain analysis).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-layout-probe --exclusive-batches 0 --rows 4200000 --steps 3 --warmup 1"
run() { local name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$name -o kt -- "$@" > $O/tr_$name.log 2>&1 || { echo $name failed; tail $O/tr_$name.log; exit 1; }; python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['value']/1e6,1), round(d['ms_per_step'],2))" $O/tr_$name.log $name; }
run base $B
run tail_a1b2 $B --tail-rows-a 1 --tail-rows-b 2
run s8 $B --streams 8
CUDASP_ROWS_A_FORCE=2 run ra2 $B
run s2 $B --streams 2
