# rocprofv3 kernel trace of the device-only bench at the N = 8 share of config 4
# (4,087,500 rows per GPU): kernel durations against the bench's HIP events,
# and the gaps between a step's commands.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_profshard; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o shard -- python3 $R/bench.py --rows ${ROWS:-4087500} --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-layout-probe --idle-samples 0 > $O/bench.json 2> $O/bench.err || { echo prof failed; tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-300
