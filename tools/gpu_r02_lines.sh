# Bench lines of the current build with the committed PMC summaries
# (profiles/r02_pmc_*): rocprofv3 kernel trace of the default bench, then the
# default line (e2e leg, CPU baselines), config-3 / config-5 lines, the
# per-batch launch line and a 2-rank round-robin rehearsal over gloo -- all on
# one box, so the lines and the trace share its clock.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -30 $O/$name.log; exit 1; }; tail -1 $O/$name.log | cut -c1-200; }
cd /tmp && export TMPDIR=/tmp
rm -rf $O/prof_bench
step prof_bench 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-layout-probe --steps 3 --warmup 1
cd $R
python tools/prof_summary.py $O/prof_bench/bench_kernel_trace.csv --out $O/r02_rocprof_bench_summary.json > /dev/null
step bench_default 600 python bench.py --steps 5 --warmup 2
step bench_cfg3 400 python bench.py --rows 9400000 --labels 1 --steps 3
step bench_cfg5 700 python bench.py --rows 100000000 --labels 16 --outputs-max 15 --steps 2 --cpu-rows 50000 --no-e2e
step bench_batches 400 python bench.py --steps 5 --warmup 2 --launch batches --no-e2e --no-cpu-baseline
step bench_2rank_rr 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --dist-backend gloo --no-layout-probe
echo all-done
