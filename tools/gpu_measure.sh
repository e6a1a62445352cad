# Full measurement sweep on one MI355X (each GPU step bounded; stop at the first
# failure): GPU tests + smoke, rocprofv3 kernel trace and PMC counters of the
# current build (summarised on the box into gpurun_out/), then the bench lines
# (default, config-3 and config-5 shapes, 2 ranks over gloo) reading those
# fresh summaries.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -30 $O/$name.log; exit 1; }; tail -1 $O/$name.log | cut -c1-300; }
cd $R
step pytest 600 python -m pytest tests -m gpu -x -q
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
cd /tmp && export TMPDIR=/tmp
rm -rf $O/prof_bench $O/pmc_sq $O/pmc_sq2 $O/pmc_fetch $O/pmc_write
step prof_bench 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 $R/bench.py --steps 2 --no-cpu-baseline
step pmc_sq 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_sq -o sq -- python3 $R/tools/quick_timing.py 300000 0
step pmc_sq2 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv -d $O/pmc_sq2 -o sq2 -- python3 $R/tools/quick_timing.py 300000 0
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o fetch -- python3 $R/bench.py --rows 3000000 --steps 1 --warmup 0 --no-cpu-baseline
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o write -- python3 $R/bench.py --rows 3000000 --steps 1 --warmup 0 --no-cpu-baseline
cd $R
python tools/prof_summary.py $O/prof_bench/bench_kernel_trace.csv --out $O/rocprof_bench_summary.json > /dev/null
python tools/pmc_summary.py sq $O/pmc_sq_counters.json $O/pmc_sq/sq_counter_collection.csv $O/pmc_sq2/sq2_counter_collection.csv --source "rocprofv3 --pmc (two passes) of python3 tools/quick_timing.py 300000 0 (0 labels, 2 outputs/row), per-dispatch averages over full 300k-row dispatches, MI355X" > /dev/null
python tools/pmc_summary.py hbm $O/pmc_k_shared_secret.json $O/pmc_fetch/fetch_counter_collection.csv $O/pmc_write/write_counter_collection.csv --probe-rows 3000000 --source "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of python3 bench.py --rows 3000000 --steps 1 --warmup 0 --no-cpu-baseline, full 300k-row dispatches, MI355X" > /dev/null
P="--pmc-sq $O/pmc_sq_counters.json --pmc-summary $O/pmc_k_shared_secret.json"
step bench_default 400 python bench.py $P
step bench_cfg3 400 python bench.py --rows 9400000 --labels 1 --steps 3 $P
step bench_cfg5 600 python bench.py --rows 100000000 --labels 16 --outputs-max 15 --steps 2 --cpu-rows 50000 $P
step bench_2rank_gloo 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --rows 3000000 --steps 2 --dist-backend gloo $P
echo all-done
