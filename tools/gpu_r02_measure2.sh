# Round-2 measurement sweep with the multi-batch launch (bench.py default
# --launch multi): GPU tests + smoke, the default bench line (e2e leg and CPU
# baselines), a rocprofv3 kernel trace of the default bench, PMC passes of
# k_scan_multi (SQ counts for 0 / 1 / 16 labels, FETCH_SIZE / WRITE_SIZE),
# summarised on the box into gpurun_out/, then the default line again with the
# summaries, config-3 / config-5 lines, the per-batch launch line, and a
# 2-rank round-robin rehearsal over gloo.
#   $1: "notests" skips the pytest step
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -30 $O/$name.log; exit 1; }; tail -1 $O/$name.log | cut -c1-300; }
cd $R
if [ "$1" != "notests" ]; then
  step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
fi
cd /tmp && export TMPDIR=/tmp
rm -rf $O/prof_bench $O/pmc_*
B="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-layout-probe"
step prof_bench 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- $B --steps 3 --warmup 1
M="--rows 3000000 --steps 1 --warmup 0 --exclusive-batches 0"
step pmc_sq_L0 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_sq_L0 -o sq -- $B $M
step pmc_grbm 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc_grbm -o grbm -- $B $M
step pmc_sq_L1 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/pmc_sq_L1 -o sq -- $B $M --labels 1
step pmc_sq_L16 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/pmc_sq_L16 -o sq -- $B $M --labels 16 --outputs-max 15
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o fetch -- python3 $R/bench.py --no-cpu-baseline --no-e2e $M
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o write -- python3 $R/bench.py --no-cpu-baseline --no-e2e $M
cd $R
python tools/prof_summary.py $O/prof_bench/bench_kernel_trace.csv --out $O/r02_rocprof_bench_summary.json > /dev/null
SRC="rocprofv3 --pmc of python3 bench.py --rows 3000000 --steps 1 --warmup 0 (one k_scan_multi launch over 10 batches), MI355X"
python tools/pmc_summary.py sq $O/r02_pmc_sq_multi_L0_k2_w26.json $O/pmc_sq_L0/sq_counter_collection.csv $O/pmc_grbm/grbm_counter_collection.csv --multi-rows 3000000 --shape "multi, 0 labels, 2 outputs/row, 26-bit windows" --source "$SRC" > /dev/null
python tools/pmc_summary.py sq $O/r02_pmc_sq_multi_L1_k2_w26.json $O/pmc_sq_L1/sq_counter_collection.csv --multi-rows 3000000 --shape "multi, 1 label, 2 outputs/row, 26-bit windows" --source "$SRC --labels 1" > /dev/null
python tools/pmc_summary.py sq $O/r02_pmc_sq_multi_L16_k1-15_w26.json $O/pmc_sq_L16/sq_counter_collection.csv --multi-rows 3000000 --shape "multi, 16 labels, 1..15 outputs/row, 26-bit windows" --source "$SRC --labels 16 --outputs-max 15" > /dev/null
python tools/pmc_summary.py hbm $O/r02_pmc_hbm_multi.json $O/pmc_fetch/fetch_counter_collection.csv $O/pmc_write/write_counter_collection.csv --multi-rows 3000000 --probe-rows 3000000 --source "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of python3 bench.py --rows 3000000 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e, MI355X" > /dev/null
P="--pmc-summary $O/r02_pmc_hbm_multi.json"
step bench_default 600 python bench.py --steps 5 --warmup 2 $P --pmc-sq $O/r02_pmc_sq_multi_L0_k2_w26.json
step bench_cfg3 400 python bench.py --rows 9400000 --labels 1 --steps 3 $P --pmc-sq $O/r02_pmc_sq_multi_L1_k2_w26.json
step bench_cfg5 700 python bench.py --rows 100000000 --labels 16 --outputs-max 15 --steps 2 --cpu-rows 50000 $P --pmc-sq $O/r02_pmc_sq_multi_L16_k1-15_w26.json --no-e2e
step bench_batches 400 python bench.py --steps 5 --warmup 2 --launch batches --no-e2e --no-cpu-baseline
step bench_2rank_rr 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --dist-backend gloo $P --no-layout-probe
echo all-done
