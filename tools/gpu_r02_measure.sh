# Round-2 measurement sweep on one MI355X (each GPU step bounded; stop at the
# first failure): GPU tests + smoke, the default bench line (with its e2e leg),
# a rocprofv3 kernel trace of the default bench, PMC passes per bench shape
# (SQ instruction counts for 0 / 1 / 16 labels; FETCH_SIZE / WRITE_SIZE for the
# default shape), summarised on the box into gpurun_out/, then the config-3 and
# config-5 bench lines and a 2-rank round-robin rehearsal over gloo.
#   $1: "notests" skips the pytest step
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -30 $O/$name.log; exit 1; }; tail -1 $O/$name.log | cut -c1-400; }
cd $R
if [ "$1" != "notests" ]; then
  step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
  step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
fi
step bench_default 500 python bench.py --steps 5 --warmup 2
cd /tmp && export TMPDIR=/tmp
rm -rf $O/prof_bench $O/pmc_*
B="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-layout-probe"
step prof_bench 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- $B --steps 2 --warmup 1
step pmc_sq_L0 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/pmc_sq_L0 -o sq -- $B --rows 3000000 --steps 1 --warmup 0
step pmc_sq_L1 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/pmc_sq_L1 -o sq -- $B --rows 3000000 --labels 1 --steps 1 --warmup 0
step pmc_sq_L16 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/pmc_sq_L16 -o sq -- $B --rows 3000000 --labels 16 --outputs-max 15 --steps 1 --warmup 0
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o fetch -- python3 $R/bench.py --rows 3000000 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o write -- python3 $R/bench.py --rows 3000000 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e
cd $R
python tools/prof_summary.py $O/prof_bench/bench_kernel_trace.csv --out $O/r02_rocprof_bench_summary.json > /dev/null
SRC="rocprofv3 --pmc of python3 bench.py --rows 3000000 --steps 1 --warmup 0 (full 300k-row dispatches, per-dispatch averages), MI355X"
python tools/pmc_summary.py sq $O/r02_pmc_sq_L0_k2_w26.json $O/pmc_sq_L0/sq_counter_collection.csv --shape "0 labels, 2 outputs/row, 26-bit windows" --source "$SRC" > /dev/null
python tools/pmc_summary.py sq $O/r02_pmc_sq_L1_k2_w26.json $O/pmc_sq_L1/sq_counter_collection.csv --shape "1 label, 2 outputs/row, 26-bit windows" --source "$SRC --labels 1" > /dev/null
python tools/pmc_summary.py sq $O/r02_pmc_sq_L16_k1-15_w26.json $O/pmc_sq_L16/sq_counter_collection.csv --shape "16 labels, 1..15 outputs/row, 26-bit windows" --source "$SRC --labels 16 --outputs-max 15" > /dev/null
python tools/pmc_summary.py hbm $O/r02_pmc_hbm_k_shared_secret.json $O/pmc_fetch/fetch_counter_collection.csv $O/pmc_write/write_counter_collection.csv --probe-rows 3000000 --source "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of python3 bench.py --rows 3000000 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e, full 300k-row dispatches, MI355X" > /dev/null
P="--pmc-summary $O/r02_pmc_hbm_k_shared_secret.json"
step bench_default_pmc 500 python bench.py --steps 5 --warmup 2 $P --pmc-sq $O/r02_pmc_sq_L0_k2_w26.json --no-e2e
step bench_cfg3 400 python bench.py --rows 9400000 --labels 1 --steps 3 $P --pmc-sq $O/r02_pmc_sq_L1_k2_w26.json
step bench_cfg5 700 python bench.py --rows 100000000 --labels 16 --outputs-max 15 --steps 2 --cpu-rows 50000 $P --pmc-sq $O/r02_pmc_sq_L16_k1-15_w26.json --no-e2e
step bench_2rank_rr 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --dist-backend gloo $P
echo all-done
