# PMC passes of the bench's k_scan_multi (each counter set its own
# run): SQ instruction counts at 0 / 1 / 16 labels, GRBM cycles, FETCH_SIZE and
# WRITE_SIZE (HBM traffic, with the layout probe as calibration), summarised
# into the JSON files bench.py reads.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_pmc; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-layout-probe --rows 3000000 --steps 1 --warmup 0 --exclusive-batches 0"
P() { name=$1; shift; timeout -s KILL 300 rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }; }
P sq_L0 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/sq_L0 -o sq -- $B
P grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/grbm -o grbm -- $B
P sq_L1 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/sq_L1 -o sq -- $B --labels 1
P sq_L16 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $O/sq_L16 -o sq -- $B --labels 16 --outputs-max 15
P fetch --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- python3 $R/bench.py --no-cpu-baseline --no-e2e --rows 3000000 --steps 1 --warmup 0 --exclusive-batches 0
P write --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- python3 $R/bench.py --no-cpu-baseline --no-e2e --rows 3000000 --steps 1 --warmup 0 --exclusive-batches 0
cd $R
SRC="rocprofv3 --pmc of python3 bench.py --rows 3000000 --steps 1 --warmup 0 (one k_scan_multi launch over 10 batches), MI355X"
python3 tools/pmc_summary.py sq $O/${MEASURE_TAG:-r05}_pmc_sq_multi_L0_k2_w26.json $O/sq_L0/sq_counter_collection.csv $O/grbm/grbm_counter_collection.csv --multi-rows 3000000 --shape "multi, 0 labels, 2 outputs/row, 26-bit windows" --source "$SRC" > /dev/null
python3 tools/pmc_summary.py sq $O/${MEASURE_TAG:-r05}_pmc_sq_multi_L1_k2_w26.json $O/sq_L1/sq_counter_collection.csv --multi-rows 3000000 --shape "multi, 1 label, 2 outputs/row, 26-bit windows" --source "$SRC --labels 1" > /dev/null
python3 tools/pmc_summary.py sq $O/${MEASURE_TAG:-r05}_pmc_sq_multi_L16_k1-15_w26.json $O/sq_L16/sq_counter_collection.csv --multi-rows 3000000 --shape "multi, 16 labels, 1..15 outputs/row, 26-bit windows" --source "$SRC --labels 16 --outputs-max 15" > /dev/null
python3 tools/pmc_summary.py hbm $O/${MEASURE_TAG:-r05}_pmc_hbm_multi.json $O/fetch/fetch_counter_collection.csv $O/write/write_counter_collection.csv --multi-rows 3000000 --probe-rows 3000000 --source "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of python3 bench.py --rows 3000000 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e, MI355X" | head -20
