# PMC passes of THIS tree's k_scan_multi<26,true> (the bench's timed kernel),
# each counter set its own run, at the configs' shapes:
#   config 4 (32.7M rows, 0 labels, 2 outputs/row): SQ counts, GRBM cycles, a
#     kernel trace (clock), FETCH_SIZE and WRITE_SIZE (with k_layout_probe as
#     the calibration of the same access width);
#   config 3 (9.4M rows, 1 label) and the config-5 shape (3M rows, 16 labels,
#     1..15 outputs): SQ counts, GRBM cycles, kernel trace;
#   the ladder-mix ceiling: the group-op and one-opcode loops (tools/microbench).
# Summaries are stamped with the kernels' machine-code hash (tools/codeobj.py):
# bench.py reads a summary only while the loaded kernel has the same stamp.
# Needs tools/microbench/{group_ops,int_throughput} built on the CPU first:
#   (cd tools/microbench && hipcc -O3 -std=c++17 --offload-arch=gfx950 -o group_ops group_ops.hip
#    && hipcc -O3 --offload-arch=gfx950 -o int_throughput int_throughput.hip)
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=${MEASURE_TAG:-r06}; O=$R/gpurun_out/${TAG}_pmc; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
LIB=$R/duckdb-cudasp-extension_amd/libcudasp_amd.so
C="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-pinned --idle-samples 0 --steps 1 --warmup 0 --exclusive-batches 0"
P() { name=$1; shift; timeout -s KILL 240 rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }; echo "$name ok"; }
SQ="SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY"
shape() { case $1 in 0) echo "--rows 32700000";; 1) echo "--rows 9400000 --labels 1";; 16) echo "--rows 3000000 --labels 16 --outputs-max 15";; esac; }
for L in 0 1 16; do
  X="$(shape $L) --no-layout-probe"
  P scan_sq_L$L --pmc $SQ --output-format csv -d $O/scan_sq_L$L -o sq -- $C $X
  P scan_grbm_L$L --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/scan_grbm_L$L -o grbm -- $C $X
  P scan_kt_L$L --kernel-trace --output-format csv -d $O/scan_kt_L$L -o kt -- $C $X
done
P fetch --pmc FETCH_SIZE --output-format csv -d $O/fetch -o fetch -- $C --rows 32700000
P write --pmc WRITE_SIZE --output-format csv -d $O/write -o write -- $C --rows 32700000
MB=$R/tools/microbench/int_throughput; GO=$R/tools/microbench/group_ops
P mb_sq --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_ANY --output-format csv -d $O/mb_sq -o sq -- $MB
P mb_grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/mb_grbm -o grbm -- $MB
P mb_kt --kernel-trace --output-format csv -d $O/mb_kt -o kt -- $MB
P go_sq --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_ANY --output-format csv -d $O/go_sq -o sq -- $GO
P go_grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/go_grbm -o grbm -- $GO
P go_kt --kernel-trace --output-format csv -d $O/go_kt -o kt -- $GO
cd $R
S="--stamp-lib $LIB --stamp k_scan_multi=^_Z12k_scan_multiILi26ELb1EE"
f() { ls $1/*$2 $1/*/*$2 2>/dev/null | head -1; }
SRC="rocprofv3 --pmc (one counter set per run) of python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e (one k_scan_multi launch), MI355X"
python3 tools/pmc_summary.py sq $O/${TAG}_pmc_sq_multi_L0_k2_w26.json $(f $O/scan_sq_L0 counter_collection.csv) $(f $O/scan_grbm_L0 counter_collection.csv) --multi-rows 32700000 --shape "multi, 0 labels, 2 outputs/row, 26-bit windows, config 4 (32.7M rows)" --source "$SRC --rows 32700000" $S > $O/sum_L0.txt
python3 tools/pmc_summary.py sq $O/${TAG}_pmc_sq_multi_L1_k2_w26.json $(f $O/scan_sq_L1 counter_collection.csv) $(f $O/scan_grbm_L1 counter_collection.csv) --multi-rows 9400000 --shape "multi, 1 label, 2 outputs/row, 26-bit windows, config 3 (9.4M rows)" --source "$SRC --rows 9400000 --labels 1" $S > $O/sum_L1.txt
python3 tools/pmc_summary.py sq $O/${TAG}_pmc_sq_multi_L16_k1-15_w26.json $(f $O/scan_sq_L16 counter_collection.csv) $(f $O/scan_grbm_L16 counter_collection.csv) --multi-rows 3000000 --shape "multi, 16 labels, 1..15 outputs/row, 26-bit windows, config-5 shape (3M rows)" --source "$SRC --rows 3000000 --labels 16 --outputs-max 15" $S > $O/sum_L16.txt
python3 tools/pmc_summary.py hbm $O/${TAG}_pmc_hbm_multi.json $(f $O/fetch counter_collection.csv) $(f $O/write counter_collection.csv) --multi-rows 32700000 --probe-rows 32700000 --source "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of python3 bench.py --rows 32700000 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e, MI355X" $S --stamp k_layout_probe=^_Z14k_layout_probe > $O/sum_hbm.txt
python3 tools/valu_ceiling.py $O --json $O/${TAG}_valu_ceiling.json --stamp-lib $LIB > $O/valu_ceiling.txt
cat $O/sum_hbm.txt | head -30; cat $O/valu_ceiling.txt
echo pmc-done
