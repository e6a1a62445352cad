# Round 3: the ladder-mix ceiling -- PMC passes over tools/microbench/group_ops
# (the kernel's doubling / mixed addition / mul / sqr in register-resident
# loops at 1-4 waves per SIMD) and the INT32 / INT64 split of k_scan_multi;
# appended to the r03_valu directory of gpu_valu_ceiling.sh.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_valu; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
GO=$R/tools/microbench/group_ops
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAVE_CYCLES SQ_WAVES"
timeout -k 10 120 $GO > $O/group_ops.txt 2>&1 || { echo group_ops failed; tail $O/group_ops.txt; exit 1; }
cat $O/group_ops.txt
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/go_sq -o sq -- $GO > $O/go_sq.log 2>&1 || { echo go_sq failed; tail $O/go_sq.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/go_grbm -o grbm -- $GO > $O/go_grbm.log 2>&1 || { echo go_grbm failed; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/go_kt -o kt -- $GO > $O/go_kt.log 2>&1 || { echo go_kt failed; exit 1; }
B="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-layout-probe --rows 3000000 --steps 1 --warmup 0 --exclusive-batches 0"
timeout -s KILL 300 rocprofv3 --pmc $SQ --output-format csv -d $O/scan_int_L0 -o sq -- $B > $O/scan_int_L0.log 2>&1 || { echo scan_int failed; tail $O/scan_int_L0.log; exit 1; }
cd $R && python3 tools/valu_ceiling.py $O --json $O/valu_ceiling.json > $O/valu_ceiling.txt && cat $O/valu_ceiling.txt
