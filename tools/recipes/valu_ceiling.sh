# The VALU ceiling of k_scan_multi's instruction mix.  PMC passes
# (each its own run, SQ / GRBM blocks within their slot limits) over
#   (a) tools/microbench/int_throughput: issue-bound loops of one opcode each
#       (calibration: what SQ_ACTIVE_INST_VALU reads when the VALU is saturated)
#   (b) the bench's k_scan_multi (one launch over 3M rows, 0 and 16 labels)
# then tools/valu_ceiling.py.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_valu; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -oE "SQ_[A-Z0-9_]+" $O/counters.txt | sort -u > $O/sq_counters.txt; wc -l $O/sq_counters.txt
grep -E "^SQ_(INSTS_VALU|ACTIVE_INST|INST_CYCLES|VALU|BUSY)" $O/sq_counters.txt | tr '\n' ' '; echo
SQ="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_ANY"
MB=$R/tools/microbench/int_throughput
timeout -s KILL 90 rocprofv3 --pmc $SQ --output-format csv -d $O/mb_sq -o sq -- $MB > $O/mb_sq.log 2>&1 || { echo mb_sq failed; tail $O/mb_sq.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/mb_grbm -o grbm -- $MB > $O/mb_grbm.log 2>&1 || { echo mb_grbm failed; tail $O/mb_grbm.log; exit 1; }
timeout -k 10 90 rocprofv3 --kernel-trace --output-format csv -d $O/mb_kt -o kt -- $MB > $O/mb_kt.log 2>&1 || { echo mb_kt failed; exit 1; }
cat $O/mb_kt.log | head -20
B="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-layout-probe --rows 3000000 --steps 1 --warmup 0 --exclusive-batches 0"
for L in 0 16; do
  X=""; [ $L = 16 ] && X="--labels 16 --outputs-max 15"
  timeout -s KILL 300 rocprofv3 --pmc $SQ --output-format csv -d $O/scan_sq_L$L -o sq -- $B $X > $O/scan_sq_L$L.log 2>&1 || { echo scan_sq failed; tail $O/scan_sq_L$L.log; exit 1; }
  timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/scan_grbm_L$L -o grbm -- $B $X > $O/scan_grbm_L$L.log 2>&1 || { echo scan_grbm failed; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/scan_kt_L$L -o kt -- $B $X > $O/scan_kt_L$L.log 2>&1 || { echo scan_kt failed; exit 1; }
done
cd $R && python3 tools/valu_ceiling.py $O > $O/valu_ceiling.txt && cat $O/valu_ceiling.txt
