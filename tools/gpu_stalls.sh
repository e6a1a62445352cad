# Wave-state counters at full occupancy (3M-row launches): where stage A's
# wave cycles go (issue vs waits), plus the kernel trace for durations.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
rm -rf $O/stall
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_WAVES --kernel-trace --output-format csv -d $O/stall -o st -- python3 $R/tools/stage_timing.py 3000000 0 3 > $O/stall.log 2>&1 || { tail -20 $O/stall.log; exit 1; }
ls $O/stall
