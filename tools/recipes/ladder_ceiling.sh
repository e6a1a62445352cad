# The ladder-mix issue ceiling alone (the group-op loops of
# tools/microbench/group_ops, now with the Yh-form doubling and addition that
# k_scan_multi's stage-A ladder runs): SQ, GRBM and kernel-trace passes, each
# its own run.  tools/valu_ceiling.py then combines them with the scan passes
# of tools/recipes/pmc.sh (same directory layout).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r06}_go; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
GO=$R/tools/microbench/group_ops
P() { name=$1; shift; timeout -s KILL 120 rocprofv3 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }; echo "$name ok"; }
P go_sq --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_ANY --output-format csv -d $O/go_sq -o sq -- $GO
P go_grbm --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/go_grbm -o grbm -- $GO
P go_kt --kernel-trace --output-format csv -d $O/go_kt -o kt -- $GO
echo go-done
