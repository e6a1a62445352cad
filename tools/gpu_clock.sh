# Effective shader clock during the scan kernels: GRBM_GUI_ACTIVE per dispatch
# against the dispatch duration (rocprofv3 --pmc with --kernel-trace only).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
rm -rf $O/clk
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $O/clk -o clk -- python3 $R/tools/stage_timing.py 3000000 0 3 > $O/clk.log 2>&1 || { tail -20 $O/clk.log; exit 1; }
ls $O/clk
