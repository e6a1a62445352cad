# Shader clock under stage A: product build vs the table-alias A/B build
# (rocprofv3 --pmc GRBM_GUI_ACTIVE per dispatch / kernel duration), to tell
# whether the scratch traffic costs issue time (latency) or clock (power).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -30 $O/$name.log; exit 1; }; tail -1 $O/$name.log | cut -c1-200; }
cd /tmp && export TMPDIR=/tmp
for v in base aliasTab base aliasTab; do
  rm -rf $O/clk_$v
  CUDASP_LIB=$R/build_variants/libcudasp_$v.so step clk_$v 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --kernel-trace --output-format csv -d $O/clk_$v -o c -- python3 $R/tools/stage_timing.py 3000000 0 5
done
echo all-done
