# Round 3: kernel + copy trace of the device-feed host at config 3 / 2 / 4
# (tools/timeline.py: fill, drain, concurrent dispatches).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_e2e_trace; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
tr() { name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/$name -o t -- $R/tools/host_e2e "$@" > $O/$name.log 2>&1 || { echo trace $name failed; tail $O/$name.log; exit 1; }
  K=$(ls $O/$name/*kernel_trace.csv $O/$name/*/*kernel_trace.csv 2>/dev/null | head -1)
  C=$(ls $O/$name/*memory_copy_trace.csv $O/$name/*/*memory_copy_trace.csv 2>/dev/null | head -1)
  python3 $R/tools/timeline.py "$K" --copies "$C" > $O/$name.txt && tail -12 $O/$name.txt; tail -1 $O/$name.log | cut -c1-300; }
tr cfg3 --rows 9400000 --labels 1 --reps 2
tr cfg2 --rows 1000000 --reps 3
