# Final GPU suite + smoke of the tree (round 3).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03e_suite; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/gpu_tests.log | tail -30; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
