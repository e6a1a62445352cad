# GPU test suite + smoke (one process each, per-test limit).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_suite; mkdir -p $O; cd $R
K=(); [ -n "$1" ] && K=(-k "$1")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $O/gpu_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/gpu_tests.log | tail -30; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
