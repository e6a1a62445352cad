# GPU tests (all, or the files given as arguments) + smoke, on the GPU box.
#   MEASURE_TAG names the output directory (gpurun_out/<tag>_tests).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_tests; mkdir -p $O; cd $R
T="${@:-tests}"
timeout -k 10 1000 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/gpu_tests.log | tail -30; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
if [ $# -eq 0 ]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
