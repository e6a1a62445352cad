# GPU tests only (one process, per-test time limit). Optional: a -k filter as $1.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
K=(); [ -n "$1" ] && K=(-k "$1")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $O/tests_only.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/tests_only.log | tail -30; tail -40 $O/tests_only.log; exit 1; }
tail -1 $O/tests_only.log
