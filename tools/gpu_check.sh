# GPU tests (one process, per-test time limit), then a short bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/check_pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/check_pytest.log | tail -30; tail -30 $O/check_pytest.log; exit 1; }
tail -1 $O/check_pytest.log
timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline > $O/check_bench.log 2>&1 || { tail -20 $O/check_bench.log; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/check_bench.log').read().strip().splitlines()[-1]); print(d['value']/1e6, d['matches'])"
