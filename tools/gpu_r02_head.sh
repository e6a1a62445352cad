# Current build on one MI355X: full GPU test suite + smoke, then the default
# bench line (multi launch, e2e leg, CPU baselines) twice.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -30 $O/$name.log; exit 1; }; tail -1 $O/$name.log | cut -c1-250; }
step pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step bench_default 600 python bench.py --steps 5 --warmup 2
step bench_default2 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
echo all-done
