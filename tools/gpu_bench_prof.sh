set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
step() { local name=$1; shift; timeout -k 10 "$@" > $R/gpurun_out/$name.log 2>&1 || { echo "$name failed"; tail -30 $R/gpurun_out/$name.log; exit 1; }; tail -1 $R/gpurun_out/$name.log | cut -c1-1500; }
step bench_default 400 python bench.py
cd /tmp && export TMPDIR=/tmp
step prof_bench 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o bench -- python3 $R/bench.py
echo all-done
