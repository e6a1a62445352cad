set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --rows 3000000 --steps 2 > gpurun_out/bench_small.log 2>&1 || { echo "bench small failed"; tail -30 gpurun_out/bench_small.log; exit 1; }
tail -2 gpurun_out/bench_small.log
timeout -k 10 500 python bench.py > gpurun_out/bench_full.log 2>&1 || { echo "bench full failed"; tail -30 gpurun_out/bench_full.log; exit 1; }
tail -2 gpurun_out/bench_full.log
