# Usage (on the GPU box): bash tools/gpu_check.sh [tag]
# pytest -m gpu, then stage timings at 300k rows for 0/1/16 labels.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-check}
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for L in 0 1 16; do
  timeout -k 10 120 python tools/quick_timing.py 300000 $L >> gpurun_out/${TAG}_timing.log 2>&1 || { echo "timing failed"; tail -20 gpurun_out/${TAG}_timing.log; exit 1; }
done
grep "rows/s" gpurun_out/${TAG}_timing.log
