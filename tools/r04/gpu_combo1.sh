# Round 4: the streaming-scan GPU tests (with the idle-exit race test), then
# the wave-rows-per-piece A/B (tools/r04/gpu_rmax_ab.sh).
set -e
mkdir -p gpurun_out/r04
timeout -k 10 300 python -u -m pytest tests/test_stream_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04/t_stream.log 2>&1
bash tools/r04/gpu_rmax_ab.sh
