# Round 4: DMA staging of streamed batches (cudasp_stream_batch.d_*,
# CUDASP_TF_STAGE) -- tests, then the kernel alone with every batch published
# (zero copy vs staged vs device memory in place), then end to end A/B.
set -e
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_stream_gpu.py tests/test_host_feeds_gpu.py tests/test_host_stream_gpu.py > gpurun_out/r04/gpu_tests_stage.log 2>&1
L=$PWD/build_variants/anymem/libcudasp_amd.so
timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2 > gpurun_out/r04/st_probe_zero.json
timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all,paced --reps 2 --staged > gpurun_out/r04/st_probe_staged.json
CUDASP_LIB=$L timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2 --device-inputs --device-results > gpurun_out/r04/st_probe_devres.json
E=./tools/host_e2e
for pass in 1 2; do
for sg in 0 1; do
  CUDASP_TF_STAGE=$sg timeout -k 10 120 $E --rows 1000000 --threads 8 --batch 300000 --labels 0 --input rows --reps 5 --outputs 2 > gpurun_out/r04/st_cfg2_${sg}_$pass.json
  CUDASP_TF_STAGE=$sg timeout -k 10 120 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 3 --outputs 2 > gpurun_out/r04/st_cfg3_${sg}_$pass.json
done
done
for sg in 0 1; do
  CUDASP_TF_STAGE=$sg timeout -k 10 200 $E --rows 32700000 --threads 8 --batch 300000 --labels 0 --input rows --reps 1 --outputs 2 > gpurun_out/r04/st_cfg4_${sg}.json
done
echo done
