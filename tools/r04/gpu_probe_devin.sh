# Round 4: k_scan_stream with every batch published at once, inputs from
# pinned host memory (zero copy) vs device memory (measurement build
# -DCUDASP_AB_STREAM_ANY_MEMORY), match rows to host vs device memory; two passes.
set -e
mkdir -p gpurun_out/r04
L=$PWD/build_variants/anymem/libcudasp_amd.so
for pass in 1 2; do
CUDASP_LIB=$L timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2 > gpurun_out/r04/devin_host_$pass.json
CUDASP_LIB=$L timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2 --device-inputs > gpurun_out/r04/devin_dev_$pass.json
CUDASP_LIB=$L timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2 --device-inputs --device-results > gpurun_out/r04/devin_devres_$pass.json
done
echo done
