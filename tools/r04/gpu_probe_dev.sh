# Round 4: the streaming kernel alone, inputs and results in device memory
# (measurement build -DCUDASP_AB_STREAM_ANY_MEMORY), vs the same build reading
# pinned host memory.
set -e
mkdir -p gpurun_out/r04
L=$PWD/build_variants/anymem/libcudasp_amd.so
CUDASP_LIB=$L timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2 > gpurun_out/r04/zd_anyzero.json 2> gpurun_out/r04/zd_anyzero.err
CUDASP_LIB=$L timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2 --device-inputs > gpurun_out/r04/zd_devin.json 2> gpurun_out/r04/zd_devin.err
CUDASP_LIB=$L timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2 --device-inputs --device-results > gpurun_out/r04/zd_devres.json 2> gpurun_out/r04/zd_devres.err
echo done
