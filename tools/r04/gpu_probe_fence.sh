# Round 4: the streaming kernel alone (all batches published) with and without
# the system-scope release fence before each batch's done word (build
# -DCUDASP_STREAM_RELEASE_FENCE=0), interleaved.
set -e
mkdir -p gpurun_out/r04
L=$PWD/build_variants/nofence/libcudasp_amd.so
for pass in 1 2; do
timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2 > gpurun_out/r04/fe_fence_$pass.json
CUDASP_LIB=$L timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2 > gpurun_out/r04/fe_nofence_$pass.json
done
echo done
