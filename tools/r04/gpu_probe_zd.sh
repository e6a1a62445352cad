# Round 4: the streaming kernel alone with every batch published: row blobs
# read per lane (64-byte-strided, CUDASP_STREAM_PF_COAL=0) vs lane-contiguous
# with an LDS transpose (=1) from pinned host memory, vs inputs in device
# memory (measurement build -DCUDASP_AB_STREAM_ANY_MEMORY); then end to end.
set -e
mkdir -p gpurun_out/r04
L=$PWD/build_variants/anymem/libcudasp_amd.so
for pass in 1 2; do
echo pass $pass
CUDASP_STREAM_PF_COAL=0 timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2 > gpurun_out/r04/zd_coal0_$pass.json
CUDASP_STREAM_PF_COAL=1 timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2 > gpurun_out/r04/zd_coal1_$pass.json
CUDASP_LIB=$L timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2 --device-inputs --device-results > gpurun_out/r04/zd_devres_$pass.json
done
E=./tools/host_e2e
for pass in 1 2; do
for c in 0 1; do
  echo e2e $pass $c
  CUDASP_STREAM_PF_COAL=$c timeout -k 10 120 $E --rows 1000000 --threads 8 --batch 300000 --labels 0 --input rows --reps 5 --outputs 2 > gpurun_out/r04/zd_cfg2_${c}_$pass.json
  CUDASP_STREAM_PF_COAL=$c timeout -k 10 120 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 3 --outputs 2 > gpurun_out/r04/zd_cfg3_${c}_$pass.json
done
done
echo done
