# Round 4: is the streaming kernel's fixed cost on small tables the zero-copy
# start (every wave's first piece read over PCIe at once)?  Inputs in host
# memory vs in device memory (--device-inputs; measurement build that accepts
# device pointers), equal clocks (--prewarm), 1M and 3M rows, two passes.
set -e
mkdir -p gpurun_out/r04
L=$PWD/build_variants/anymem/libcudasp_amd.so
for pass in 1 2; do
  for n in 1000000 3000000; do
    CUDASP_LIB=$L timeout -k 10 200 python tools/stream_probe.py --rows $n --labels 0 --modes all --reps 3 --prewarm > gpurun_out/r04/di_host_${n}_$pass.json
    CUDASP_LIB=$L timeout -k 10 200 python tools/stream_probe.py --rows $n --labels 0 --modes all --reps 3 --prewarm --device-inputs > gpurun_out/r04/di_dev_${n}_$pass.json
  done
done
echo done
