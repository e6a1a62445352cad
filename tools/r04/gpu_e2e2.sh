# Round 4: pinned-memory CPU access speeds, then end-to-end configs 2/3 with
# the non-blocking slot ring, and the config-3 trace.
set -e
mkdir -p gpurun_out/r04
timeout -k 10 60 ./tools/microbench/hostmem_read > gpurun_out/r04/hostmem_read.json
E=./tools/host_e2e
timeout -k 10 120 $E --rows 1000000 --threads 8 --batch 300000 --labels 0 --input rows --reps 5 --outputs 2 > gpurun_out/r04/e2e2_cfg2.json
timeout -k 10 120 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 3 --outputs 2 > gpurun_out/r04/e2e2_cfg3.json
rm -f gpurun_out/r04/tr_cfg*.bin
export LD_LIBRARY_PATH=$PWD/build_variants/strace:$LD_LIBRARY_PATH
CUDASP_STREAM_TRACE_FILE=gpurun_out/r04/tr_cfg3.bin timeout -k 10 150 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 1 --outputs 2 > gpurun_out/r04/tr_cfg3.json
echo done
