# Round 4: k_scan_stream event traces (measurement build, -DCUDASP_STREAM_TRACE=1)
# of the table-function host at configs 2 and 3; analysed by tools/stream_trace.py.
set -e
mkdir -p gpurun_out/r04
rm -f gpurun_out/r04/tr_cfg*.bin
export LD_LIBRARY_PATH=$PWD/build_variants/strace:$LD_LIBRARY_PATH
CUDASP_STREAM_TRACE_FILE=gpurun_out/r04/tr_cfg2.bin timeout -k 10 150 ./tools/host_e2e --rows 1000000 --threads 8 --batch 300000 --labels 0 --input rows --reps 2 --outputs 2 > gpurun_out/r04/tr_cfg2.json
CUDASP_STREAM_TRACE_FILE=gpurun_out/r04/tr_cfg3.bin timeout -k 10 150 ./tools/host_e2e --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 1 --outputs 2 > gpurun_out/r04/tr_cfg3.json
echo done
