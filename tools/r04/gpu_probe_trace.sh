# Round 4: event trace of k_scan_stream with every batch published at once
# (tools/stream_probe.py --modes all), to compare with k_scan_multi's time.
set -e
mkdir -p gpurun_out/r04
rm -f gpurun_out/r04/tr_probe.bin
CUDASP_LIB=$PWD/build_variants/strace/libcudasp_amd.so CUDASP_STREAM_TRACE_FILE=gpurun_out/r04/tr_probe.bin timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 1 > gpurun_out/r04/tr_probe.json
echo done
