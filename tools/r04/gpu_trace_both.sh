# Round 4: where the streaming kernel's fixed ~1.3 ms over k_scan_multi goes:
# per-wave start/end of k_scan_multi (CUDASP_MULTI_TRACE) and the event trace
# of k_scan_stream (CUDASP_STREAM_TRACE) on the same 3M rows, equal clocks.
set -e
mkdir -p gpurun_out/r04
L=$PWD/build_variants/trace/libcudasp_amd.so
CUDASP_LIB=$L timeout -k 10 200 python tools/multi_trace.py --rows 3000000 > gpurun_out/r04/tb_multi_3m.json
rm -f gpurun_out/r04/tb_stream_3m.bin
CUDASP_LIB=$L CUDASP_STREAM_TRACE_FILE=gpurun_out/r04/tb_stream_3m.bin timeout -k 10 200 python tools/stream_probe.py --rows 3000000 --labels 0 --modes all --reps 1 --prewarm > gpurun_out/r04/tb_stream_3m.json
echo done
