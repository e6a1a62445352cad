# Round 4: is part of k_scan_stream's excess the GPU clock ramping up after
# idle?  The probe as before, then with 100 ms of idle before every timed run
# of either kernel, then with k_scan_multi run right before every streaming
# run (warm clock).  1M, 3M and 9.4M rows.
set -e
mkdir -p gpurun_out/r04
for n in 1000000 3000000 9400000; do
  timeout -k 10 200 python tools/stream_probe.py --rows $n --labels 0 --modes all --reps 3 > gpurun_out/r04/wm_base_$n.json
  timeout -k 10 200 python tools/stream_probe.py --rows $n --labels 0 --modes all --reps 3 --gap-ms 100 > gpurun_out/r04/wm_gap_$n.json
  timeout -k 10 200 python tools/stream_probe.py --rows $n --labels 0 --modes all --reps 3 --prewarm > gpurun_out/r04/wm_pre_$n.json
done
echo done
