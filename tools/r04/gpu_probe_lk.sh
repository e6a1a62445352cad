# Round 4: the streaming kernel alone (all batches published) after dropping
# the per-wave-row batch lookups and counting completions per run of
# wave-rows; then configs 2 and 3 end to end.
set -e
mkdir -p gpurun_out/r04
for pass in 1 2; do
timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2 > gpurun_out/r04/lk_probe_$pass.json
timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 0 --modes all --reps 2 > gpurun_out/r04/lk_probe0_$pass.json
done
E=./tools/host_e2e
for pass in 1 2; do
  timeout -k 10 120 $E --rows 1000000 --threads 8 --batch 300000 --labels 0 --input rows --reps 5 --outputs 2 > gpurun_out/r04/lk_cfg2_$pass.json
  timeout -k 10 120 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 3 --outputs 2 > gpurun_out/r04/lk_cfg3_$pass.json
done
echo done
