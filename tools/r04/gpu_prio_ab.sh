# Round 4: wave priority by piece age (CUDASP_STREAM_PRIO_US) A/B at configs
# 2 and 3 end to end, the streaming kernel alone (stream_probe, all batches
# published), and a config-3 trace with priorities on.
set -e
mkdir -p gpurun_out/r04
E=./tools/host_e2e
for pass in 1 2; do
for p in 0 300 1000 3000; do
  CUDASP_STREAM_PRIO_US=$p timeout -k 10 120 $E --rows 1000000 --threads 8 --batch 300000 --labels 0 --input rows --reps 5 --outputs 2 > gpurun_out/r04/prio_cfg2_${p}_$pass.json
  CUDASP_STREAM_PRIO_US=$p timeout -k 10 120 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 3 --outputs 2 > gpurun_out/r04/prio_cfg3_${p}_$pass.json
done
done
for p in 0 1000; do
  CUDASP_STREAM_PRIO_US=$p timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 > gpurun_out/r04/prio_probe_$p.json
done
rm -f gpurun_out/r04/tr_cfg*.bin
export LD_LIBRARY_PATH=$PWD/build_variants/strace:$LD_LIBRARY_PATH
CUDASP_STREAM_PRIO_US=1000 CUDASP_STREAM_TRACE_FILE=gpurun_out/r04/tr_cfg3.bin timeout -k 10 150 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 1 --outputs 2 > gpurun_out/r04/tr_cfg3.json
echo done
