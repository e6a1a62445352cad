# Round 4: wave priority by piece age at equal clocks (--prewarm): the
# streaming kernel alone with CUDASP_STREAM_PRIO_US 0 / 3000 (default) /
# 10000 at 3M and 9.4M rows, and end to end at config 3, two passes.
set -e
mkdir -p gpurun_out/r04
E=./tools/host_e2e
for pass in 1 2; do
  for p in 3000 0 10000; do
    for n in 3000000 9400000; do
      CUDASP_STREAM_PRIO_US=$p timeout -k 10 200 python tools/stream_probe.py --rows $n --labels 0 --modes all --reps 3 --prewarm > gpurun_out/r04/pq_${p}_${n}_$pass.json
    done
    CUDASP_STREAM_PRIO_US=$p timeout -k 10 120 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 3 --warm-reps 3 --outputs 2 > gpurun_out/r04/pq_${p}_e2e3_$pass.json
  done
done
echo done
