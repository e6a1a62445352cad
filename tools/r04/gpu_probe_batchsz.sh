# Round 4: per-batch costs of the streaming kernel?  The same rows in 300k-row
# batches and in one batch, equal clocks (--prewarm), 1M and 3M rows.
set -e
mkdir -p gpurun_out/r04
for pass in 1 2; do
  for n in 1000000 3000000; do
    for b in 300000 $n; do
      timeout -k 10 200 python tools/stream_probe.py --rows $n --batch $b --labels 0 --modes all --reps 3 --prewarm > gpurun_out/r04/bs_${n}_${b}_$pass.json
    done
  done
done
echo done
