# Round 4: is k_scan_stream's excess over k_scan_multi per row or per query?
# The same probe (every batch published at once) at four table sizes, no labels
# and 16 labels with 1..15 outputs.
set -e
mkdir -p gpurun_out/r04
for n in 1000000 3000000 9400000 32700000; do
  timeout -k 10 200 python tools/stream_probe.py --rows $n --labels 0 --modes all --reps 2 > gpurun_out/r04/sz_l0_$n.json
done
for n in 1000000 3000000 12000000; do
  timeout -k 10 200 python tools/stream_probe.py --rows $n --labels 16 --kmax 15 --modes all --reps 2 > gpurun_out/r04/sz_l16_$n.json
done
echo done
