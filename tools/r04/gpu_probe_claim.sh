# Round 4: k_scan_stream's claim sizes (A/B knob CUDASP_STREAM_CLAIM_FLOOR:
# 0 = k_scan_multi's adaptive rule, 2/3/4 = at least that many wave-rows while
# that many per wave are published, 255 = guided rem / waves) at 1M, 3M and
# 9.4M rows, then end to end at configs 2 and 3.
set -e
mkdir -p gpurun_out/r04
E=./tools/host_e2e
for pass in 1 2; do
  echo pass $pass
  for f in 0 2 4 255; do
    for n in 1000000 3000000 9400000; do
      CUDASP_STREAM_CLAIM_FLOOR=$f timeout -k 10 200 python tools/stream_probe.py --rows $n --labels 0 --modes all --reps 2 > gpurun_out/r04/cf${f}_${n}_$pass.json
    done
    CUDASP_STREAM_CLAIM_FLOOR=$f timeout -k 10 120 $E --rows 1000000 --threads 8 --batch 300000 --labels 0 --input rows --reps 5 --outputs 2 > gpurun_out/r04/cf${f}_e2e2_$pass.json
    CUDASP_STREAM_CLAIM_FLOOR=$f timeout -k 10 120 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 3 --outputs 2 > gpurun_out/r04/cf${f}_e2e3_$pass.json
  done
done
echo done
