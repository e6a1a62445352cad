# Round 4: the prefetch in one round trip per piece (CUDASP_STREAM_PF_GROUP=1,
# all wave-rows' loads together, outputs copied in 16-byte pieces) against the
# groups of 3 (=0): kernel alone with every batch published (config 3 and the
# config-5 output shape), then end-to-end configs 2/3; interleaved, two passes.
set -e
mkdir -p gpurun_out/r04
E=./tools/host_e2e
for pass in 1 2; do
  echo pass $pass
  for g in 0 1; do
    CUDASP_STREAM_PF_GROUP=$g timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2 > gpurun_out/r04/pf${g}_cfg3_$pass.json
    CUDASP_STREAM_PF_GROUP=$g timeout -k 10 200 python tools/stream_probe.py --rows 3000000 --labels 16 --kmax 15 --modes all --reps 2 > gpurun_out/r04/pf${g}_k15_$pass.json
    CUDASP_STREAM_PF_GROUP=$g timeout -k 10 120 $E --rows 1000000 --threads 8 --batch 300000 --labels 0 --input rows --reps 5 --outputs 2 > gpurun_out/r04/pf${g}_e2e2_$pass.json
    CUDASP_STREAM_PF_GROUP=$g timeout -k 10 120 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 3 --outputs 2 > gpurun_out/r04/pf${g}_e2e3_$pass.json
  done
done
echo done
