# Round 4: the streaming kernel's wave-rows per piece (CUDASP_MULTI_ROWS 4 / 5
# / 6 = default) end to end at configs 2, 3 and 4, cold and warm queries
# (host_e2e --warm-reps), two interleaved passes.  Round 3 saw +3% at config 2
# for 4 and 5 (profiles/r03_stream_knobs.txt) with the clock ramp unseparated.
set -e
mkdir -p gpurun_out/r04
E=./tools/host_e2e
for pass in 1 2; do
  echo pass $pass
  for r in 6 5 4; do
    CUDASP_MULTI_ROWS=$r timeout -k 10 120 $E --rows 1000000 --threads 8 --batch 300000 --labels 0 --input rows --reps 5 --warm-reps 5 --outputs 2 > gpurun_out/r04/rm${r}_cfg2_$pass.json
    CUDASP_MULTI_ROWS=$r timeout -k 10 120 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 3 --warm-reps 3 --outputs 2 > gpurun_out/r04/rm${r}_cfg3_$pass.json
    CUDASP_MULTI_ROWS=$r timeout -k 10 200 $E --rows 32700000 --threads 8 --batch 300000 --labels 0 --input rows --reps 1 --warm-reps 1 --outputs 2 > gpurun_out/r04/rm${r}_cfg4_$pass.json
  done
done
echo done
