# Round 3: batch ramp of the device feeds (CUDASP_TF_RAMP: first slots close at
# batch_size / 8, / 4, / 2) A/B, interleaved on one box, configs 2 / 3 / 4.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_ramp; mkdir -p $O; cd $R
e2e() { name=$1; shift; timeout -k 10 300 tools/host_e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "e2e $name failed"; tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.load(open('$O/$name.json')); print('$name', round(d['tx_per_s']/1e6,1), d['seconds_all'], d['emitted_equal_planted'], d['launches'])"; }
for i in 1 2 3; do
  for ramp in 0 1; do
    CUDASP_TF_RAMP=$ramp e2e cfg2_r${ramp}_$i --rows 1000000 --reps 5
    CUDASP_TF_RAMP=$ramp e2e cfg3_r${ramp}_$i --rows 9400000 --labels 1 --reps 3
  done
done
for ramp in 0 1; do CUDASP_TF_RAMP=$ramp e2e cfg4_r${ramp} --rows 32700000 --reps 3; done
