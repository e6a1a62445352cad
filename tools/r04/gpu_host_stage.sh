# Round 4: the host feed with copy-engine staging of each slot (measurement
# build with the CUDASP_TF_STAGE knob restored) against the in-place reads,
# end to end at configs 2 and 3 (cold / warm queries), two passes; then one
# rocprofv3 kernel trace of a staged config-2 run (blit kernels would show up
# as __amd_rocclr_copyBuffer).
set -e
mkdir -p gpurun_out/r04
export LD_LIBRARY_PATH=$PWD/build_variants/stage:$LD_LIBRARY_PATH
E=$PWD/tools/host_e2e
for pass in 1 2; do
  for st in 0 1; do
    CUDASP_TF_STAGE=$st timeout -k 10 60 $E --rows 1000000 --threads 8 --batch 300000 --labels 0 --input rows --reps 5 --warm-reps 5 --outputs 2 > gpurun_out/r04/hs${st}_cfg2_$pass.json
    CUDASP_TF_STAGE=$st timeout -k 10 90 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 3 --warm-reps 3 --outputs 2 > gpurun_out/r04/hs${st}_cfg3_$pass.json
  done
done
cd /tmp && export TMPDIR=/tmp
CUDASP_TF_STAGE=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04/hs_prof -o hs -- $E --rows 1000000 --threads 8 --batch 300000 --labels 0 --reps 2 --outputs 2 > $GRAFT_REPO_ROOT/gpurun_out/r04/hs_prof.json
echo done
