# Round 4: end-to-end rates (tools/host_e2e) at configs 2, 3 and 4, the
# streaming kernel against k_scan_multi on the same rows (tools/stream_probe.py),
# the 8-logical-GPU rehearsal, then event traces of configs 2 and 3 (trace build).
set -e
mkdir -p gpurun_out/r04
E=./tools/host_e2e
for i in; do
  timeout -k 10 120 $E --rows 1000000 --threads 8 --batch 300000 --labels 0 --input rows --reps 5 --outputs 2 > gpurun_out/r04/e2e_cfg2_$i.json
  timeout -k 10 120 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 3 --outputs 2 > gpurun_out/r04/e2e_cfg3_$i.json
done


timeout -k 10 200 python tools/stream_probe.py --rows 9400000 --labels 1 > gpurun_out/r04/probe_cfg3.json
rm -f gpurun_out/r04/tr_cfg*.bin
export LD_LIBRARY_PATH=$PWD/build_variants/strace:$LD_LIBRARY_PATH
CUDASP_STREAM_TRACE_FILE=gpurun_out/r04/tr_cfg2.bin timeout -k 10 150 $E --rows 1000000 --threads 8 --batch 300000 --labels 0 --input rows --reps 2 --outputs 2 > gpurun_out/r04/tr_cfg2.json
CUDASP_STREAM_TRACE_FILE=gpurun_out/r04/tr_cfg3.bin timeout -k 10 150 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 1 --outputs 2 > gpurun_out/r04/tr_cfg3.json
echo done
