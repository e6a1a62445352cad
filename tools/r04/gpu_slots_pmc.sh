# Round 4: streaming-feed slot count x wave priority A/B at config 3 (and 2),
# then PMC passes of k_scan_stream vs k_scan_multi on the same rows
# (tools/stream_probe.py, all batches published).
set -e
mkdir -p gpurun_out/r04
E=./tools/host_e2e
for pass in 1 2; do
for sl in 16 32; do
for p in 0 3000 10000; do
  CUDASP_TF_STREAM_SLOTS=$sl CUDASP_STREAM_PRIO_US=$p timeout -k 10 120 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 3 --outputs 2 > gpurun_out/r04/sp_cfg3_${sl}_${p}_$pass.json
done
done
done
for p in 0 3000 10000; do
  CUDASP_STREAM_PRIO_US=$p timeout -k 10 120 $E --rows 1000000 --threads 8 --batch 300000 --labels 0 --input rows --reps 5 --outputs 2 > gpurun_out/r04/sp_cfg2_${p}.json
  CUDASP_TF_STREAM_SLOTS=32 CUDASP_STREAM_PRIO_US=$p timeout -k 10 200 $E --rows 32700000 --threads 8 --batch 300000 --labels 0 --input rows --reps 1 --outputs 2 > gpurun_out/r04/sp_cfg4_32_${p}.json
done
R=$PWD; O=$R/gpurun_out/r04/pmc; mkdir -p $O
B="python3 $R/tools/stream_probe.py --rows 3000000 --labels 1 --reps 1"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $O/sq1 -o sq -- $B > $O/sq1.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/sq2 -o sq -- $B > $O/sq2.log 2>&1
echo done
