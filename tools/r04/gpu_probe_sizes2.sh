# Round 4: the size sweep's remaining points (a 600k-row batch at 32.7M rows:
# the descriptor ring holds 64 batches), then one PMC pass of both kernels on
# the same 3M rows (L2 hits/misses, fabric reads, wave cycles and waits).
set -e
mkdir -p gpurun_out/r04
timeout -k 10 200 python tools/stream_probe.py --rows 32700000 --batch 600000 --labels 0 --modes all --reps 2 > gpurun_out/r04/sz_l0_32700000.json
for n in 1000000 3000000 12000000; do
  timeout -k 10 200 python tools/stream_probe.py --rows $n --labels 16 --kmax 15 --modes all --reps 2 > gpurun_out/r04/sz_l16_$n.json
done
R=$PWD; O=$R/gpurun_out/r04/pmc3; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES --output-format csv -d $O/p1 -o p -- python3 $R/tools/stream_probe.py --rows 3000000 --labels 0 --modes all --reps 1 > $O/p1.log 2>&1
echo done
