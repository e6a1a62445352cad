# Round 4: instruction-cache behaviour of k_scan_stream (200 KB of code) vs
# k_scan_multi (141 KB) on the same 3M rows: one PMC pass.
set -e
R=$PWD; O=$R/gpurun_out/r04/pmc_ic; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/p1 -o p -- python3 $R/tools/stream_probe.py --rows 3000000 --labels 0 --modes all --reps 1 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
echo done
