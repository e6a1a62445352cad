# Profiling sweep on one MI355X (each GPU step bounded; stop at the first failure):
#  1. rocprofv3 --kernel-trace --stats of the default bench (roofline kernel_ms cross-check)
#  2. SQ counters (two --pmc passes) of tools/quick_timing.py at a 300k-row batch
#  3. FETCH_SIZE / WRITE_SIZE (separate passes) of a 3M-row bench
# Summaries: tools/prof_summary.py and tools/pmc_summary.py, run afterwards on the CSVs.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
step() { local name=$1; shift; timeout -k 10 "$@" > $R/gpurun_out/$name.log 2>&1 || { echo "$name failed"; tail -30 $R/gpurun_out/$name.log; exit 1; }; tail -1 $R/gpurun_out/$name.log | cut -c1-400; }
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/prof_bench $R/gpurun_out/pmc_sq $R/gpurun_out/pmc_sq2 $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write
step prof_bench 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_bench -o bench -- python3 $R/bench.py --steps 2 --no-cpu-baseline
step pmc_sq 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/pmc_sq -o sq -- python3 $R/tools/quick_timing.py 300000 0
step pmc_sq2 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv -d $R/gpurun_out/pmc_sq2 -o sq2 -- python3 $R/tools/quick_timing.py 300000 0
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o fetch -- python3 $R/bench.py --rows 3000000 --steps 1 --warmup 0 --no-cpu-baseline
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o write -- python3 $R/bench.py --rows 3000000 --steps 1 --warmup 0 --no-cpu-baseline
echo all-done
