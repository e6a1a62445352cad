set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $R/gpurun_out/pmc_sq -o sq -- python3 $R/tools/quick_timing.py 300000 0 > $R/gpurun_out/pmc_sq.log 2>&1 || { echo "pmc sq failed"; tail -20 $R/gpurun_out/pmc_sq.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv -d $R/gpurun_out/pmc_sq2 -o sq2 -- python3 $R/tools/quick_timing.py 300000 0 > $R/gpurun_out/pmc_sq2.log 2>&1 || { echo "pmc sq2 failed"; tail -20 $R/gpurun_out/pmc_sq2.log; exit 1; }
echo done
