# Multi-rank rehearsals of the multi-batch bench on one MI355X over gloo:
# 4 ranks, round-robin config 4 (each rank its 28 batches, balanced batch size, in one
# k_scan_multi launch per step, 4 processes sharing the GPU).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 4 --steps 3 --dist-backend gloo --no-layout-probe > $O/r4.log 2>&1 || { echo failed; tail -30 $O/r4.log; exit 1; }
tail -1 $O/r4.log | cut -c1-300
echo all-done
