# 2 ranks (gloo) on one GPU; bench prints per-batch diagnostics when a rank's
# found count differs from its planted count.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for s in 2 2 2; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --rows 3000000 --steps $s --dist-backend gloo --no-cpu-baseline > $O/d_2rank_$s.log 2>&1 || exit 1
grep -a -o '"matches.*\|rank [01]:.*' $O/d_2rank_$s.log || true
done
