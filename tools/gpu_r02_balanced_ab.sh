# Balanced round-robin batch sizing (bench default --batch-size 0) vs fixed
# 300000-row batches: rank 0's share of config 4 at N = 2 / 4 / 8, run alone on
# one GPU (the SCALE shares), then a 2-rank gloo rehearsal of the default.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
B="python bench.py --no-cpu-baseline --no-e2e --no-layout-probe --exclusive-batches 0 --steps 5 --warmup 2"
for round in 1 2; do
for s in "8 4200000 300000" "8 4087510 291965" "4 8400000 300000" "4 8175020 291965" "2 16500000 300000" "2 16350015 297273"; do
  set -- $s
  timeout -k 10 300 $B --rows $2 --batch-size $3 > $O/bal_b.log 2>&1 || { echo "bench failed $s"; tail -20 $O/bal_b.log; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('$O/bal_b.log') if l.startswith('{\"metric')][-1]);ms=d['ms_per_step'];print('N', sys.argv[1], 'share rows', sys.argv[2], 'batch', sys.argv[3], round(ms,2), 'ms', 'job-equivalent', round(32.7e6/ms/1e3,2), 'M tx/s', d['matches']['found'], d['matches']['expected_planted'])" $1 $2 $3 | tee -a $O/balanced_ab.txt
done
done
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --dist-backend gloo --no-layout-probe > $O/bal_r2.log 2>&1 || { echo r2 failed; tail -30 $O/bal_r2.log; exit 1; }
tail -1 $O/bal_r2.log | cut -c1-200 | tee -a $O/balanced_ab.txt
python3 -c "import json;d=json.loads([l for l in open('$O/bal_r2.log') if l.startswith('{\"metric')][-1]);print('2-rank', d['config']['batch_size'], d['config']['batches_rank0'], d['matches'])" | tee -a $O/balanced_ab.txt
echo all-done
