# Round 3: the contiguous-rows shard (bench default) rehearsed with 2 and 4
# gloo ranks sharing one GPU (value vs the round-robin secondary line), and
# the default N = 1 line with the OpenSSL CPU baseline.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_shard; mkdir -p $O; cd $R
timeout -k 10 900 python -u bench.py --steps 5 --warmup 2 > $O/n1.json 2> $O/n1.err || { echo "n1 failed"; tail -20 $O/n1.err; exit 1; }
python - $O/n1.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("n1 value %.1f M" % (d["value"] / 1e6), d["config"]["shard"], d["matches"])
for k in ("cpu_baseline", "cpu_baseline_optimized", "cpu_baseline_openssl"):
    v = d.get(k, {})
    print(k, v.get("value"), v.get("cores"), v.get("flags_match_gpu"), v.get("sample"), v.get("error"))
PY
for n in 2 4; do
  timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2952$n bench.py --gpus $n --steps 5 --warmup 2 --dist-backend gloo --no-e2e > $O/rank$n.json 2> $O/rank$n.err || { echo "$n-rank failed"; tail -30 $O/rank$n.err; exit 1; }
  python - $O/rank$n.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], "value %.1f M" % (d["value"] / 1e6), "roundrobin %.1f M" % (d["value_roundrobin"] / 1e6),
      d["config"]["shard"], d["config"]["batch_size"], d["config"]["batches_rank0"], d["matches"], d["roundrobin"])
PY
done
