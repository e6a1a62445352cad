# Round 3: bench lines (device-resident value + e2e through the host) at the
# BASELINE configs' shapes on one box, then a 2-rank gloo rehearsal of the
# N > 1 path (balanced secondary, e2e child over all visible GPUs).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_bench; mkdir -p $O; cd $R
b() { name=$1; shift; timeout -k 10 900 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "bench $name failed"; tail -20 $O/$name.err; exit 1; }; python - "$O/$name.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d.get("e2e", {})
print(sys.argv[1].split("/")[-1], "value %.1f M" % (d["value"] / 1e6), "e2e %.1f M" % ((d.get("e2e_tx_s") or 0) / 1e6),
      "ratio %.3f" % ((d.get("e2e_tx_s") or 0) / d["value"]), "found", d["matches"], "e2e exact", e.get("emitted_equal_planted"),
      "bal", d.get("value_balanced"), "cpu", d.get("cpu_baseline", {}).get("value"), d.get("host_cores_allotted"))
PY
}
b default --steps 10 --warmup 3
b cfg2 --rows 1000000 --steps 10 --warmup 3
b cfg3 --rows 9400000 --labels 1 --steps 10 --warmup 3
b cfg5 --rows 100000000 --labels 16 --outputs-max 15 --steps 3 --warmup 1 --cpu-rows 300000
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo > $O/rehearsal_2rank.json 2> $O/rehearsal_2rank.err || { echo "2-rank failed"; tail -30 $O/rehearsal_2rank.err; exit 1; }
tail -c 600 $O/rehearsal_2rank.json
