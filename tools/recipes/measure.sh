# Measurement set of a tree (e2e legs: streaming feeds and per-slot launches), on one box: GPU suite + smoke,
# rocprofv3 kernel trace (+ --stats) of the default bench command, then the
# bench lines at the configs' shapes and the 2-rank rehearsal.
#   $1: "notests" skips pytest + smoke
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_measure; mkdir -p $O; cd $R
if [ "$1" != "notests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/gpu_tests.log | tail -30; tail -60 $O/gpu_tests.log; exit 1; }
  tail -1 $O/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
cd /tmp && export TMPDIR=/tmp
rm -rf $O/prof_bench
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-layout-probe --idle-samples 0 --steps 3 --warmup 1 > $O/prof_bench.log 2>&1 || { echo prof failed; tail -20 $O/prof_bench.log; exit 1; }
tail -1 $O/prof_bench.log | cut -c1-200
cd $R
python3 tools/prof_summary.py $(ls $O/prof_bench/*kernel_trace.csv $O/prof_bench/*/*kernel_trace.csv 2>/dev/null | head -1) --out $O/rocprof_bench_summary.json > $O/prof_summary.txt && head -20 $O/prof_summary.txt
b() { name=$1; shift; timeout -k 10 900 python -u bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "bench $name failed"; tail -20 $O/$name.err; exit 1; }; python3 - "$O/$name.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d.get("e2e", {})
print(sys.argv[1].split("/")[-1], "value %.1f M" % (d["value"] / 1e6), "kernel_ms %.2f ms_per_step %.2f" % (d["roofline"]["kernel_ms"], d["ms_per_step"]),
      "e2e %.1f M" % ((d.get("e2e_tx_s") or 0) / 1e6), "ratio %.3f" % ((d.get("e2e_tx_s") or 0) / d["value"]),
      "like-for-like", d.get("e2e_vs_device"), "warm %.1f M" % ((d.get("e2e_warm_tx_s") or 0) / 1e6),
      "found %s" % d["matches"]["found"], "planted %s" % d["matches"]["expected_planted"], "e2e exact", e.get("emitted_equal_planted"), "e2e_launch %.1f M" % ((d.get("e2e_launch_tx_s") or 0) / 1e6), d.get("e2e_launch", {}).get("emitted_equal_planted"), "streaming_feeds", e.get("streaming_feeds"))
PY
}
b default --steps 10 --warmup 3
b cfg2 --rows 1000000 --steps 10 --warmup 3
b cfg3 --rows 9400000 --labels 1 --steps 10 --warmup 3
b cfg5 --rows 100000000 --labels 16 --outputs-max 15 --steps 3 --warmup 1 --cpu-rows 300000
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo > $O/rehearsal_2rank.json 2> $O/rehearsal_2rank.err || { echo "2-rank failed"; tail -30 $O/rehearsal_2rank.err; exit 1; }
echo all-done
