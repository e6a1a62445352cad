# A/B of k_scan_multi's PRIO instance (CUDASP_MULTI_PRIO_US: the streaming
# kernel's wave priority by piece age in the stage-A ladder) against the
# default instance, device-resident bench steps at 1M / 3M / 32.7M rows,
# interleaved, two passes.  (Round 5; the PRIO instance was removed after this
# A/B, profiles/r05_multi_prio_ab.txt: it needs the round-5 commit that had it.)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_prio; mkdir -p $O; cd $R
B="python3 bench.py --no-cpu-baseline --no-e2e --no-layout-probe --idle-samples 0 --exclusive-batches 0"
for pass in 1 2; do
  for rows in 1000000 3000000 32700000; do
    steps=20; [ $rows = 32700000 ] && steps=5
    for p in 0 3000 1000; do
      f=$O/r${rows}_p${p}_$pass.json
      CUDASP_MULTI_PRIO_US=$p timeout -k 10 300 $B --rows $rows --steps $steps --warmup 3 > $f 2> $f.err || { echo "bench $rows $p failed"; tail -5 $f.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], 'M tx/s %.2f' % (d['value']/1e6), 'kernel_ms %.3f' % d['roofline']['kernel_ms'], 'found', d['matches']['found'], d['matches']['expected_planted'])" $f
    done
  done
done
