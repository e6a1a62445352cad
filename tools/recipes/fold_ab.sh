# A/B of the spend key folded into the fixed-base table's top window
# (default) against the separate F = P0 + B addition (CUDASP_FB_FOLD=0):
# device-resident bench steps at config 4 (32.7M rows) and config 3 (9.4M
# rows, 1 label), interleaved, three passes on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_fold; mkdir -p $O; cd $R
B="python3 bench.py --no-cpu-baseline --no-e2e --no-layout-probe --idle-samples 0 --exclusive-batches 0"
for pass in 1 2 3; do
  for cfg in "32700000 0 5" "9400000 1 10"; do
    set -- $cfg
    for fold in 1 0; do
      f=$O/r$1_L$2_fold${fold}_$pass.json
      CUDASP_FB_FOLD=$fold timeout -k 10 300 $B --rows $1 --labels $2 --steps $3 --warmup 2 > $f 2> $f.err || { echo "bench $cfg fold $fold failed"; tail -5 $f.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1], 'M tx/s %.2f' % (d['value']/1e6), 'kernel_ms %.3f' % d['roofline']['kernel_ms'], 'folded', d['config']['spend_key_folded'], 'found', d['matches']['found'], d['matches']['expected_planted'])" $f
    done
  done
done
