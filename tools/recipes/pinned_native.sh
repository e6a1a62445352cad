# The C pinned table (cudasp_pinned_*, NativePinnedTable): its GPU tests beside
# PinnedTable's, then both scanned at configs 2, 3 and 4 on the same box
# (tools/pinned_bench.py, each table pinned once and scanned 3 times), then a
# short soak of both against cudasp_scan_arrow.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_pinned_native; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_pinned_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for cfg in "1000000 0" "9400000 1" "32700000 0"; do
  set -- $cfg
  for impl in native python; do
    f=""; [ $impl = native ] && f="--native"
    timeout -k 10 600 python -u tools/pinned_bench.py --rows $1 --labels $2 --reps 3 $f > $O/${impl}_$1.json 2> $O/${impl}_$1.err || { echo "$impl $1 failed"; tail -20 $O/${impl}_$1.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[3], sys.argv[2], '%.1f M exact %s pin %.2f s scans %s' % (d['tx_per_s']/1e6, d['exact'], d['pin_s'], [s['s'] for s in d['scans']]))" $O/${impl}_$1.json $1 $impl
  done
done
timeout -k 10 300 python -u tools/soak_pinned.py --minutes ${SOAK_MIN:-3} --seed 7 > $O/soak.log 2>&1 || { echo "soak failed"; tail -5 $O/soak.log; exit 1; }
tail -1 $O/soak.log
