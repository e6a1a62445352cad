# The resident placement of the C table (CUDASP_TABLE_HBM: appended once into
# HBM in k_scan_multi's layout, each scan one cudasp_scan_device_batches launch
# per GPU) beside the pinned placement, from C++ (tools/host_e2e --pinned 0
# [--hbm]); pinned GPU tests first.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_resident_c; mkdir -p $O; cd $R
timeout -k 10 400 python -u -m pytest tests/test_pinned_gpu.py -x -v --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" $O/tests.log | head; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
python3 -c "import bench; open('$O/labels1.bin','wb').write(b''.join(bench.label_keys(1)))"
for cfg in "1000000 0" "9400000 1" "32700000 0"; do
  set -- $cfg
  lf=""; [ $2 -gt 0 ] && lf="--labels-file $O/labels1.bin"
  for pl in hbm pinned; do
    f=""; [ $pl = hbm ] && f="--hbm"
    timeout -k 10 300 tools/host_e2e --rows $1 --batch 300000 --labels $2 $lf --outputs 2 --reps 5 --pinned 0 $f > $O/${pl}_$1.json 2> $O/${pl}_$1.err || { echo "$pl $1 failed"; tail -5 $O/${pl}_$1.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.1f M exact %s pin %.2f s scans %s device_bytes %.2f GB' % (d['tx_per_s']/1e6, d['emitted_equal_planted'], d['pin_s'], [round(x,4) for x in d['seconds_all']], d['device_bytes']/1e9))" $O/${pl}_$1.json ${pl}_$1
  done
done
