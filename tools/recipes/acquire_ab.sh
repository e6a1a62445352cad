# The streaming kernel's per-piece system-scope acquire (the default) against
# the build without it (build_variants/pf_noacq, -DCUDASP_AB_PF_NO_ACQUIRE:
# unsafe, measurement only), end to end through tools/host_e2e at configs 2, 3
# and 4 (default 16 slots), interleaved, two passes; then the slot-reuse tests.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_acqab; mkdir -p $O; cd $R
python3 -c "import bench; open('$O/labels1.bin','wb').write(b''.join(bench.label_keys(1)))"
for pass in 1 2; do
  for cfg in "1000000 0 5" "9400000 1 3" "32700000 0 2"; do
    set -- $cfg; rows=$1; lab=$2; reps=$3
    lf=""; [ $lab -gt 0 ] && lf="--labels-file $O/labels1.bin"
    for lib in default pf_noacq; do
      lp=""; [ $lib != default ] && lp="$R/build_variants/$lib"
      LD_LIBRARY_PATH=$lp timeout -k 10 300 tools/host_e2e --rows $rows --threads 8 --batch 300000 --labels $lab $lf --outputs 2 --reps $reps --warm-reps $reps > $O/e2e.json 2> $O/e2e.err; rc=$?
      echo "pass$pass rows=$rows labels=$lab $lib rc=$rc $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('tx/s %.1f M warm %.1f M exact %s' % (d['tx_per_s']/1e6, d['warm_tx_per_s']/1e6, d['emitted_equal_planted']))" $O/e2e.json)"
      [ $rc -eq 124 -o $rc -eq 137 ] && exit 1
    done
  done
done
timeout -k 10 300 python -u -m pytest tests/test_host_stream_gpu.py -m gpu -x -q -k slot_reuse --timeout 120 --timeout-method thread > $O/tests.log 2>&1; tail -1 $O/tests.log
