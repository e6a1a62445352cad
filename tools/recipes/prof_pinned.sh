# rocprofv3 kernel traces of the C table's scans (tools/host_e2e --pinned 0
# [--hbm], config 4, 3 timed scans + 1 warm-up): the resident placement runs
# one k_scan_multi per scan, the pinned placement one k_scan_stream.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_prof_pinned; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
for pl in hbm pinned; do
  f=""; [ $pl = hbm ] && f="--hbm"
  rm -rf $O/$pl
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$pl -o scan -- $R/tools/host_e2e --rows ${ROWS:-32700000} --batch 300000 --outputs 2 --reps ${REPS:-3} --pinned 0 $f > $O/$pl.log 2>&1 || { echo "prof $pl failed"; tail -20 $O/$pl.log; exit 1; }
  grep -h "emitted_equal_planted" $O/$pl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$pl', '%.1f M exact %s' % (d['tx_per_s']/1e6, d['emitted_equal_planted']))"
  s=$(ls $O/$pl/*kernel_stats.csv $O/$pl/*/*kernel_stats.csv 2>/dev/null | head -1); head -6 "$s"
done
