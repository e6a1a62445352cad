# Streaming scan iteration: stream GPU tests, probe at 3M and 9.4M rows,
# then end to end stream vs launch at configs 2 and 3.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_stream_q; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests/test_stream_gpu.py -x -v --timeout 100 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rows in 3000000 9400000; do
  timeout -k 10 300 python -u tools/stream_probe.py --rows $rows > $O/probe_$rows.json 2> $O/probe_$rows.err || { tail -30 $O/probe_$rows.err; exit 1; }
  python -c "import json; d=json.load(open('$O/probe_$rows.json')); print($rows, 'multi %.1f' % (d['multi_tx_s']/1e6), ' '.join('%s %.1f' % (m, d['stream_%s_tx_s' % m]/1e6) for m in ('all','dev_all','paced')), d['flags_equal'], d['counters_all'])"
done
e2e() { name=$1; shift; timeout -k 10 300 tools/host_e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "e2e $name failed"; tail -5 $O/$name.err; cat $O/$name.json; exit 1; }; python -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', round(d['tx_per_s']/1e6,1), d['seconds_all'], d['emitted_equal_planted'], d['launches'], d.get('streaming_feeds'), d['harvest_wait_s'])"; }
for mode in stream launch stream; do
  if [ $mode = stream ]; then export CUDASP_TF_MODE=stream; else unset CUDASP_TF_MODE; fi
  e2e cfg2_$mode --rows 1000000 --reps 5
  e2e cfg3_$mode --rows 9400000 --labels 1 --reps 3
done
echo all-done
