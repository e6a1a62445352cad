# Elastic streaming kernel (idle exit + relaunch, compare-and-swap claims):
# stream and host-feed GPU tests, probe, then end to end stream vs launch.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_stream_q4; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_stream_gpu.py tests/test_host_feeds_gpu.py tests/test_sql_cases_gpu.py tests/test_arrow_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u tools/stream_probe.py --rows 9400000 --labels 1 --in-flight 16 --reps 2 > $O/probe.json 2> $O/probe.err || { tail -30 $O/probe.err; exit 1; }
python -c "import json; d=json.load(open('$O/probe.json')); print('probe', 'multi %.1f' % (d['multi_tx_s']/1e6), ' '.join('%s %.1f' % (m, d['stream_%s_tx_s' % m]/1e6) for m in ('all','dev_all','paced')), d['flags_equal'], d['counters_paced'])"
python -c "import bench; open('$O/labels16.bin','wb').write(b''.join(bench.label_keys(16)))"
e2e() { name=$1; shift; timeout -k 10 300 tools/host_e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "e2e $name failed"; tail -5 $O/$name.err; cat $O/$name.json; exit 1; }; python -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', round(d['tx_per_s']/1e6,1), d['seconds_all'], d['emitted_equal_planted'], d['launches'], d.get('streaming_feeds'), d['harvest_wait_s'])"; }
for mode in stream launch stream; do
  export CUDASP_TF_MODE=$mode
  e2e cfg2_$mode --rows 1000000 --reps 5
  e2e cfg3_$mode --rows 9400000 --labels 1 --reps 3
  e2e cfg4_$mode --rows 32700000 --reps 2
done
export CUDASP_TF_MODE=stream
e2e cfg5_stream --rows 100000000 --labels 16 --labels-file $O/labels16.bin --outputs-max 15
echo all-done
