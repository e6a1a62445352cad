# Streaming scan iteration 2: probe with labels (in-flight 8 / 16), then end
# to end stream vs launch at configs 3, 4 and 5.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_stream_q2; mkdir -p $O; cd $R
python -c "import bench; open('$O/labels16.bin','wb').write(b''.join(bench.label_keys(16)))"
for spec in "1 8" "1 16" "16 8"; do
  set -- $spec
  timeout -k 10 300 python -u tools/stream_probe.py --rows 9400000 --labels $1 --in-flight $2 --reps 2 > $O/probe_L$1_f$2.json 2> $O/probe_L$1_f$2.err || { tail -30 $O/probe_L$1_f$2.err; exit 1; }
  python -c "import json; d=json.load(open('$O/probe_L$1_f$2.json')); print('L$1 f$2', 'multi %.1f' % (d['multi_tx_s']/1e6), ' '.join('%s %.1f' % (m, d['stream_%s_tx_s' % m]/1e6) for m in ('all','dev_all','paced')), d['flags_equal'], d['counters_paced'])"
done
e2e() { name=$1; shift; timeout -k 10 300 tools/host_e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "e2e $name failed"; tail -5 $O/$name.err; cat $O/$name.json; exit 1; }; python -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', round(d['tx_per_s']/1e6,1), d['seconds_all'], d['emitted_equal_planted'], d['launches'], d.get('streaming_feeds'), d['harvest_wait_s'], d['copy_s'])"; }
for mode in stream launch; do
  if [ $mode = stream ]; then export CUDASP_TF_MODE=stream; else unset CUDASP_TF_MODE; fi
  e2e cfg3_$mode --rows 9400000 --labels 1 --reps 3
  e2e cfg3L0_$mode --rows 9400000 --reps 3
  e2e cfg4_$mode --rows 32700000 --reps 2
  e2e cfg5_$mode --rows 100000000 --labels 16 --labels-file $O/labels16.bin --outputs-max 15
done
echo all-done
