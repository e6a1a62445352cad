# Streaming scan iteration 3 (16 slots per streaming feed): end to end
# stream vs launch at configs 2, 3, 4 and 5, interleaved; the streaming host test.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_stream_q3; mkdir -p $O; cd $R
python -c "import bench; open('$O/labels16.bin','wb').write(b''.join(bench.label_keys(16)))"
e2e() { name=$1; shift; timeout -k 10 300 tools/host_e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "e2e $name failed"; tail -5 $O/$name.err; cat $O/$name.json; exit 1; }; python -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', round(d['tx_per_s']/1e6,1), d['seconds_all'], d['emitted_equal_planted'], d['launches'], d.get('streaming_feeds'), d['harvest_wait_s'], d['copy_s'])"; }
for mode in stream launch stream launch; do
  if [ $mode = stream ]; then export CUDASP_TF_MODE=stream; else unset CUDASP_TF_MODE; fi
  e2e cfg2_$mode --rows 1000000 --reps 5
  e2e cfg3_$mode --rows 9400000 --labels 1 --reps 3
  e2e cfg4_$mode --rows 32700000 --reps 2
done
for mode in stream launch; do
  if [ $mode = stream ]; then export CUDASP_TF_MODE=stream; else unset CUDASP_TF_MODE; fi
  e2e cfg5_$mode --rows 100000000 --labels 16 --labels-file $O/labels16.bin --outputs-max 15
  e2e cfg4cols_$mode --rows 32700000 --reps 2 --input columns
done
unset CUDASP_TF_MODE
timeout -k 10 600 python -u -m pytest tests/test_host_feeds_gpu.py tests/test_stream_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo all-done
