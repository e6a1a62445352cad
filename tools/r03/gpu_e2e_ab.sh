# Round 3: device-feed end to end after the stream budget fix; ramp A/B;
# then the host-feed and multi-batch GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_e2e_ab; mkdir -p $O; cd $R
python -c "import bench; open('$O/labels16.bin','wb').write(b''.join(bench.label_keys(16)))"
e2e() { name=$1; shift; timeout -k 10 300 tools/host_e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "e2e $name failed"; tail -5 $O/$name.err; cat $O/$name.json; exit 1; }; python -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', round(d['tx_per_s']/1e6,1), d['seconds_all'], d['emitted_equal_planted'], d['launches'], d['harvest_wait_s'], d['streams_per_feed'], d['gpu_max_hw_queues'])"; }
for ramp in 0 1; do
  export CUDASP_TF_RAMP=$ramp
  e2e cfg2_r$ramp --rows 1000000 --reps 7
  e2e cfg3_r$ramp --rows 9400000 --labels 1 --reps 3
  e2e cfg4_r$ramp --rows 32700000 --reps 2
done
unset CUDASP_TF_RAMP
e2e cfg5 --rows 100000000 --labels 16 --labels-file $O/labels16.bin --outputs-max 15
e2e cfg4_cols --rows 32700000 --reps 2 --input columns
timeout -k 10 900 python -u -m pytest tests/test_host_feeds_gpu.py tests/test_multi_batch_gpu.py tests/test_fixed_base_widths_gpu.py tests/test_sql_cases_gpu.py tests/test_arrow_gpu.py -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/gpu_tests.log | tail -30; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
