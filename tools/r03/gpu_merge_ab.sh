# (The merged-launch build this recipe measured was reverted after the A/B; CUDASP_TF_MERGE has no effect now.)
# Round 3: merged launches (CUDASP_TF_MERGE=1: 2 streams, an idle stream takes
# all ready slots, up to 4, in one cudasp_scan_device_batches launch) -- the
# host GPU tests under it first, then e2e A/B interleaved on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_merge; mkdir -p $O; cd $R
CUDASP_TF_MERGE=1 timeout -k 10 600 python -u -m pytest tests/test_host_feeds_gpu.py tests/test_sql_cases_gpu.py tests/test_arrow_gpu.py tests/test_variants_gpu.py -x -v --timeout 300 --timeout-method thread > $O/tests_merge.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/tests_merge.log | tail -30; tail -40 $O/tests_merge.log; exit 1; }
tail -1 $O/tests_merge.log
python -c "import bench; open('$O/labels16.bin','wb').write(b''.join(bench.label_keys(16)))"
e2e() { name=$1; shift; timeout -k 10 300 tools/host_e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "e2e $name failed"; tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.load(open('$O/$name.json')); print('$name', round(d['tx_per_s']/1e6,1), d['seconds_all'], d['emitted_equal_planted'], d['launches'], d['streams_per_feed'])"; }
for i in 1 2; do
  for m in 0 1; do
    CUDASP_TF_MERGE=$m e2e cfg2_m${m}_$i --rows 1000000 --reps 5
    CUDASP_TF_MERGE=$m e2e cfg3_m${m}_$i --rows 9400000 --labels 1 --reps 3
    CUDASP_TF_MERGE=$m e2e cfg4_m${m}_$i --rows 32700000 --reps 3
  done
done
for m in 0 1; do CUDASP_TF_MERGE=$m e2e cfg5_m$m --rows 100000000 --labels 16 --labels-file $O/labels16.bin --outputs-max 15; done
