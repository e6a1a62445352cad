# Round 3: why the device feeds run 32.7M rows at ~131M tx/s end to end:
# hardware queues and streams per feed A/B, then kernel + copy traces.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_e2e_diag; mkdir -p $O; cd $R
e2e() { name=$1; shift; timeout -k 10 300 tools/host_e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "e2e $name failed"; tail -5 $O/$name.err; cat $O/$name.json; exit 1; }; python -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', d['tx_per_s']/1e6, d['seconds_all'], d['emitted_equal_planted'], d['launches'], d['harvest_wait_s'], d['streams_per_feed'], d['gpu_max_hw_queues'])"; }
for st in 4 3 2; do CUDASP_TF_STREAMS=$st e2e s${st}_q4 --rows 32700000 --reps 2; done
for st in 4 8; do GPU_MAX_HW_QUEUES=16 CUDASP_TF_STREAMS=$st e2e s${st}_q16 --rows 32700000 --reps 2 || true; done
cd /tmp && export TMPDIR=/tmp
for q in 4 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr_q$q -o t -- $R/tools/host_e2e --rows 32700000 > $O/tr_q$q.log 2>&1 || { echo trace failed; tail $O/tr_q$q.log; exit 1; }
  K=$(ls $O/tr_q$q/*kernel_trace.csv $O/tr_q$q/*/*kernel_trace.csv 2>/dev/null | head -1)
  C=$(ls $O/tr_q$q/*memory_copy_trace.csv $O/tr_q$q/*/*memory_copy_trace.csv 2>/dev/null | head -1)
  python3 $R/tools/timeline.py "$K" --copies "$C" > $O/tr_q$q.txt && tail -30 $O/tr_q$q.txt
done
