# Round 3: device-feed uploads on the null stream (default) vs on the scan
# stream (CUDASP_TF_UPLOAD=stream), interleaved on one box; slot ring depth.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_upload; mkdir -p $O; cd $R
e2e() { name=$1; shift; timeout -k 10 300 tools/host_e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "e2e $name failed"; tail -5 $O/$name.err; exit 1; }; python -c "
import json; d=json.load(open('$O/$name.json')); print('$name', round(d['tx_per_s']/1e6,1), d['seconds_all'], d['emitted_equal_planted'], d['launches'])"; }
for i in 1 2; do
  for up in null stream; do
    CUDASP_TF_UPLOAD=$up e2e cfg2_${up}_$i --rows 1000000 --reps 5
    CUDASP_TF_UPLOAD=$up e2e cfg3_${up}_$i --rows 9400000 --labels 1 --reps 3
    CUDASP_TF_UPLOAD=$up e2e cfg4_${up}_$i --rows 32700000 --reps 3
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr_cfg3 -o t -- $R/tools/host_e2e --rows 9400000 --labels 1 --reps 2 > $O/tr_cfg3.log 2>&1 || { echo trace failed; exit 1; }
python3 $R/tools/timeline.py $O/tr_cfg3/t_kernel_trace.csv --copies $O/tr_cfg3/t_memory_copy_trace.csv > $O/tr_cfg3.txt && tail -9 $O/tr_cfg3.txt
