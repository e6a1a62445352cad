# Hypothesis check for profiles/r05n_pinned_c.txt: 4 and 8 logical GPUs on one
# card scan slower than 1 because their streams share GPU_MAX_HW_QUEUES = 4
# hardware queues (persistent kernels on a shared queue run one after
# another).  Same runs at 4 (default) and 16 queues.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_pinned_c_q; mkdir -p $O; cd $R
for q in 4 16; do
  for dv in 0,0 0,0,0,0 0,0,0,0,0,0,0,0; do
    tag=q${q}_$(echo $dv | tr ',' '_')
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 tools/host_e2e --rows 32700000 --batch 300000 --outputs 2 --reps 3 --pinned $dv > $O/$tag.json 2> $O/$tag.err || { echo "$tag failed"; tail -5 $O/$tag.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], '%.1f M exact %s scans %s' % (d['tx_per_s']/1e6, d['emitted_equal_planted'], [round(x,4) for x in d['seconds_all']]))" $O/$tag.json $tag
  done
done
