# The C pinned table driven from C++ (tools/host_e2e --pinned: appended once
# in Arrow runs, scanned R times; each scan must return exactly the planted
# rows): configs 2, 3 (1 label) and 4 on the whole card, then config 4 over 4
# and 8 logical GPUs on the one card (the N-GPU path's publish loop rehearsed).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_pinned_c; mkdir -p $O; cd $R
python3 -c "import bench; open('$O/labels1.bin','wb').write(b''.join(bench.label_keys(1)))"
for cfg in "1000000 0 0" "9400000 1 0" "32700000 0 0" "32700000 0 0,0,0,0" "32700000 0 0,0,0,0,0,0,0,0"; do
  set -- $cfg
  lf=""; [ $2 -gt 0 ] && lf="--labels-file $O/labels1.bin"
  tag=$1_$(echo $3 | tr ',' '_')
  timeout -k 10 300 tools/host_e2e --rows $1 --batch 300000 --labels $2 $lf --outputs 2 --reps 5 --pinned $3 > $O/pinned_$tag.json 2> $O/pinned_$tag.err || { echo "pinned $tag failed"; tail -5 $O/pinned_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('C pinned', sys.argv[2], '%.1f M exact %s pin %.2f s scans %s batches %d' % (d['tx_per_s']/1e6, d['emitted_equal_planted'], d['pin_s'], [round(x,4) for x in d['seconds_all']], d['batches']))" $O/pinned_$tag.json $tag
done
