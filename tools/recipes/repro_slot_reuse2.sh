# Second soak failure (seed 2, run 19): streaming feed, 4 slots, ragged output
# lists.  Which factor matters: slots, labels, ragged lists, threads.
#   SHAPES="slots labels threads outs;..." (outs: k2, k8, max15), VARIANTS = build_variants to try
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_repro2; mkdir -p $O; cd $R
python3 -c "import bench; open('$O/labels1.bin','wb').write(b''.join(bench.label_keys(1)))"
for lib in default ${VARIANTS}; do
  lp=""; [ "$lib" != default ] && lp="$R/build_variants/$lib"
  IFS=';' read -ra shapes <<< "${SHAPES:-4 1 3 max15;4 0 1 k8;16 1 3 max15}"
  for v in "${shapes[@]}"; do
    set -- $v; slots=$1; lab=$2; th=$3; outs=$4
    lf=""; [ $lab -gt 0 ] && lf="--labels-file $O/labels1.bin"
    oa="--outputs 2"; [ $outs = max15 ] && oa="--outputs-max 15"; [ $outs = k8 ] && oa="--outputs 8"
    LD_LIBRARY_PATH=$lp CUDASP_TF_DEVICE_MAP=0 CUDASP_TF_STREAM_SLOTS=$slots timeout -k 10 120 tools/host_e2e --rows 300001 --threads $th --batch 2048 --input rows --labels $lab $lf $oa --reps 3 > $O/run.json 2> $O/run.err; rc=$?
    echo "$lib slots=$slots labels=$lab threads=$th outs=$outs rc=$rc $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print({k:d.get(k) for k in ('matches','planted','emitted_equal_planted','launches')})" $O/run.json)"
    grep -A4 "not exact" $O/run.err | head -6
    [ $rc -eq 124 -o $rc -eq 137 ] && exit 1
  done
done
exit 0
