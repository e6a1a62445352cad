# Streaming feed with few slots (CUDASP_TF_STREAM_SLOTS=4) and tiny batches:
# each slot's host memory is rewritten for a new batch a few batches later.
# Runs the default library and the diagnosis builds given in VARIANTS
# (build_variants/<v>/libcudasp_amd.so through LD_LIBRARY_PATH).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_repro; mkdir -p $O; cd $R
python3 -c "import bench; open('$O/labels2.bin','wb').write(b''.join(bench.label_keys(2)))"
for lib in default ${VARIANTS}; do
  lp=""; [ "$lib" != default ] && lp="$R/build_variants/$lib"
  for v in "4 2 16 1" "4 0 1 2048" "4 2 16 1" "16 2 16 1"; do
    set -- $v; slots=$1; lab=$2; th=$3; bs=$4
    lf=""; [ $lab -gt 0 ] && lf="--labels-file $O/labels2.bin"
    LD_LIBRARY_PATH=$lp CUDASP_TF_DEVICE_MAP=0 CUDASP_TF_STREAM_SLOTS=$slots timeout -k 10 120 tools/host_e2e --rows 65536 --threads $th --batch $bs --input rows --labels $lab $lf --outputs 2 --reps 3 > $O/run.json 2> $O/run.err; rc=$?
    echo "$lib slots=$slots labels=$lab threads=$th batch=$bs rc=$rc $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print({k:d.get(k) for k in ('matches','planted','emitted_equal_planted','tx_per_s')})" $O/run.json)"
    [ $rc -eq 124 -o $rc -eq 137 ] && exit 1
  done
done
exit 0
