# Runtime rows per thread (CUDASP_MULTI_ROWS) on a build with 6 pending slots per piece
# (build_variants/m6: CUDASP_MULTI_RMAX=6) at 0, 1 and 16 labels, interleaved rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
B="python bench.py --no-cpu-baseline --no-e2e --no-layout-probe --exclusive-batches 0"
IFS=',' read -r -a SH <<< "${SHAPES:-9400000 --labels 1,9400000 --labels 16 --outputs-max 15,32700000,4200000}"
for round in $(seq ${AB_ROUNDS:-2}); do
for rt in ${RTS:-6 5 4}; do
for rows in "${SH[@]}"; do
  CUDASP_MULTI_ROWS=$rt CUDASP_LIB=$R/build_variants/m6/libcudasp_amd.so timeout -k 10 300 $B --rows $rows --steps 5 --warmup 2 > $O/rt_b.log 2>&1 || { echo "bench failed $rt"; tail -20 $O/rt_b.log; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('$O/rt_b.log') if l.startswith('{\"metric')][-1]);print('rows/thread', sys.argv[1], 'rows', sys.argv[2], round(d['value']/1e6,2), 'M tx/s', round(d['ms_per_step'],2), 'ms', d['matches']['found'], d['matches']['expected_planted'])" $rt "$rows" | tee -a $O/rt_ab.txt
done
done
done
