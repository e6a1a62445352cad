# k_scan_multi rows per thread (CUDASP_MULTI_RMAX builds in build_variants/r<R>, pipelined schedule):
# default bench and a rank's N = 8 share (or SHAPES="rows [bench options],..."), interleaved rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
B="python bench.py --no-cpu-baseline --no-e2e --no-layout-probe --exclusive-batches 0"
for round in $(seq ${AB_ROUNDS:-2}); do
for v in ${VARIANTS:-r6 r4 r5 r8}; do
IFS=',' read -r -a SH <<< "${SHAPES:-32700000,4200000}"
for rows in "${SH[@]}"; do
  CUDASP_LIB=$R/build_variants/$v/libcudasp_amd.so timeout -k 10 300 $B --rows $rows --steps 5 --warmup 2 > $O/rmax_b.log 2>&1 || { echo "bench failed $v"; tail -20 $O/rmax_b.log; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('$O/rmax_b.log') if l.startswith('{\"metric')][-1]);print(sys.argv[1], 'rows', sys.argv[2], round(d['value']/1e6,2), 'M tx/s', round(d['ms_per_step'],2), 'ms', d['matches']['found'], d['matches']['expected_planted'])" $v "$rows" | tee -a $O/rmax_ab.txt
done
done
done
