# Shape of the fused single-batch k_scan_multi launch (CUDASP_FUSED_ROWS rows per thread x
# CUDASP_FUSED_PIECES pieces per wave): the per-batch bench line (4 streams) and the end-to-end
# host, interleaved rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
export CUDASP_FB_BITS=26
for round in $(seq ${AB_ROUNDS:-2}); do
for shape in ${SHAPES:-4:1 6:1 4:2 6:2 5:1}; do
  export CUDASP_FUSED_ROWS=${shape%%:*} CUDASP_FUSED_PIECES=${shape##*:}
  timeout -k 10 300 python bench.py --launch batches --no-cpu-baseline --no-e2e --no-layout-probe --exclusive-batches 0 --steps 5 --warmup 2 > $O/fs_b.log 2>&1 || { echo "bench failed $shape"; tail -20 $O/fs_b.log; exit 1; }
  timeout -k 10 120 ./tools/host_e2e 32700000 8 300000 0 2 rows > $O/fs_e.log 2> $O/fs_e_err.log || { echo "e2e failed $shape"; tail -5 $O/fs_e_err.log; exit 1; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('$O/fs_b.log') if l.startswith('{\"metric')][-1]); e=json.loads(open('$O/fs_e.log').read().strip().splitlines()[-1])
print('rows:pieces', sys.argv[1], 'batches', round(d['value']/1e6,2), 'M tx/s', d['matches']['found'], '| e2e', round(e['tx_per_s']/1e6,2), 'M tx/s', e['matches'], e['planted'])" $shape | tee -a $O/fused_shape_ab.txt
done
done
