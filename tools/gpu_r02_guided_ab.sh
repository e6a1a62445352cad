# Guided-scheduling thresholds of k_scan_multi (CUDASP_MULTI_G1 / G2, hundredths of the grid's waves)
# at the current rows per thread: every SCALE share, interleaved rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
B="python bench.py --no-cpu-baseline --no-e2e --no-layout-probe --exclusive-batches 0"
for round in $(seq ${AB_ROUNDS:-2}); do
for g in ${GS:-150:400 100:300 250:600 150:800 50:200}; do
for rows in ${ROWS:-32700000 8400000 4200000}; do
  CUDASP_MULTI_G1=${g%%:*} CUDASP_MULTI_G2=${g##*:} timeout -k 10 300 $B --rows $rows --steps 5 --warmup 2 > $O/guided_b.log 2>&1 || { echo "bench failed $g"; tail -20 $O/guided_b.log; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('$O/guided_b.log') if l.startswith('{\"metric')][-1]);print('g1:g2', sys.argv[1], 'rows', sys.argv[2], round(d['value']/1e6,2), 'M tx/s', round(d['ms_per_step'],2), 'ms', d['matches']['found'], d['matches']['expected_planted'])" $g $rows | tee -a $O/guided_ab.txt
done
done
done
