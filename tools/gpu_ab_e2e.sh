# Host end-to-end A/B: the in-tree library vs build_variants/old (same ABI), rows and columns, 8 threads, 2 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for round in $(seq ${AB_ROUNDS:-2}); do
for v in new old; do
for mode in rows columns; do
  if [ $v = old ]; then export LD_LIBRARY_PATH=$R/build_variants/old; else unset LD_LIBRARY_PATH; fi
  timeout -k 10 300 ./tools/host_e2e ${E2E_ROWS:-32700000} 8 300000 0 2 $mode > $O/e2e_ab.log 2> $O/e2e_ab_err.log || { echo "failed $v $mode"; tail -5 $O/e2e_ab_err.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('$O/e2e_ab.log').read().strip().splitlines()[-1]);print(sys.argv[1], d['input'], round(d['tx_per_s']/1e6,2), 'M tx/s', d['matches'], d['planted'])" $v
done
done
done
