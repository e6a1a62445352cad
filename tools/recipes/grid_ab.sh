# k_scan_multi grid: every wave slot (3 waves per SIMD, 768 blocks) against 2 per
# SIMD (512 blocks, CUDASP_MULTI_BLOCKS), device-resident bench steps at 1M,
# the N = 8 share of config 4 and config 4, interleaved, two passes.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_grid; mkdir -p $O; cd $R
for pass in 1 2; do
  for rows in 1000000 4087500 32700000; do
    for bl in 768 512; do
      steps=10; [ $rows -le 4087500 ] && steps=20
      CUDASP_MULTI_BLOCKS=$bl timeout -k 10 300 python -u bench.py --rows $rows --steps $steps --warmup 3 --no-cpu-baseline --no-e2e --no-layout-probe --idle-samples 0 > $O/r${rows}_b${bl}_$pass.json 2> $O/r${rows}_b${bl}_$pass.err || { echo "bench $rows $bl failed"; tail -20 $O/r${rows}_b${bl}_$pass.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1].split('/')[-1].ljust(26), 'M tx/s %7.2f' % (d['value']/1e6), 'kernel_ms %8.3f' % d['roofline']['kernel_ms'], 'found', d['matches']['found'], 'of', d['matches']['expected_planted'])" $O/r${rows}_b${bl}_$pass.json
    done
  done
done
