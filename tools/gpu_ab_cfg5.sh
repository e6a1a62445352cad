# A/B of build_variants/*.so at config-5 shape (16 labels, 1..15 outputs/row), 9.4M rows.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
for round in 1 2; do
for lib in build_variants/*.so; do
  CUDASP_LIB=$R/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-layout-probe --rows 9400000 --labels 16 --outputs-max 15 --steps 3 > $O/bench_ab.log 2>&1 || { tail -5 $O/bench_ab.log; exit 1; }
  python -c "import json,sys;d=json.loads(open('$O/bench_ab.log').read().strip().splitlines()[-1]);print(sys.argv[1], round(d['value']/1e6,2), 'M tx/s', d['matches']['found'], round(d['roofline']['match_kernel_ms'],3))" $lib
done
done
