# Stage-B rows per thread (one shared Z inversion and one label inversion per
# thread): library builds with CUDASP_ROWS_B = 6 / 8 / 12 / 16 (build_variants/rb*.so,
# the shape forced with CUDASP_ROWS_B_FORCE), default bench and a config-5-shaped
# run (16 labels, 1..15 outputs per row), 2 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
B="python bench.py --no-cpu-baseline --no-e2e --no-layout-probe"
one() { local tag=$1 rb=$2; shift 2; CUDASP_LIB=$R/build_variants/rb$rb.so CUDASP_ROWS_B_FORCE=$rb timeout -k 10 300 $B "$@" > $O/rowsb.log 2>&1 || { echo "$tag rb$rb failed"; tail -20 $O/rowsb.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; m=d['matches']
print('%-5s rb%-3s %.1f M tx/s  B %.3f ms  found %d/%d' % (sys.argv[2], sys.argv[3], d['value']/1e6, r['match_kernel_ms'], m['found'], m['expected_planted']))" $O/rowsb.log $tag $rb; }
for round in 1 2; do
  for rb in 6 8 12 16; do one cfg4 $rb --steps 5 --warmup 2; done
  for rb in 6 8 12 16; do one L16 $rb --rows 6000000 --labels 16 --outputs-max 15 --steps 3 --warmup 1; done
done
echo all-done
