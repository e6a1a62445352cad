# Label compares behind a 64-bit membership filter of the row's outputs
# (build_variants/filter = the in-tree build) vs without (build_variants/base):
# the GPU label tests, then 0-, 1- and 16-label bench shapes, interleaved rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "label or multi or variant or sql" --timeout 300 --timeout-method thread > $O/filter_tests.log 2>&1 || { echo tests failed; tail -30 $O/filter_tests.log; exit 1; }
tail -1 $O/filter_tests.log
B="python bench.py --no-cpu-baseline --no-e2e --no-layout-probe --exclusive-batches 0"
for round in $(seq ${AB_ROUNDS:-3}); do
for v in filter base; do
for shape in "9400000 --labels 16 --outputs-max 15" "9400000 --labels 1" "32700000"; do
  CUDASP_LIB=$R/build_variants/$v/libcudasp_amd.so timeout -k 10 300 $B --rows $shape --steps 5 --warmup 2 > $O/filter_b.log 2>&1 || { echo "bench failed $v"; tail -20 $O/filter_b.log; exit 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open('$O/filter_b.log') if l.startswith('{\"metric')][-1]);print(sys.argv[1], 'rows', sys.argv[2], round(d['value']/1e6,2), 'M tx/s', round(d['ms_per_step'],2), 'ms', d['matches']['found'], d['matches']['expected_planted'])" $v "$shape" | tee -a $O/filter_ab.txt
done
done
done
