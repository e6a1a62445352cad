# Fixed-base window widths on one MI355X: the width tests, then the
# device-resident bench at 26 / 22 / 7 (LDS-staged) bits, and one rocprofv3
# kernel trace of the 7-bit bench for the per-kernel durations.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -30 $O/$name.log; exit 1; }; tail -1 $O/$name.log | cut -c1-200; }
cd $R
step widths_tests 300 python -u -m pytest tests/test_fixed_base_widths_gpu.py -x -v --timeout 200 --timeout-method thread
B="python bench.py --no-cpu-baseline --no-e2e --no-layout-probe --steps 5 --warmup 2"
for w in 26 22 7; do
  step bench_w$w 300 $B --fb-bits $w
done
cd /tmp && export TMPDIR=/tmp
step prof_w7 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_w7 -o w7 -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-layout-probe --steps 2 --warmup 1 --fb-bits 7
cd $R
python tools/prof_summary.py $O/prof_w7/w7_kernel_trace.csv --out $O/r02_rocprof_w7_summary.json > /dev/null
echo all-done
