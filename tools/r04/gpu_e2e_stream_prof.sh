# Round 4: rocprofv3 kernel traces on one box of (1) tools/host_e2e at config 4
# with its streaming feed: a warm-up query, 2 queries from an idle GPU and 2
# right after a busy kernel (--warm-reps), and (2) the bench's device-resident
# k_scan_multi steps (3 back to back, then 3 each after 100 ms idle) on the
# same rows -- the streaming kernel's duration against k_scan_multi's in the
# same clock states.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r04_e2e_stream_prof; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
rm -rf $O/prof $O/profb
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o e2e -- $R/tools/host_e2e --rows 32700000 --reps 2 --warm-reps 2 > $O/e2e.json 2> $O/e2e.err || { tail -20 $O/e2e.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profb -o bench -- python3 $R/bench.py --no-cpu-baseline --no-e2e --no-layout-probe --steps 3 --warmup 1 --idle-samples 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cd $R && for d in prof profb; do python3 - $(ls $O/$d/*kernel_trace.csv $O/$d/*/*kernel_trace.csv 2>/dev/null | head -1) <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    k = r["Kernel_Name"]
    if "scan_stream" in k or "stream_start" in k or "scan_multi" in k or "k_busy" in k:
        print(k[:44], "%.3f ms" % ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6), "start", r["Start_Timestamp"])
PY
done
echo done
