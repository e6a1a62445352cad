# rocprofv3 kernel trace of the end-to-end host with its streaming feeds at
# config 4 (k_scan_stream launches and durations against the query's wall time).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_e2e_stream_prof; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o e2e -- $R/tools/host_e2e --rows 32700000 --reps 2 > $O/e2e.json 2> $O/e2e.err || { tail -20 $O/e2e.err; exit 1; }
cat $O/e2e.json
cd $R && python3 - $(ls $O/prof/*kernel_trace.csv $O/prof/*/*kernel_trace.csv 2>/dev/null | head -1) <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    k = r["Kernel_Name"]
    if "scan_stream" in k or "stream_relaunch" in k or "scan_multi" in k:
        print(k[:44], "%.3f ms" % ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6), "start", r["Start_Timestamp"], "grid", r.get("Grid_Size", r.get("Grid_Size_X", "")))
PY
cp $(ls $O/prof/*kernel_stats.csv $O/prof/*/*kernel_stats.csv 2>/dev/null | head -1) $O/kernel_stats.csv
