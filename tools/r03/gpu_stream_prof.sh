# Kernel trace of the streaming probe (k_scan_stream durations vs k_scan_multi).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_stream_prof; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o probe -- python3 $R/tools/stream_probe.py --rows ${1:-3000000} > $O/probe.json 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe.json
cd $R && python3 - $(ls $O/prof/*kernel_trace.csv $O/prof/*/*kernel_trace.csv 2>/dev/null | head -1) <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    k = r["Kernel_Name"]
    if "scan_stream" in k or "scan_multi" in k:
        print(k[:40], "%.3f ms" % ((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6), "grid", r.get("Grid_Size", r.get("Grid_Size_X", "")))
PY
