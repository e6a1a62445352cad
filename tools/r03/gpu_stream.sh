# Streaming scan (cudasp_stream_*): GPU tests (the stream API, then the
# table-function host that now runs it), then the probe against the
# device-resident multi-batch kernel.  $1: probe rows (default 3000000).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_stream; mkdir -p $O; cd $R
if [ -z "$NOTEST" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_stream_gpu.py -x -v --timeout 100 --timeout-method thread > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
  timeout -k 10 600 python -u -m pytest tests/test_host_feeds_gpu.py tests/test_sql_cases_gpu.py tests/test_arrow_gpu.py -x -v --timeout 120 --timeout-method thread > $O/tests_host.log 2>&1 || { tail -60 $O/tests_host.log; exit 1; }
  tail -2 $O/tests_host.log
fi
ROWS=${1:-3000000}
timeout -k 10 300 python -u tools/stream_probe.py --rows $ROWS > $O/probe_$ROWS.json 2> $O/probe_$ROWS.err || { tail -30 $O/probe_$ROWS.err; exit 1; }
cat $O/probe_$ROWS.json
