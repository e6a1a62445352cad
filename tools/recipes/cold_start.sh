# Cold start of the table-function host: a 1M-row
# config-2 table written once, then fresh processes whose first GPU work is
# the first query (host_e2e --table-in): first_query_s against the warm
# queries' median, with the default (26-bit) and the 22-bit fixed-base table,
# the scanner-creation share (--cold-phases) and a HIP API + kernel trace of
# one cold process.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r06}_cold; mkdir -p $O; cd $R
E=$R/tools/host_e2e; T=/tmp/cudasp_cfg2_table.bin
timeout -k 10 180 $E --rows 1000000 --table-out $T > $O/gen.json || { echo gen failed; exit 1; }
q() { name=$1; shift; timeout -k 10 180 "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -5 $O/$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'first %.4f s, warm median %.4f s, ratio %.2f, hip_init %.3f, scanner_create %.3f, prewarm %.3f, exact %s %s' % (d['first_query_s'], d['seconds'], d['first_query_s'] / d['seconds'], d['hip_init_s'], d['scanner_create_s'], d['prewarm_s'], d['first_query_exact'], d['emitted_equal_planted']))" $O/$name.json $name; }
q cold_a $E --rows 1000000 --table-in $T --reps 5
q cold_b $E --rows 1000000 --table-in $T --reps 5
q phases $E --rows 1000000 --table-in $T --reps 5 --cold-phases
q prewarmed $E --rows 1000000 --table-in $T --reps 5 --prewarm
q prewarmed_b $E --rows 1000000 --table-in $T --reps 5 --prewarm
CUDASP_FB_BITS=22 q cold22 $E --rows 1000000 --table-in $T --reps 5
CUDASP_FB_BITS=22 q phases22 $E --rows 1000000 --table-in $T --reps 5 --cold-phases
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $O/prof -o cold -- $E --rows 1000000 --table-in $T --reps 2 > $O/prof.log 2>&1 || { echo prof failed; tail -5 $O/prof.log; exit 1; }
timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv -d $O/prof_pw -o pw -- $E --rows 1000000 --table-in $T --reps 2 --prewarm > $O/prof_pw.log 2>&1 || { echo prof_pw failed; tail -5 $O/prof_pw.log; exit 1; }
ls -R $O/prof | head -20
echo cold-done
