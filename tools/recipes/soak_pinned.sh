# Randomized soak of the pinned tables (tools/soak_pinned.py: PinnedTable and
# NativePinnedTable in both placements against cudasp_scan_arrow), then the
# default bench line (pinned and resident legs included).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_soak_pinned; mkdir -p $O; cd $R
timeout -k 10 $((${SOAK_MIN:-5} * 60 + 120)) python -u tools/soak_pinned.py --minutes ${SOAK_MIN:-5} --seed ${SEED:-11} > $O/soak.log 2>&1 || { echo "soak failed"; tail -5 $O/soak.log; exit 1; }
tail -1 $O/soak.log
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo "bench failed"; tail -20 $O/bench_default.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_default.json').read().strip().splitlines()[-1])
print('value %.1f M e2e %.1f M pinned %.1f M (%s) resident %.1f M (%s)' % (d['value']/1e6, d['e2e_tx_s']/1e6, d['pinned_tx_s']/1e6, d['pinned']['emitted_equal_planted'], d['resident_tx_s']/1e6, d['resident']['emitted_equal_planted']))"
