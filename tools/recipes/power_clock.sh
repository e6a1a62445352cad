# Power and clocks while k_scan_multi runs (config 4, 30 steps): rocm-smi
# samples every ~2 s beside the bench, then the idle reading.  Read-only
# queries (no settings are changed).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r06}_power; mkdir -p $O; cd $R
timeout -k 5 20 rocm-smi --showpower --showclocks --showtemp --showmaxpower > $O/idle.txt 2>&1 || true
timeout -k 10 300 python3 -u bench.py --rows 32700000 --steps 30 --warmup 2 --no-cpu-baseline --no-e2e --no-layout-probe --no-cold-start --idle-samples 0 > $O/bench.json 2> $O/bench.err &
B=$!
for i in $(seq 1 40); do
  sleep 2
  kill -0 $B 2>/dev/null || break
  { date +%s.%N; timeout -k 5 10 rocm-smi --showpower --showclocks --showtemp 2>&1 | grep -E "Power|sclk|fclk|mclk|socclk|Temperature" ; } >> $O/samples.txt
done
wait $B; rc=$?
cat $O/idle.txt | grep -E "Power|sclk|fclk|mclk|Max" | head -12
grep -E "Power \(|sclk" $O/samples.txt | tail -24
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('M tx/s %.2f' % (d['value']/1e6), 'MHz', d['clock']['shader_mhz'])" $O/bench.json
exit $rc
