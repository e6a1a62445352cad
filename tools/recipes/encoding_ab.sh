# A/B of the field reductions' limb masks as SGPR operands (4-byte VOP2
# v_and_b32, tools/gen_fe_asm.py --smask, library in ab/smask/) against the
# default 32-bit literals (8-byte encodings), and with the simple limb ops' constants in SGPRs too (-DCUDASP_SCONST=1, ab/sconst/): the encoding microbench
# (tools/microbench/int_throughput) first, then device-resident bench steps
# at config 4, interleaved, three passes on one box.  Result
# (profiles/r06_encoding_ab.txt): no gain per MHz, so both variants' code was
# reverted; the microbench part still runs as is (VARIANTS=default for the
# bench part alone).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r06}_enc; mkdir -p $O; cd $R
if [ -z "$SKIP_MB" ]; then
  timeout -k 10 120 ./tools/microbench/int_throughput > $O/int_throughput.txt 2>&1 || { echo "microbench failed"; cat $O/int_throughput.txt; exit 1; }
  cat $O/int_throughput.txt
fi
B="python3 -u bench.py --no-cpu-baseline --no-e2e --no-layout-probe --no-cold-start --idle-samples 0 --exclusive-batches 0"
for pass in $(seq 1 ${PASSES:-3}); do
  for v in ${VARIANTS:-default smask sconst}; do
    lib=duckdb-cudasp-extension_amd/libcudasp_amd.so; [ $v != default ] && lib=ab/$v/libcudasp_amd.so
    f=$O/${v}_$pass.json
    CUDASP_LIB=$lib timeout -k 10 300 $B --rows 32700000 --steps ${STEPS:-10} --warmup 2 > $f 2> $f.err || { echo "bench $v failed"; tail -5 $f.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; c=d['clock']['shader_mhz']; print(sys.argv[1].split('/')[-1].ljust(16), 'M tx/s %.2f' % (d['value']/1e6), 'kernel_ms %.3f' % r['kernel_ms'], 'MHz %.1f' % c, 'k tx/s/MHz %.2f' % (d['value']/1e3/c), 'found', d['matches']['found'], 'of', d['matches']['expected_planted'])" $f
  done
done
