# A/B of the doubled limbs as v_add_u32 x, x (dbl32, the default build)
# against the committed base build's v_lshlrev_b32 / v_mul_lo_u32 (library
# copied to ab/base/): device-resident bench steps at config 4, interleaved,
# three passes on one box; then the field/parity GPU tests on the new build.
# Result (profiles/r06_encoding_ab.txt): +0.1%, inside the spread; reverted.
set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
MEASURE_TAG=${MEASURE_TAG:-r06y} VARIANTS="base default" bash tools/recipes/encoding_ab.sh > /dev/null || exit 1
O=$R/gpurun_out/${MEASURE_TAG:-r06y}_enc
for pass in 1 2 3; do for v in base default; do f=$O/${v}_$pass.json
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; c=d['clock']['shader_mhz']; print(sys.argv[1].split('/')[-1].ljust(16), 'M tx/s %.2f' % (d['value']/1e6), 'kernel_ms %.3f' % r['kernel_ms'], 'MHz %.1f' % c, 'k tx/s/MHz %.2f' % (d['value']/1e3/c), 'found', d['matches']['found'], 'of', d['matches']['expected_planted'])" $f
done; done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_synth.py tests/test_gpu_field.py tests/test_labels16_gpu.py tests/test_full_configs_gpu.py > $O/tests.txt 2>&1; rc=$?; tail -3 $O/tests.txt; exit $rc
