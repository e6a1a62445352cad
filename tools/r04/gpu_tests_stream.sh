# Round 4: the streaming-scan and host GPU tests after the prefetch / match
# compaction / timeout rework.
set -e
mkdir -p gpurun_out/r04
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_host_feeds_gpu.py tests/test_sql_cases_gpu.py tests/test_arrow_gpu.py tests/test_labels16_gpu.py tests/test_variants_gpu.py > gpurun_out/r04/gpu_tests_stream.log 2>&1
echo done
