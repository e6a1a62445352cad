set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/e2e_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/e2e_pytest.log; exit 1; }
tail -1 gpurun_out/e2e_pytest.log
for T in 8 16 32; do
  timeout -k 10 300 ./tools/host_e2e 32700000 $T 300000 0 2 >> gpurun_out/e2e.log 2> gpurun_out/e2e_err.log || { echo "host_e2e failed T=$T"; tail -20 gpurun_out/e2e_err.log; exit 1; }
  tail -1 gpurun_out/e2e.log
done
