# Round 4: bench lines at configs 2 and 3 with the after-idle device step and
# the warm e2e queries (host_e2e --warm-reps).
set -e
mkdir -p gpurun_out/r04
timeout -k 10 120 ./tools/host_e2e --rows 200000 --threads 4 --batch 100000 --labels 0 --reps 1 --warm-reps 1 --outputs 2 > gpurun_out/r04/wb_smoke.json
timeout -k 10 600 python -u bench.py --rows 1000000 --steps 10 --warmup 3 --no-cpu-baseline --no-layout-probe > gpurun_out/r04/wb_cfg2.json 2> gpurun_out/r04/wb_cfg2.err
timeout -k 10 600 python -u bench.py --rows 9400000 --labels 1 --steps 10 --warmup 3 --no-cpu-baseline --no-layout-probe > gpurun_out/r04/wb_cfg3.json 2> gpurun_out/r04/wb_cfg3.err
echo done
