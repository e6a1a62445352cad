# Round 4: the workers' first tickets handed out by index (k_stream_start)
# instead of ~3k serialized same-address atomics: streaming GPU tests, then
# the kernel alone against the previous build (equal clocks: --prewarm) at
# 1M / 3M / 9.4M rows and end to end at configs 2 and 3 (host_e2e links the
# in-tree library; the previous build through LD_LIBRARY_PATH), two passes.
set -e
mkdir -p gpurun_out/r04
timeout -k 10 400 python -u -m pytest tests/test_stream_gpu.py tests/test_host_stream_gpu.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r04/t_first.log 2>&1 || { tail -30 gpurun_out/r04/t_first.log; exit 1; }
tail -1 gpurun_out/r04/t_first.log
E=./tools/host_e2e
for pass in 1 2; do
  echo pass $pass
  for v in prev new; do
    L=""
    [ $v = prev ] && L=$PWD/build_variants/prev/libcudasp_amd.so
    for n in 1000000 3000000 9400000; do
      CUDASP_LIB=$L timeout -k 10 200 python tools/stream_probe.py --rows $n --labels 0 --modes all --reps 3 --prewarm > gpurun_out/r04/fc_${v}_${n}_$pass.json
    done
    LDP=$LD_LIBRARY_PATH
    [ $v = prev ] && export LD_LIBRARY_PATH=$PWD/build_variants/prev:$LD_LIBRARY_PATH
    timeout -k 10 120 $E --rows 1000000 --threads 8 --batch 300000 --labels 0 --input rows --reps 5 --warm-reps 5 --outputs 2 > gpurun_out/r04/fc_${v}_e2e2_$pass.json
    timeout -k 10 120 $E --rows 9400000 --threads 8 --batch 300000 --labels 1 --input rows --reps 3 --warm-reps 3 --outputs 2 > gpurun_out/r04/fc_${v}_e2e3_$pass.json
    export LD_LIBRARY_PATH=$LDP
  done
done
echo done
