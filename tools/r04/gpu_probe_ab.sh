# Round 4: what makes k_scan_stream slower than k_scan_multi on the same rows
# (all batches published): measurement-only builds without the ladder's
# priority hook, without the prefetch's outputs copy (results wrong, timing
# only), without the emit's completion wait (unsafe, timing only), and the
# per-lane blob loads; interleaved, two passes.
set -e
mkdir -p gpurun_out/r04
P="python tools/stream_probe.py --rows 9400000 --labels 1 --modes all --reps 2"
for pass in 1 2; do
  echo pass $pass
  timeout -k 10 200 $P > gpurun_out/r04/ab_base_$pass.json
  for v in NO_TICK NO_OUTCOPY NO_EMIT_WAIT; do
    CUDASP_LIB=$PWD/build_variants/ab_$v/libcudasp_amd.so timeout -k 10 200 $P > gpurun_out/r04/ab_${v}_$pass.json
  done
  CUDASP_STREAM_PF_COAL=0 timeout -k 10 200 $P > gpurun_out/r04/ab_coal0_$pass.json
  CUDASP_STREAM_PRIO_US=0 timeout -k 10 200 $P > gpurun_out/r04/ab_prio0_$pass.json
done
echo done
