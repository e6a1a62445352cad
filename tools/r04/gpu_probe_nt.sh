# Round 4: does the streaming kernel's staging evict the ladder's scratch from
# L2/MALL?  Non-temporal stores for the outputs mirror copy (nt_mirror), nt
# row-blob staging (nt_stg), both, and no outputs copy (timing only) against
# the base build, k_scan_multi run right before every streaming run (--prewarm:
# equal clocks); 3M and 9.4M rows, two interleaved passes.
set -e
mkdir -p gpurun_out/r04
for pass in 1 2; do
  echo pass $pass
  for v in base nt_mirror nt_stg nt_both no_outcopy; do
    L=""
    [ $v != base ] && L=$PWD/build_variants/$v/libcudasp_amd.so
    for n in 3000000 9400000; do
      CUDASP_LIB=$L timeout -k 10 200 python tools/stream_probe.py --rows $n --labels 0 --modes all --reps 3 --prewarm > gpurun_out/r04/nt_${v}_${n}_$pass.json
    done
  done
done
echo done
