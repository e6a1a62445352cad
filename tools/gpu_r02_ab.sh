# Round-2 A/Bs on one MI355X:
#  1. scratch traffic: the product build vs CUDASP_AB_SCRATCH_ALIAS=1024 (per-row
#     scratch folded into an L2-sized region; timing only), asymptotic 3M-row
#     stage timing, 2 rounds, plus one FETCH_SIZE pass of each;
#  2. end-to-end (table-function host) at 22- vs 26-bit fixed-base windows,
#     3 runs each, 16 hardware queues;
#  3. end-to-end at 4 hardware queues, 6 runs under a rocprofv3 kernel trace
#     (the bimodality of round 1).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
step() { local name=$1; shift; timeout -k 10 "$@" > $O/$name.log 2>&1 || { echo "$name failed"; tail -30 $O/$name.log; exit 1; }; tail -1 $O/$name.log | cut -c1-220; }
cd $R
for round in 1 2; do
  for v in base alias1024; do
    CUDASP_LIB=$R/build_variants/libcudasp_$v.so step ab_${v}_$round 200 python tools/stage_timing.py 3000000 0 5
  done
done
cd /tmp && export TMPDIR=/tmp
for v in base alias1024; do
  CUDASP_LIB=$R/build_variants/libcudasp_$v.so step pmc_fetch_$v 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$v -o f -- python3 $R/tools/stage_timing.py 300000 0 3
done
cd $R
for i in 1 2 3; do
  for w in 22 26; do
    GPU_MAX_HW_QUEUES=16 CUDASP_FB_BITS=$w step e2e_w${w}_$i 120 tools/host_e2e 32700000 8 300000 0 2 rows
  done
done
cd /tmp
for i in 1 2 3 4 5 6; do
  GPU_MAX_HW_QUEUES=4 CUDASP_FB_BITS=26 step e2e_q4_$i 180 rocprofv3 --kernel-trace --output-format csv -d $O/e2e_q4_$i -o t -- $R/tools/host_e2e 32700000 8 300000 0 2 rows
done
echo all-done
