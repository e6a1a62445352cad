# A/B of the slot copies with and without non-temporal stores (CUDASP_TF_NT), null-device host ceiling on the CPU-generated config-4 table.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r05c_nt; mkdir -p $O; cd $R
E=./tools/host_e2e
for pass in 1 2; do
for nt in 0 1; do
  for cfg in "8 rows 16" "8 columns 16" "1 rows 8" "8 rows 12"; do
    set -- $cfg
    MAP=$(python3 -c "print(','.join(['0'] * $1))")
    f=$O/nt${nt}_f$1_$2_t$3_p$pass.json
    CUDASP_TF_NT=$nt CUDASP_TF_DEVICE_MAP=$MAP timeout -k 10 300 $E --null-device --cpu-table --rows 32700000 --threads $3 --batch 300000 --outputs 2 --input $2 --reps 5 > $f 2>/dev/null || { echo "fail $cfg"; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], 'M rows/s %.1f' % (d['tx_per_s']/1e6), 'copy_s %.3f reserve_s %.3f call %.3f' % (d['copy_s'], d['reserve_s'], d['thread_call_s_mean']))" $f
  done
done
done
