# The table-function host's own ceiling: tools/host_e2e
# --null-device over the config-4 table (32.7M rows, 2 outputs/row, 300000-row
# batches): the feeds reserve, copy into the pinned slots and harvest as in a
# real query, but mark every slot done with no device work, so tx/s is what
# the executor threads alone sustain on this box's CPU share.  Thread sweep,
# row chunks (per-row pointers), DuckDB vectors (string_t / list_entry_t as
# the extension now passes them) and Arrow columns, with 1 feed (one GPU) and 8 feeds
# (CUDASP_TF_DEVICE_MAP=0 x 8: the N = 8 host's feeds, one per logical GPU);
# then one real query at the same shape.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_host; mkdir -p $O; cd $R
{ echo "nproc $(nproc)"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; echo "OMP_NUM_THREADS=$OMP_NUM_THREADS"; } > $O/cpus.txt
E=./tools/host_e2e
for feeds in ${FEEDS:-1 8}; do
  MAP=$(python3 -c "print(','.join(['0'] * $feeds))")
  for inp in ${INPUTS:-rows columns vectors}; do
    for t in ${THREADS:-8 16 32 64}; do
      f=$O/null_f${feeds}_${inp}_t$t.json
      CUDASP_TF_DEVICE_MAP=$MAP CUDASP_TF_MODE=stream GPU_MAX_HW_QUEUES=16 timeout -k 10 300 $E --null-device --rows 32700000 --threads $t --batch 300000 --outputs 2 --input $inp --reps 3 > $f || { echo "null $feeds $inp $t failed"; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], 'feeds', d['feeds'], 'M rows/s %.1f' % (d['tx_per_s']/1e6), 'in host calls %.1f' % (d['host_call_tx_per_s']/1e6), 'copy_s %.3f reserve_s %.3f call_s_mean %.3f' % (d['copy_s'], d['reserve_s'], d['thread_call_s_mean']))" $f
    done
  done
done
[ -n "$NO_REAL" ] && exit 0
timeout -k 10 300 $E --rows 32700000 --threads 8 --batch 300000 --outputs 2 --input rows --reps 3 > $O/real_rows_t8.json || { echo "real failed"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('real 8 threads M tx/s %.1f' % (d['tx_per_s']/1e6), 'copy_s %.3f' % d['copy_s'])" $O/real_rows_t8.json
cat $O/cpus.txt
