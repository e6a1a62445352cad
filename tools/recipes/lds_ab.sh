# A/B of the odd-multiple table's y coordinates in LDS (LdsY, scan_rows.hpp)
# through the table-function host: tools/host_e2e streaming queries (k_scan_stream)
# at config 4 (32.7M rows) and config 2 (1M rows), each library variant under
# ab/<name>/ loaded through LD_LIBRARY_PATH (host_e2e's RUNPATH yields to it),
# interleaved, three passes on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r06}_ldse2e; mkdir -p $O; cd $R
for pass in $(seq 1 ${PASSES:-3}); do
  for rows in 32700000 1000000; do
    for v in ${VARIANTS:-base y5s3}; do
      f=$O/${v}_r${rows}_$pass.json
      LD_LIBRARY_PATH=$R/ab/$v timeout -k 10 300 ./tools/host_e2e --rows $rows --threads 8 --batch 300000 --outputs 2 --input rows --reps 5 > $f 2> $f.err || { echo "host_e2e $v $rows failed"; tail -5 $f.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1].ljust(26), 'M tx/s %.2f' % (d['tx_per_s']/1e6), 'seconds', d.get('seconds'), 'exact', d.get('exact', d.get('emitted_equal_planted')))" $f
    done
  done
done
