# Round 3: the table-function host end to end (device feeds) at the configs'
# shapes, thread counts and input formats.  Each run under its own limit.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_e2e_sweep; mkdir -p $O; cd $R
python -c "import bench; open('$O/labels16.bin','wb').write(b''.join(bench.label_keys(16)))"
e2e() { name=$1; shift; timeout -k 10 300 tools/host_e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "e2e $name failed"; tail -5 $O/$name.err; cat $O/$name.json; exit 1; }; python -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', d['tx_per_s']/1e6, d['seconds_all'], d['emitted_equal_planted'], d['launches'], d['harvest_wait_s'], d['thread_call_s_mean'])"; }
e2e cfg4_t8 --rows 32700000 --threads 8 --reps 2
e2e cfg4_t16 --rows 32700000 --threads 16 --reps 2
e2e cfg4_t8_cols --rows 32700000 --threads 8 --reps 2 --input columns
e2e cfg4_t16_cols --rows 32700000 --threads 16 --reps 2 --input columns
e2e cfg2_t8 --rows 1000000 --reps 7
e2e cfg2_t16 --rows 1000000 --threads 16 --reps 7
e2e cfg3_t8 --rows 9400000 --labels 1 --reps 3
e2e cfg3_t16 --rows 9400000 --labels 1 --threads 16 --reps 3
e2e cfg5_t16 --rows 100000000 --labels 16 --labels-file $O/labels16.bin --outputs-max 15 --threads 16
