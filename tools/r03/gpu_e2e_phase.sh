# Round 3: where the executor threads' time goes (reserve / copy / launch /
# harvest wait) at config 4, pinned-allocation flags A/B, thread counts.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_e2e_phase; mkdir -p $O; cd $R
e2e() { name=$1; shift; timeout -k 10 300 tools/host_e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "e2e $name failed"; tail -5 $O/$name.err; cat $O/$name.json; exit 1; }; python -c "
import json; d=json.load(open('$O/$name.json')); print('$name', round(d['tx_per_s']/1e6,1), d['seconds_all'], d['emitted_equal_planted'], {k: d[k] for k in ('harvest_wait_s','reserve_s','copy_s','launch_s','thread_call_s_mean')})"; }
nproc; grep -m1 "model name" /proc/cpuinfo; numactl -H 2>/dev/null | head -3 || true
for p in default noncoherent coherent; do CUDASP_TF_PINNED=$p e2e pin_$p --rows 32700000 --reps 3; done
e2e t4 --rows 32700000 --reps 3 --threads 4
e2e t12 --rows 32700000 --reps 3 --threads 12
e2e t16 --rows 32700000 --reps 3 --threads 16
e2e t16_cols --rows 32700000 --reps 3 --threads 16 --input columns
