# Small-launch repeatability on the default stream: two processes sharing the
# GPU (the setting that exposed the stream-ordering race), then the 2-rank bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O; cd $R
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 100 > $O/stress_pytest.log 2>&1 || { tail -20 $O/stress_pytest.log; exit 1; }
tail -1 $O/stress_pytest.log
timeout -k 10 240 python -u tools/stress_values.py --iters ${ITERS:-2000} --seed 2 --tag p0 > $O/stress_p0.log 2>&1 &
P0=$!
timeout -k 10 240 python -u tools/stress_values.py --iters ${ITERS:-2000} --seed 3 --tag p1 > $O/stress_p1.log 2>&1 &
P1=$!
wait $P0; r0=$?; wait $P1; r1=$?
tail -qn1 $O/stress_p0.log $O/stress_p1.log
[ $r0 = 0 ] && [ $r1 = 0 ] || { echo "stress failed ($r0 $r1)"; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --rows 3000000 --steps 2 --dist-backend gloo --no-cpu-baseline > $O/stress_2rank.log 2>&1 || { tail -20 $O/stress_2rank.log; exit 1; }
grep -a -o '"matches.*\|rank [01]:.*' $O/stress_2rank.log
