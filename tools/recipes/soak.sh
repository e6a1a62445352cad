# Randomized soak of the table-function host (tools/soak_host.py): seeded random
# query shapes for SOAK_MIN minutes, every query's emitted rows == planted and
# each run's 512-row sample equal to the C oracle.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r05}_soak; mkdir -p $O; cd $R
timeout -k 10 $(( ${SOAK_MIN:-8} * 60 + 300 )) python -u tools/soak_host.py --minutes ${SOAK_MIN:-8} --seed ${SOAK_SEED:-1} --out $O/soak.jsonl > $O/soak.log 2>&1 || { tail -5 $O/soak.log; exit 1; }
tail -1 $O/soak.log
