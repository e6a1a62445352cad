# Streaming feeds at configs 2 and 3: ramp off, smaller slots, rows per
# thread, against the defaults (interleaved, one box).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_stream_knobs; mkdir -p $O; cd $R
e2e() { name=$1; shift; timeout -k 10 300 env $ENVV tools/host_e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "e2e $name failed"; tail -5 $O/$name.err; cat $O/$name.json; exit 1; }; python -c "import json,sys; d=json.load(open('$O/$name.json')); print('$name', round(d['tx_per_s']/1e6,1), d['seconds_all'], d['emitted_equal_planted'], d['launches'], d.get('streaming_feeds'), d['thread_done_s_min'], d['thread_done_s_max'])"; }
for rep in 1 2; do
  for v in default ramp0 b150k b100k rows4 rows5; do
    ENVV="CUDASP_TF_MODE=stream"; B=300000
    case $v in
      ramp0) ENVV="$ENVV CUDASP_TF_RAMP=0";;
      b150k) B=150000;;
      b100k) B=100000;;
      rows4) ENVV="$ENVV CUDASP_MULTI_ROWS=4";;
      rows5) ENVV="$ENVV CUDASP_MULTI_ROWS=5";;
    esac
    e2e cfg2_${v}_$rep --rows 1000000 --reps 5 --batch $B
    e2e cfg3_${v}_$rep --rows 9400000 --labels 1 --reps 3 --batch $B
  done
done
echo all-done
