# Round 3: GPU suite, then the table-function host end to end at the
# configs' shapes (device feeds).  Each step under its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r03_tests_e2e; mkdir -p $O; cd $R
K=(); [ -n "$1" ] && K=(-k "$1")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" > $O/gpu_tests.log 2>&1 || { grep -E "PASS|FAIL|Error|error" $O/gpu_tests.log | tail -30; tail -60 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
python -c "import bench; open('$O/labels16.bin','wb').write(b''.join(bench.label_keys(16)))"
e2e() { name=$1; shift; timeout -k 10 300 tools/host_e2e "$@" > $O/$name.json 2> $O/$name.err || { echo "e2e $name failed"; tail -5 $O/$name.err; cat $O/$name.json; exit 1; }; cat $O/$name.json; }
e2e cfg2 --rows 1000000 --reps 5
e2e cfg3 --rows 9400000 --labels 1 --reps 3
e2e cfg4 --rows 32700000
e2e cfg5 --rows 100000000 --labels 16 --labels-file $O/labels16.bin --outputs-max 15
