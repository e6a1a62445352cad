# LDS bank conflicts of k_scan_multi<26,true> with the odd-multiple y table in
# LDS (config 4, one step): SQ_INSTS_LDS, SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE
# (rocprofv3 --pmc, one pass), summarised per kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${MEASURE_TAG:-r06}_lds; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
C="python3 $R/bench.py --no-cpu-baseline --no-e2e --no-cold-start --no-layout-probe --idle-samples 0 --steps 1 --warmup 0 --exclusive-batches 0"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU --output-format csv -d $O/pmc -o lds -- $C > $O/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc.log; exit 1; }
cd $R
python3 - $O <<'PY'
import csv, glob, sys, collections
o = sys.argv[1]
f = (glob.glob(o + "/pmc/*counter_collection.csv") + glob.glob(o + "/pmc/*/*counter_collection.csv"))[0]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "k_scan_multi" not in k and "k_shared_secret" not in k:
        continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(k, r["Counter_Name"])] += 1
for k, c in agg.items():
    print(k[:60], {x: c[x] for x in sorted(c)})
    if c.get("SQ_LDS_IDX_ACTIVE"):
        print("  bank-conflict cycles / LDS-active cycles = %.4f" % (c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"]))
PY
