"""Summarise a rocprofv3 --kernel-trace CSV: per kernel, dispatch count and
average duration, overall and restricted to full-batch dispatches (those with
the kernel's largest grid, or grid >= --min-grid threads when given), and the
full-batch dispatches that ran alone on the GPU (overlapping no other
dispatch), which is what bench.py's roofline kernel_ms averages."""
import argparse
import collections
import csv
import json

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--min-grid", type=int, default=0, help="0: the kernel's largest grid")
ap.add_argument("--out")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
per = collections.defaultdict(list)
spans = []
for r in rows:
    name = r["Kernel_Name"].split("(")[0]
    t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    d = (t1 - t0) / 1e6
    g = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    per[name].append((g, d))
    spans.append((t0, t1, name, g))
# Exclusive dispatches: those that overlap no other dispatch in time (the
# single-stream pass bench.py runs after its timed steps; its roofline
# kernel_ms averages these).
spans.sort()
excl = collections.defaultdict(list)
prev_end = -1  # latest end of the dispatches that started earlier
for i, (t0, t1, name, g) in enumerate(spans):
    next_start = spans[i + 1][0] if i + 1 < len(spans) else None
    if prev_end <= t0 and (next_start is None or next_start >= t1):
        excl[name].append((g, (t1 - t0) / 1e6))
    prev_end = max(prev_end, t1)
agg = {}
for name, v in per.items():
    gmin = a.min_grid if a.min_grid else max(g for g, _ in v)
    agg[name] = {"all": [d for _, d in v], "full": [d for g, d in v if g >= gmin], "grid": gmin}
res = {}
for k, v in agg.items():
    ex = [d for g, d in excl.get(k, []) if g >= v["grid"]]
    res[k] = dict(dispatches=len(v["all"]), avg_ms=sum(v["all"]) / len(v["all"]),
                  full_batch_grid=v["grid"], full_batch_dispatches=len(v["full"]),
                  full_batch_avg_ms=(sum(v["full"]) / len(v["full"])) if v["full"] else None,
                  exclusive_full_batch_dispatches=len(ex),
                  exclusive_full_batch_avg_ms=(sum(ex) / len(ex)) if ex else None)
res = dict(sorted(res.items(), key=lambda kv: -kv[1]["avg_ms"] * kv[1]["dispatches"]))
print(json.dumps({k: v for k, v in list(res.items())[:6]}, indent=1))
if a.out:
    json.dump(dict(source=a.trace, full_batch="largest grid per kernel" if not a.min_grid else
                   "grid >= %d threads" % a.min_grid, kernels=res), open(a.out, "w"), indent=1)
