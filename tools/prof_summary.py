"""Summarise a rocprofv3 --kernel-trace CSV: per kernel, dispatch count and
average duration, overall and restricted to full-batch dispatches (those with
the kernel's largest grid, or grid >= --min-grid threads when given), which is
what bench.py's roofline kernel_ms averages."""
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
for r in rows:
    name = r["Kernel_Name"].split("(")[0]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    g = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    per[name].append((g, d))
agg = {}
for name, v in per.items():
    gmin = a.min_grid if a.min_grid else max(g for g, _ in v)
    agg[name] = {"all": [d for _, d in v], "full": [d for g, d in v if g >= gmin], "grid": gmin}
res = {}
for k, v in agg.items():
    res[k] = dict(dispatches=len(v["all"]), avg_ms=sum(v["all"]) / len(v["all"]),
                  full_batch_grid=v["grid"], full_batch_dispatches=len(v["full"]),
                  full_batch_avg_ms=(sum(v["full"]) / len(v["full"])) if v["full"] else None)
res = dict(sorted(res.items(), key=lambda kv: -kv[1]["avg_ms"] * kv[1]["dispatches"]))
print(json.dumps({k: v for k, v in list(res.items())[:6]}, indent=1))
if a.out:
    json.dump(dict(source=a.trace, full_batch="largest grid per kernel" if not a.min_grid else
                   "grid >= %d threads" % a.min_grid, kernels=res), open(a.out, "w"), indent=1)
