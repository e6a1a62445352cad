"""Summarise a rocprofv3 --kernel-trace CSV: per kernel, dispatch count and
average duration, overall and restricted to full-batch dispatches (grid size
>= --min-grid threads), which is what bench.py's roofline kernel_ms averages."""
import argparse
import collections
import csv
import json

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--min-grid", type=int, default=299_000)
ap.add_argument("--out")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
agg = collections.defaultdict(lambda: {"all": [], "full": []})
for r in rows:
    name = r["Kernel_Name"].split("(")[0]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    g = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
    agg[name]["all"].append(d)
    if g >= a.min_grid:
        agg[name]["full"].append(d)
res = {}
for k, v in agg.items():
    res[k] = dict(dispatches=len(v["all"]), avg_ms=sum(v["all"]) / len(v["all"]),
                  full_batch_dispatches=len(v["full"]),
                  full_batch_avg_ms=(sum(v["full"]) / len(v["full"])) if v["full"] else None)
res = dict(sorted(res.items(), key=lambda kv: -kv[1]["avg_ms"] * kv[1]["dispatches"]))
print(json.dumps({k: v for k, v in list(res.items())[:6]}, indent=1))
if a.out:
    json.dump(dict(source=a.trace, min_grid_threads=a.min_grid, kernels=res), open(a.out, "w"), indent=1)
