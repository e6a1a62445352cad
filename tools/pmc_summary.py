"""Turn rocprofv3 --pmc counter-collection CSVs into the JSON summaries under
profiles/ that bench.py reads.

  python tools/pmc_summary.py sq   OUT.json  CSV [CSV ...]   # SQ_* / GRBM_* averages per dispatch
  python tools/pmc_summary.py hbm  OUT.json  FETCH_CSV WRITE_CSV --rows N
  ... --stamp-lib LIB --stamp k_scan_multi=REGEX   # stamp the kernels' machine code

With --stamp-lib, `code_stamp` records the SHA-256 of each named kernel's
machine code in the library the run loaded (tools/codeobj.py); bench.py uses a
summary only while the loaded library's kernel has the same stamp.

`sq`: per kernel, the average of every counter per dispatch (dispatches with the
largest grid only for the scan kernels, so partial batches do not dilute).
`hbm`: per kernel FETCH_SIZE / WRITE_SIZE in KiB per launch; FETCH_SIZE is
doubled as MI355X_MICROARCH.md's HBM section prescribes for gfx950 (it reports
half of wide coalesced reads); hbm_bytes_per_launch = 2 FETCH + WRITE of
k_shared_secret, match_kernel_hbm_bytes_per_launch the same for k_match<false>.
With --probe-rows N (the rows of one k_layout_probe launch, which reads
72 + 8k bytes per row with dword loads and writes 1), the probe calibrates
the counters for this access width: probe_fetch_calibration = bytes read /
raw FETCH_SIZE bytes, probe_hbm_bytes_per_row = the doubled-FETCH + WRITE
traffic per row.
"""
import argparse
import collections
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

SCAN_KERNELS = ("k_shared_secret", "void k_match<false>", "void k_match<true>", "k_layout_probe", "k_scan_multi")


def kernel_key(name):
    """Kernel name without arguments; the full-batch instances of stage A
    (4 rows per thread, CUDASP_ROWS_A) and stage B (6, CUDASP_ROWS_B) keep the
    plain names bench.py looks up, the small-launch instances (rows_a_for,
    rows_b_for) stay separate."""
    k = name.split("(")[0]
    if re.fullmatch(r"void k_scan_multi<\d+(, (true|false))?>", k):  # the multi-batch kernel, any width / schedule
        return "k_scan_multi"
    m = re.fullmatch(r"void k_shared_secret<(\d+)>", k)
    if m:
        k = "k_shared_secret" if m.group(1) == "4" else "k_shared_secret<%s>" % m.group(1)
    m = re.fullmatch(r"void k_match<(true|false), (\d+)(?:, (\d+))?>", k)
    if m:  # stage B: 6 rows per thread (CUDASP_ROWS_B) for full batches; any fixed-base width
        k = "void k_match<%s>" % m.group(1) if m.group(2) == "6" else "void k_match<%s, %s>" % m.groups()[:2]
    return k


def load(paths):
    """{kernel: {counter: [(grid, value) per dispatch]}} (counters summed per dispatch)."""
    per = collections.defaultdict(lambda: collections.defaultdict(dict))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = kernel_key(r["Kernel_Name"])
            key = (p, r["Dispatch_Id"])
            grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
            c = r["Counter_Name"]
            prev = per[k][c].get(key, (grid, 0.0))
            per[k][c][key] = (grid, prev[1] + float(r["Counter_Value"]))
    return per


def averages(per):
    out = {}
    for k, counters in per.items():
        out[k] = {}
        for c, disp in counters.items():
            vals = list(disp.values())
            if k in SCAN_KERNELS:
                gmax = max(g for g, _ in vals)
                vals = [(g, v) for g, v in vals if g == gmax]
            out[k][c] = sum(v for _, v in vals) / len(vals)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["sq", "hbm"])
    ap.add_argument("out")
    ap.add_argument("csvs", nargs="+")
    ap.add_argument("--rows", type=int, default=300000)
    ap.add_argument("--source", default="")
    ap.add_argument("--shape", default="", help="the run's shape (labels, outputs per row, window width)")
    ap.add_argument("--algorithmic-bytes-per-row", type=float, default=89.0)
    ap.add_argument("--probe-rows", type=int, default=0)
    ap.add_argument("--probe-outputs-per-row", type=float, default=2.0)
    ap.add_argument("--multi-rows", type=int, default=0,
                    help="rows of one k_scan_multi launch (cudasp_scan_device_batches) in the profiled run")
    ap.add_argument("--stamp-lib", default="", help="the library the profiled run loaded: its kernels' machine "
                    "code is stamped into the summary (tools/codeobj.py) so bench.py can refuse stale counters")
    ap.add_argument("--stamp", action="append", default=[], metavar="KEY=REGEX",
                    help="kernel to stamp, e.g. k_scan_multi=^_Z12k_scan_multiILi26ELb1EE (repeatable)")
    a = ap.parse_args()
    if a.mode == "sq":
        res = dict(source=a.source, shape=a.shape, rows_per_launch=a.rows, per_kernel=averages(load(a.csvs)))
        if a.multi_rows:
            res["multi_rows_per_launch"] = a.multi_rows
    else:
        fetch = averages(load([a.csvs[0]]))
        write = averages(load([a.csvs[1]]))
        per = {}
        for k in set(fetch) | set(write):
            per[k] = dict(FETCH_SIZE_KiB_per_launch=fetch.get(k, {}).get("FETCH_SIZE", 0.0),
                          WRITE_SIZE_KiB_per_launch=write.get(k, {}).get("WRITE_SIZE", 0.0))

        def hbm(k):
            v = per.get(k)
            return None if v is None else (2 * v["FETCH_SIZE_KiB_per_launch"] + v["WRITE_SIZE_KiB_per_launch"]) * 1024

        res = dict(source=a.source,
                   correction="FETCH_SIZE doubled per MI355X_MICROARCH.md HBM section (gfx950 reports half of wide "
                              "coalesced reads); WRITE_SIZE as reported; units KiB",
                   per_kernel=per, kernel="k_shared_secret", hbm_bytes_per_launch=hbm("k_shared_secret"),
                   match_kernel_hbm_bytes_per_launch=hbm("void k_match<false>"), rows_per_launch=a.rows,
                   algorithmic_bytes_per_launch=a.algorithmic_bytes_per_row * a.rows)
        if a.multi_rows and hbm("k_scan_multi"):
            res.update(multi_rows_per_launch=a.multi_rows,
                       multi_hbm_bytes_per_row=hbm("k_scan_multi") / a.multi_rows)
        pv = per.get("k_layout_probe")
        if pv and a.probe_rows:
            read = a.probe_rows * (72 + 8 * a.probe_outputs_per_row)
            raw = pv["FETCH_SIZE_KiB_per_launch"] * 1024
            res.update(probe_rows=a.probe_rows, probe_read_bytes=read, probe_write_bytes=a.probe_rows,
                       probe_fetch_calibration=read / raw if raw else None,
                       probe_hbm_bytes_per_row=hbm("k_layout_probe") / a.probe_rows)
    if a.stamp_lib:
        import codeobj
        res["code_stamp"] = {key: codeobj.kernel_stamp(a.stamp_lib, rx)
                             for key, rx in (x.split("=", 1) for x in a.stamp)}
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "per_kernel"}, indent=1))
    for k in SCAN_KERNELS:
        if k in res["per_kernel"]:
            print(k, json.dumps(res["per_kernel"][k]))


if __name__ == "__main__":
    main()
