"""The VALU ceiling of a kernel's own instruction mix, from rocprofv3 PMC
passes (tools/r03/gpu_valu_ceiling.sh writes the directory this reads).

For every dispatch of the calibration microbenchmark
(tools/microbench/int_throughput: issue-bound loops of one opcode each) and
of k_scan_multi it reports, per kernel (median over its dispatches):

  cycles C        GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs)
  clock f         C / kernel-trace duration (the same dispatch ordinal of a
                  separate --kernel-trace run)
  U               VALU busy fraction = 4 SQ_ACTIVE_INST_VALU / (C x SIMDs):
                  SQ_ACTIVE_INST_VALU counts quad-cycles in which a wave issues
                  a VALU instruction (MI355X_MICROARCH.md, PMC units)
  c               SIMD cycles per VALU wave-instruction = 4 A / SQ_INSTS_VALU

The calibration loops saturate the VALU by construction, so their U says what
the counter reads at the issue limit (U_sat); a kernel's fraction of its own
mix ceiling is U / U_sat -- the share of SIMD cycles its VALU instructions
could have filled that they did fill, at the clock it ran.  The ceiling in
wave-instructions/s is then achieved / (U / U_sat), and at the 2.4 GHz peak
clock ceiling x 2.4 GHz / f.

  python tools/valu_ceiling.py DIR [--json OUT]
"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import kernel_key  # noqa: E402

SIMDS = 256 * 4
XCDS = 8
PEAK_HZ = 2.4e9


def counters(path_glob):
    """{kernel: [ {counter: value} per dispatch, in dispatch order ]}."""
    out = collections.defaultdict(dict)
    for p in glob.glob(path_glob):
        for r in csv.DictReader(open(p)):
            k = kernel_key(r["Kernel_Name"])
            d = int(r["Dispatch_Id"])
            e = out[k].setdefault(d, collections.defaultdict(float))
            e[r["Counter_Name"]] += float(r["Counter_Value"])
    return {k: [v[d] for d in sorted(v)] for k, v in out.items()}


def durations(path_glob):
    out = collections.defaultdict(list)
    for p in glob.glob(path_glob):
        rows = sorted(csv.DictReader(open(p)), key=lambda r: int(r["Dispatch_Id"]))
        for r in rows:
            out[kernel_key(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return out


def analyse(sq, grbm, kt, skip_first):
    res = {}
    for k, disp in sq.items():
        g = grbm.get(k, [])
        t = kt.get(k, [])
        rows = []
        for i, c in enumerate(disp):
            if skip_first and i == 0:
                continue
            if i >= len(g) or "SQ_INSTS_VALU" not in c or c["SQ_INSTS_VALU"] == 0:
                continue
            cyc = g[i]["GRBM_GUI_ACTIVE"] / XCDS
            a = c.get("SQ_ACTIVE_INST_VALU", 0.0)
            row = dict(cycles=cyc, valu=c["SQ_INSTS_VALU"], active_valu=a,
                       U=4 * a / (cyc * SIMDS) if cyc else None, c=4 * a / c["SQ_INSTS_VALU"],
                       any_U=4 * c.get("SQ_ACTIVE_INST_ANY", 0.0) / (cyc * SIMDS) if cyc else None,
                       busy=c.get("SQ_BUSY_CYCLES"), wave_cycles=c.get("SQ_WAVE_CYCLES"))
            if i < len(t) and t[i] > 0:
                row["seconds"] = t[i]
                row["clock_hz"] = cyc / t[i]
                row["valu_per_s"] = c["SQ_INSTS_VALU"] / t[i]
            rows.append(row)
        if rows:
            med = {key: statistics.median([r[key] for r in rows if r.get(key) is not None])
                   for key in rows[0] if any(r.get(key) is not None for r in rows)}
            med["dispatches"] = len(rows)
            res[k] = med
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    d = a.dir
    mb = analyse(counters(d + "/mb_sq/*counter_collection.csv"), counters(d + "/mb_grbm/*counter_collection.csv"),
                 durations(d + "/mb_kt/*kernel_trace.csv"), skip_first=True)
    print("calibration (issue-bound one-opcode loops):")
    for k, r in sorted(mb.items()):
        print("  %-24s U %.3f  cycles/VALU-instr %.2f  clock %.2f GHz" % (k, r["U"], r["c"], r.get("clock_hz", 0) / 1e9))
    sat = [r["U"] for r in mb.values() if r.get("U")]
    u_sat = max(sat) if sat else 1.0
    print("U at saturation (max over the loops): %.3f" % u_sat)
    out = dict(u_saturated=u_sat, calibration={k: dict(U=r["U"], cycles_per_valu=r["c"],
                                                        clock_hz=r.get("clock_hz")) for k, r in mb.items()})
    for L in (0, 16):
        sc = analyse(counters(d + "/scan_sq_L%d/*counter_collection.csv" % L),
                     counters(d + "/scan_grbm_L%d/*counter_collection.csv" % L),
                     durations(d + "/scan_kt_L%d/*kernel_trace.csv" % L), skip_first=False)
        r = sc.get("k_scan_multi")
        if not r:
            continue
        frac = r["U"] / u_sat
        ach = r.get("valu_per_s")
        ceiling = ach / frac if ach else None
        f = r.get("clock_hz")
        print("k_scan_multi, %d labels: U %.3f -> %.3f of the mix ceiling; cycles/VALU-instr %.2f; clock %.2f GHz; "
              "achieved %.3e wave-instr/s; ceiling %.3e at this clock, %.3e at 2.4 GHz"
              % (L, r["U"], frac, r["c"], (f or 0) / 1e9, ach or 0, ceiling or 0,
                 (ceiling * PEAK_HZ / f) if (ceiling and f) else 0))
        out["k_scan_multi_L%d" % L] = dict(U=r["U"], frac_of_mix_ceiling=frac, cycles_per_valu=r["c"], clock_hz=f,
                                           achieved_wave_instr_per_s=ach, mix_ceiling_wave_instr_per_s=ceiling,
                                           mix_ceiling_at_peak_clock=(ceiling * PEAK_HZ / f) if (ceiling and f) else None,
                                           any_issue_U=r.get("any_U"), valu_per_dispatch=r["valu"],
                                           seconds=r.get("seconds"))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
