"""The VALU ceiling of k_scan_multi's own instruction mix, from rocprofv3
PMC passes (tools/recipes/valu_ceiling.sh writes the directory this reads).

Per dispatch (median over a kernel's dispatches):
  cycles C   GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs)
  clock f    C / kernel-trace duration (same dispatch ordinal, separate
             --kernel-trace run)
  U          4 x SQ_INSTS_VALU / (C x SIMDs): VALU issue in units of one
             wave-instruction per 4 SIMD cycles.  (SQ_ACTIVE_INST_VALU reads
             exactly one quad-cycle per VALU instruction on gfx950 -- the
             calibration shows it -- so it is an instruction count here, not
             the pipe's occupancy, and the ceiling has to be measured.)

The ceiling is measured, not assumed: issue-bound loops with no memory
traffic -- one opcode each (tools/microbench/int_throughput: VOP3 ops read
U ~ 0.95-0.97, v_add_u32 1.70, v_addc with an SGPR carry-in 0.66) and the
kernel's own group operations (tools/microbench/group_ops: the ladder's
doubling and mixed addition, register-resident, 1-4 waves per SIMD).  The
ladder mix (126 doublings x 893 + 39 mixed additions x 1576 VALU, ~88% of
k_scan_multi's instructions) at 3 waves per SIMD -- the kernel's occupancy --
gives U_ladder, the issue rate this instruction mix sustains when nothing
else limits it.  k_scan_multi's fraction of that ceiling is U / U_ladder
(the other ~12% of its instructions -- inversion, SHA-256, stage B -- are
taken at the ladder's rate), and the ceiling in wave-instructions/s is
achieved / fraction (x 2.4 GHz / f at the peak clock).

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


def key_of(r):
    """Kernel name without arguments; the calibration loops also by grid
    (group_ops runs one kernel at 1..4 waves per SIMD)."""
    k = kernel_key(r["Kernel_Name"])
    if k.startswith("void loop<"):
        k += " grid %s" % (r.get("Grid_Size") or r.get("Grid_Size_X"))
    return k


def counters(path_glob):
    """{kernel: [ {counter: value} per dispatch, in dispatch order ]}."""
    out = collections.defaultdict(dict)
    for p in glob.glob(path_glob):
        for r in csv.DictReader(open(p)):
            k = key_of(r)
            d = int(r["Dispatch_Id"])
            e = out[k].setdefault(d, collections.defaultdict(float))
            e[r["Counter_Name"]] += float(r["Counter_Value"])
    return {k: [v[d] for d in sorted(v)] for k, v in out.items()}


def durations(path_glob):
    out = collections.defaultdict(list)
    for p in glob.glob(path_glob):
        rows = sorted(csv.DictReader(open(p)), key=lambda r: int(r["Dispatch_Id"]))
        for r in rows:
            out[key_of(r)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
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
                       U=4 * c["SQ_INSTS_VALU"] / (cyc * SIMDS) if cyc else None, c=4 * a / c["SQ_INSTS_VALU"],
                       any_U=4 * c.get("SQ_ACTIVE_INST_ANY", 0.0) / (cyc * SIMDS) if cyc else None,
                       busy=c.get("SQ_BUSY_CYCLES"), wave_cycles=c.get("SQ_WAVE_CYCLES"),
                       int64=c.get("SQ_INSTS_VALU_INT64"), int32=c.get("SQ_INSTS_VALU_INT32"))
            if i < len(t) and t[i] > 0:
                row["seconds"] = t[i]
                row["clock_hz"] = cyc / t[i]
                row["valu_per_s"] = c["SQ_INSTS_VALU"] / t[i]
            rows.append(row)
        if rows:
            med = {key: statistics.median([r[key] for r in rows if r.get(key) is not None])
                   for key in set().union(*rows) if any(r.get(key) is not None for r in rows)}
            med["dispatches"] = len(rows)
            res[k] = med
    return res


# Stage A's ladder for the bench's scan key after the digit search: 126
# doublings and 39 mixed additions of 893 and 1576 VALU;
# ~88% of k_scan_multi's instructions.
LADDER = ((126 * 893, "dbl"), (39 * 1576, "madd"))
# rows of one k_scan_multi launch in tools/recipes/pmc.sh's scan passes, by label count
ROWS = {0: 32_700_000, 1: 9_400_000, 16: 3_000_000}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json", default="")
    ap.add_argument("--stamp-lib", default="", help="the library the scan passes loaded: stamp k_scan_multi's "
                    "machine code into the JSON (tools/codeobj.py)")
    ap.add_argument("--fb-bits", type=int, default=26)
    a = ap.parse_args()
    d = a.dir
    out = {}
    mb = analyse(counters(d + "/mb_sq/*counter_collection.csv"), counters(d + "/mb_grbm/*counter_collection.csv"),
                 durations(d + "/mb_kt/*kernel_trace.csv"), skip_first=True)
    print("one-opcode loops (int_throughput; U = 4 x VALU instructions / SIMD cycles, 1.0 = one per 4 cycles):")
    for k, r in sorted(mb.items()):
        print("  %-24s U %.3f  clock %.2f GHz" % (k, r["U"], r.get("clock_hz", 0) / 1e9))
    out["one_opcode_loops"] = {k: dict(U=r["U"], clock_hz=r.get("clock_hz")) for k, r in mb.items()}
    go = analyse(counters(d + "/go_sq/*counter_collection.csv"), counters(d + "/go_grbm/*counter_collection.csv"),
                 durations(d + "/go_kt/*kernel_trace.csv"), skip_first=False)
    names = {"void loop<0>": "dbl", "void loop<1>": "madd", "void loop<2>": "mul", "void loop<3>": "sqr",
             "void loop<20>": "ydbl", "void loop<21>": "yadd"}
    print("group-operation loops (group_ops: register-resident, issue-bound; by waves per SIMD):")
    gu = {}
    for k, r in sorted(go.items()):
        base, grid = k.split(" grid ")
        w = int(grid) // (256 * 256)
        nm = names.get(base, base)
        gu[(nm, w)] = r["U"]
        print("  %-6s %d waves/SIMD  U %.3f  int64 share %.2f  clock %.2f GHz"
              % (nm, w, r["U"], r.get("int64", 0) / r["valu"] if r.get("int64") else 0, r.get("clock_hz", 0) / 1e9))
    out["group_op_loops"] = {"%s_w%d" % k: v for k, v in gu.items()}
    u_ladder = None
    # the ladder's own operations (gej_double_neg_yh / gej_add_ge_yh, the Yh
    # form k_scan_multi runs) when measured, else the plain forms
    dbl, add = ("ydbl", "yadd") if ("ydbl", 3) in gu and ("yadd", 3) in gu else ("dbl", "madd")
    if (dbl, 3) in gu and (add, 3) in gu:
        tot = sum(n for n, _ in LADDER)
        u_ladder = tot / sum(n / gu[(dbl if op == "dbl" else add, 3)] for n, op in LADDER)
        print("ladder mix at 3 waves/SIMD (126 %s x 893 + 39 %s x 1576 VALU): U %.3f" % (dbl, add, u_ladder))
    out["ladder_ops"] = [dbl, add]
    # The kernel's other instructions (inversions' divsteps, SHA-256, stage B,
    # compares) issue at most at the 4-byte-encoded VOP2 rate (v_add_u32,
    # the fastest one-opcode loop); with the ladder's share of the kernel's
    # per-row VALU (the bench key's 126 doublings and 39 additions over the
    # measured count), 1 / (share / U_ladder + (1 - share) / U_vop2) bounds
    # the issue rate of the whole mix from above.
    u_vop2 = max((r["U"] for r in mb.values()), default=None)
    out["vop2_U"] = u_vop2
    out["ladder_mix_U"] = u_ladder
    for L in (0, 1, 16):
        sc = analyse(counters(d + "/scan_sq_L%d/*counter_collection.csv" % L),
                     counters(d + "/scan_grbm_L%d/*counter_collection.csv" % L),
                     durations(d + "/scan_kt_L%d/*kernel_trace.csv" % L), skip_first=False)
        r = sc.get("k_scan_multi")
        if not r:
            continue
        f = r.get("clock_hz")
        ach = r.get("valu_per_s")
        frac = r["U"] / u_ladder if u_ladder else None
        ceiling = ach / frac if (ach and frac) else None
        print("k_scan_multi, %d labels: U %.3f; clock %.2f GHz; achieved %.3e wave-instr/s; frac of the ladder-mix "
              "ceiling %s; ceiling %s wave-instr/s at this clock, %s at 2.4 GHz"
              % (L, r["U"], (f or 0) / 1e9, ach or 0, "%.3f" % frac if frac else "-",
                 "%.3e" % ceiling if ceiling else "-", "%.3e" % (ceiling * PEAK_HZ / f) if (ceiling and f) else "-"))
        per_row = r["valu"] * 64.0 / ROWS.get(L, 1) if ROWS.get(L) else None
        share = sum(n for n, _ in LADDER) / per_row if per_row else None
        bound = (1.0 / (share / u_ladder + (1 - share) / u_vop2)) if (share and u_ladder and u_vop2) else None
        if bound:
            print("  ladder share of its VALU %.3f (of %.0f per row); mix upper bound U %.3f; kernel at %.3f of it"
                  % (share, per_row, bound, r["U"] / bound))
        out["k_scan_multi_L%d" % L] = dict(U=r["U"], clock_hz=f, achieved_wave_instr_per_s=ach,
                                           valu_per_row=per_row, ladder_share=share, mix_U_upper_bound=bound,
                                           frac_of_mix_upper_bound=(r["U"] / bound) if bound else None,
                                           frac_of_ladder_mix_ceiling=frac,
                                           mix_ceiling_wave_instr_per_s=ceiling,
                                           mix_ceiling_at_peak_clock=(ceiling * PEAK_HZ / f) if (ceiling and f) else None,
                                           valu_per_dispatch=r["valu"], seconds=r.get("seconds"))
    if a.stamp_lib:
        import codeobj
        out["code_stamp"] = dict(k_scan_multi=codeobj.kernel_stamp(a.stamp_lib, codeobj.multi_pattern(a.fb_bits)))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
