"""Fill / drain analysis of a rocprofv3 --kernel-trace CSV of bench.py.

Splits the dispatches into bursts (a bench step, or the warmup) separated by
idle gaps, and for each burst reports its span, the summed dispatch time per
kernel, and how long the GPU ran with fewer wave slots requested than it holds:
the wave demand at time t is the sum of grid / 64 over the dispatches running at
t, against the device's slots (CUs x 4 SIMDs x waves per SIMD).  A dispatch's
demand is counted until it ends, so the tail of a launch (its last waves) still
counts as full demand: the figure is a lower bound of the idle slots.

  python tools/timeline.py TRACE.csv [--slots 3072] [--gap-ms 0.5] [--copies COPY_TRACE.csv]

Per burst it also gives the fill and the drain: from the burst's first dispatch
to the first moment the demand reaches the slots, and from the last such moment
to the burst's end.  With --copies (a rocprofv3 --memory-copy-trace CSV) it
adds the copies that overlap the burst: their count and summed time per
direction.
"""
import argparse
import collections
import csv


def bursts(spans, gap_ns):
    out, cur, end = [], [], 0
    for s in sorted(spans):
        if cur and s[0] > end + gap_ns:
            out.append(cur)
            cur = []
        end = max(end, s[1]) if cur else s[1]
        cur.append(s)
    if cur:
        out.append(cur)
    return out


def profile(burst, slots):
    """Time (ms) with wave demand < slots, and with 0 / 1 / 2 / 3 / >= 4 dispatches running."""
    ev = []
    for t0, t1, name, waves in burst:
        ev.append((t0, 1, waves))
        ev.append((t1, -1, waves))
    ev.sort()
    under = 0.0
    by_count = collections.Counter()
    full_first = full_last = None
    demand, running, prev = 0, 0, ev[0][0]
    for t, d, w in ev:
        dt = (t - prev) / 1e6
        if dt > 0:
            if demand < slots:
                under += dt
            elif full_first is None:
                full_first = prev
            if demand >= slots:
                full_last = t
            by_count[min(running, 4)] += dt
        demand += d * w
        running += d
        prev = t
    return under, by_count, full_first, full_last


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--slots", type=int, default=256 * 4 * 3)
    ap.add_argument("--gap-ms", type=float, default=0.5)
    ap.add_argument("--copies")
    a = ap.parse_args()
    copies = []
    if a.copies:
        for r in csv.DictReader(open(a.copies)):
            d = r.get("Direction") or r.get("Kind") or "?"
            copies.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), d))
    spans = []
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"].split("(")[0]
        g = int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0)
        spans.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, max(1, g // 64)))
    for i, b in enumerate(bursts(spans, a.gap_ms * 1e6)):
        t0 = min(s[0] for s in b)
        t1 = max(s[1] for s in b)
        per = collections.defaultdict(float)
        for s in b:
            per[s[2]] += (s[1] - s[0]) / 1e6
        under, by_count, ff, fl = profile(b, a.slots)
        print("burst %d: %d dispatches, span %.2f ms, demand < %d slots for %.2f ms; running 1/2/3/>=4: %s" % (
            i, len(b), (t1 - t0) / 1e6, a.slots, under,
            " / ".join("%.2f" % by_count[k] for k in (1, 2, 3, 4))))
        for k, v in sorted(per.items(), key=lambda kv: -kv[1])[:4]:
            print("    %-40s %8.2f ms summed" % (k[:40], v))
        if ff is not None:
            print("    fill %.2f ms, drain %.2f ms" % ((ff - t0) / 1e6, (t1 - fl) / 1e6))
        cs = [c for c in copies if c[1] >= t0 and c[0] <= t1]
        if cs:
            cper = collections.defaultdict(lambda: [0, 0.0])
            for c in cs:
                cper[c[2]][0] += 1
                cper[c[2]][1] += (c[1] - c[0]) / 1e6
            for k, (n, ms) in sorted(cper.items()):
                print("    %-24s %5d copies %8.2f ms summed" % (k[:24], n, ms))


if __name__ == "__main__":
    main()
