"""Analyse a k_scan_stream event trace (measurement builds only).

A library built with -DCUDASP_STREAM_TRACE=1 appends every query's kernel
events to $CUDASP_STREAM_TRACE_FILE at cudasp_stream_finish (scan_kernels.hip,
StreamTraceEv: u64 t, u64 a, u32 wave, kind, b, c; t in 100 MHz wall-clock
ticks).  This prints, for the chosen query: when batches were mirrored and
completed, how many worker waves were inside an iteration over time, the
claim sizes, per-iteration durations by piece size and the tail.

  python tools/stream_trace.py gpurun_out/trace.bin [--query -1] [--bin-us 250]
"""
import argparse
import collections
import json
import sys

import numpy as np

EV = np.dtype([("t", "<u8"), ("a", "<u8"), ("wave", "<u4"), ("kind", "<u4"), ("b", "<u4"), ("c", "<u4")])
START, CLAIM, PIECE, ITER_END, EXIT, PUB, DONE = range(1, 8)


def load(path):
    raw = open(path, "rb").read()
    out, off = [], 0
    while off + 4 <= len(raw):
        n = int(np.frombuffer(raw, "<u4", 1, off)[0])
        off += 4
        q = np.frombuffer(raw, EV, n, off)
        off += n * EV.itemsize
        if (q["wave"] != 0xFFFFFFFF).any():  # a record of host events alone: a finish without a query
            out.append(q)
    return out


def simd_key(a):
    hw, xcc = a & 0xFFFFFFFF, a >> 32
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    return (int(xcc), int(se), int(sh), int(cu), int(simd))


HOST_NAMES = {101: "publish", 102: "launch", 103: "finish:closed", 104: "finish:waited", 105: "finish:exited",
              106: "finish:end", 110: "tf_init", 111: "flush", 112: "harvested", 113: "flush:harvested",
              114: "thread_final"}


def host_events(hev, dev_pubs):
    """Host events on the kernel's clock: a host publish of batch s is
    mirrored by the first poller pass with seen <= s < pub, so the smallest
    (GPU - host) difference over the batches is the clock offset (plus the
    poller's ~1 us pass)."""
    ht = hev["t"].astype(np.int64) / 1000.0  # us
    offs = []
    for e, t in zip(hev, ht):
        if e["kind"] != 101:
            continue
        seq = int(e["b"])
        for g_us, (b_hi, b_lo) in dev_pubs:
            if b_lo <= seq < b_hi:
                offs.append(g_us - t)
                break
    if not offs:
        return [], None
    off = min(offs)
    out = [(round(float(t + off), 1), HOST_NAMES.get(int(e["kind"]), str(int(e["kind"]))), int(e["a"]), int(e["b"]))
           for e, t in zip(hev, ht)]
    return out, off


def analyse(ev, bin_us=250.0):
    hev = ev[ev["wave"] == 0xFFFFFFFF]
    ev = ev[ev["wave"] != 0xFFFFFFFF]
    ev = np.sort(ev, order="t")
    t0 = int(ev["t"].min())
    us = (ev["t"].astype(np.int64) - t0) / 100.0
    k = ev["kind"]
    res = {"events": int(len(ev))}
    starts = ev[k == START]
    exits = ev[k == EXIT]
    res["waves"] = int(len(starts))
    res["span_us"] = round(float(us.max()), 1)
    pubs = [(round(float(u), 1), int(e["b"]), int(e["a"])) for u, e in zip(us[k == PUB], ev[k == PUB])]
    res["pubs_us_batches_wr"] = pubs
    dev_pubs = [(float(u), (int(e["b"]), int(e["c"]))) for u, e in zip(us[k == PUB], ev[k == PUB])]
    if len(hev):
        hl, _ = host_events(hev, dev_pubs)
        res["host_us"] = [h for h in hl if h[1] != "harvested"]
        res["host_harvested_us"] = [(h[0], h[3], round(h[2] / 1000.0, 1)) for h in hl if h[1] == "harvested"]
    dones = [(round(float(u), 1), int(e["b"])) for u, e in zip(us[k == DONE], ev[k == DONE])]
    res["done_us_batch"] = dones
    # per wave: iterations (PIECE .. ITER_END)
    by_wave = collections.defaultdict(list)
    for u, e in zip(us, ev):
        if e["kind"] in (PIECE, ITER_END, START, EXIT, CLAIM):
            by_wave[int(e["wave"])].append((float(u), int(e["kind"]), int(e["a"]), int(e["b"]), int(e["c"])))
    iters = []  # (wave, start, end, count, count_p, count_q)
    place = {}
    for w, lst in by_wave.items():
        cur = None
        for u, kind, a, b, c in lst:
            if kind == START:
                place[w] = simd_key(a)
            elif kind == PIECE:
                cur = (u, b, c & 0xFF, c >> 8)
            elif kind == ITER_END and cur is not None:
                iters.append((w, cur[0], u, cur[1], cur[2], cur[3]))
                cur = None
    it = np.array([(s, e, c, p, q) for _, s, e, c, p, q in iters]) if iters else np.zeros((0, 5))
    span = res["span_us"]
    nb = int(span // bin_us) + 1
    busy = np.zeros(nb)
    for s, e, *_ in it:
        b0, b1 = int(s // bin_us), int(e // bin_us)
        for b in range(b0, b1 + 1):
            lo, hi = max(s, b * bin_us), min(e, (b + 1) * bin_us)
            if hi > lo:
                busy[b] += (hi - lo) / bin_us
    res["bin_us"] = bin_us
    res["busy_waves_per_bin"] = [round(float(x)) for x in busy]
    rows_started = np.zeros(nb)
    for s, e, c, *_ in it:
        rows_started[min(int(s // bin_us), nb - 1)] += c
    res["wave_rows_started_per_bin"] = [int(x) for x in rows_started]
    # durations of iterations by (count, count_p) for work iterations
    dur = collections.defaultdict(list)
    for s, e, c, p, q in it:
        dur[(int(c), int(p))].append(e - s)
    res["iter_us_by_count_countp"] = {f"{c},{p}": [len(v), round(float(np.median(v)), 1), round(float(np.max(v)), 1)]
                                      for (c, p), v in sorted(dur.items())}
    claims = ev[k == CLAIM]
    res["claims"] = int(len(claims))
    res["claim_rows_hist"] = {int(x): int(n) for x, n in zip(*np.unique(claims["b"], return_counts=True))}
    # the tail: iterations still running in the last 1 ms
    last = float(it[:, 1].max()) if len(it) else 0.0
    res["last_iter_end_us"] = round(last, 1)
    tail = [(w, round(s, 1), round(e, 1), int(c), int(p)) for w, s, e, c, p, q in iters if e > last - 1000]
    tail.sort(key=lambda x: x[2])
    res["tail_iters_last_1ms"] = len(tail)
    res["tail_last_20"] = tail[-20:]
    # per SIMD: summed iteration time of its waves
    simd_busy = collections.defaultdict(float)
    simd_last = collections.defaultdict(float)
    for w, s, e, c, p, q in iters:
        key = place.get(w)
        simd_busy[key] += e - s
        simd_last[key] = max(simd_last[key], e)
    if simd_last:
        ends = np.array(list(simd_last.values()))
        res["simds"] = len(simd_last)
        res["simd_last_end_us_pct"] = {p: round(float(np.percentile(ends, p)), 1) for p in (0, 10, 50, 90, 99, 100)}
    res["exits_us_pct"] = {p: round(float(np.percentile(us[k == EXIT], p)), 1) for p in (0, 50, 100)} if len(exits) else {}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--query", type=int, default=-1)
    ap.add_argument("--bin-us", type=float, default=250.0)
    a = ap.parse_args()
    qs = load(a.path)
    if not qs:
        sys.exit("no queries in trace")
    res = analyse(qs[a.query], a.bin_us)
    res["queries"] = len(qs)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
