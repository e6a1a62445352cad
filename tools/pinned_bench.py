"""Throughput of cudasp_amd.PinnedTable (measurement only): bench.py's synthetic
table (T_g = (s0 + g) G, splitmix64 outputs, planted base and label matches)
built on the GPU, brought to host memory as an Arrow table (txid = BE64(g)
padded to 32 bytes, height, tweak_key fixed_size_binary(64), outputs
list<int64>), pinned once (PinnedTable), then scanned `--reps` times in place:
one streaming kernel per scan reads every batch from pinned host memory, no
host copy per query.  Each scan must find exactly the planted rows.

  python tools/pinned_bench.py --rows 32700000 --reps 3 [--labels 1] [--outputs-max 15]

Prints one JSON line: the pin (one-time copy) seconds, each scan's seconds and
tx/s, and the median.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "duckdb-cudasp-extension_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32_700_000)
    ap.add_argument("--batch-size", type=int, default=300_000)
    ap.add_argument("--labels", type=int, default=0)
    ap.add_argument("--outputs-max", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--probe", action="store_true", help="diagnosis: scan the last batch alone two ways")
    ap.add_argument("--devices", default="0", help="GPUs of the scans, e.g. 0,1,2,3 (batches round-robin)")
    ap.add_argument("--native", action="store_true", help="the C pinned table (NativePinnedTable, cudasp_pinned_*)")
    a = ap.parse_args()
    import pyarrow as pa
    import torch

    import bench
    from cudasp_amd import NativePinnedTable, PinnedTable, _native, assign_gpu
    lib = _native.load()
    device = 0
    torch.cuda.set_device(device)
    labels = bench.label_keys(a.labels)
    gen = torch.cuda.Stream(device)
    t0 = time.perf_counter()
    batches = bench.rank_batches("rows", a.rows, a.batch_size, 0, 1, assign_gpu)
    tab = bench.Table(lib, device, batches, a.batch_size, 2, labels, dev_stream=gen, kmax=a.outputs_max)
    # host Arrow table in row order
    rows, offs_all, vals = [], [np.zeros(1, dtype=np.int64)], []
    base = 0
    for b in range(tab.nb):
        m = tab.sizes[b]
        x = tab.cols(tab.tx, b).cpu().numpy().view(np.uint32)  # (8, m): packed with stride m
        y = tab.cols(tab.ty, b).cpu().numpy().view(np.uint32)
        rows.append(np.ascontiguousarray(np.concatenate([x.T, y.T], axis=1).astype("<u4")).view(np.uint8))
        ln = tab.lens[b][:m].cpu().numpy().astype(np.int64)
        of = tab.offs[b][:m].cpu().numpy().astype(np.int64)
        outs = tab.outs[b].cpu().numpy()
        first = np.cumsum(ln) - ln  # each row's list, gathered to row order
        vals.append(outs[np.repeat(of - first, ln) + np.arange(int(ln.sum()))])
        offs_all.append(base + np.cumsum(ln))
        base += int(ln.sum())
    g = np.arange(a.rows, dtype=np.uint64)
    txid = np.zeros((a.rows, 32), dtype=np.uint8)
    txid[:, 24:] = g.astype(">u8").view(np.uint8).reshape(-1, 8)
    height = (800000 + g // 4000).astype(np.int32)
    tweak = np.concatenate(rows).reshape(-1)
    offsets = np.concatenate(offs_all).astype(np.int64)
    values = np.concatenate(vals).astype(np.int64)
    expected = tab.expected
    del tab, rows, vals
    torch.cuda.empty_cache()
    table = pa.table({
        "txid": pa.FixedSizeBinaryArray.from_buffers(pa.binary(32), a.rows, [None, pa.py_buffer(txid.reshape(-1))]),
        "height": pa.array(height),
        "tweak_key": pa.FixedSizeBinaryArray.from_buffers(pa.binary(64), a.rows, [None, pa.py_buffer(tweak)]),
        "outputs": pa.LargeListArray.from_arrays(pa.array(offsets), pa.array(values)),
    })
    t_build = time.perf_counter() - t0
    t0 = time.perf_counter()
    devices = [int(x) for x in a.devices.split(",")]
    pt = (NativePinnedTable if a.native else PinnedTable)(table, batch_size=a.batch_size, devices=devices)
    t_pin = time.perf_counter() - t0
    scans = []
    for r in range(a.reps + 1):  # the first scan warms the process (tables, scratch)
        out = pt.scan(bench.SCAN_KEY, bench.SPEND_KEY, labels)
        st = dict(pt.last_stats)
        got = np.sort(np.frombuffer(out.column("txid").combine_chunks().cast(pa.binary(32)).buffers()[1],
                                    dtype=np.uint8).reshape(-1, 32)[:, 24:].copy().view(">u8").reshape(-1).astype(np.int64)) \
            if out.num_rows else np.zeros(0, dtype=np.int64)
        want = np.sort(np.concatenate([np.arange(0, a.rows, 1000)] + ([np.arange(1, a.rows, 1000)] if a.labels else [])))
        st["exact"] = bool(got.size == want.size and (got == want).all())
        if not st["exact"]:
            extra, missing = np.setdiff1d(got, want), np.setdiff1d(want, got)
            st["diff"] = dict(emitted=int(got.size), planted=int(want.size), extra=extra[:8].tolist(),
                              missing=missing[:8].tolist(), n_extra=int(extra.size), n_missing=int(missing.size),
                              duplicates=int(got.size - np.unique(got).size))
        scans.append(st)
    if a.probe:  # diagnosis: the last batch alone, pinned and through the Arrow host path
        from cudasp_amd import cudasp_scan_arrow
        r0 = (a.rows - 1) // a.batch_size * a.batch_size
        sl = table.slice(r0)
        with (NativePinnedTable if a.native else PinnedTable)(sl, batch_size=a.batch_size) as p2:
            n_pinned = p2.scan(bench.SCAN_KEY, bench.SPEND_KEY, labels).num_rows
        n_arrow = cudasp_scan_arrow(sl, bench.SCAN_KEY, bench.SPEND_KEY, labels, batch_size=a.batch_size).num_rows
        print(json.dumps(dict(probe_last_batch_rows=a.rows - r0, pinned=n_pinned, arrow=n_arrow)), flush=True)
    timed = scans[1:]
    med = float(np.median([s["scan_s"] for s in timed]))
    res = dict(what="PinnedTable.scan: pinned host table scanned in place (one streaming kernel, no host copies)",
               rows=a.rows, batch_size=a.batch_size, native=a.native, labels=a.labels, outputs_max=a.outputs_max, devices=devices,
               expected=expected, exact=all(s["exact"] for s in scans), build_s=round(t_build, 2),
               pin_s=round(t_pin, 2), scans=[dict(s=round(s["scan_s"], 4), tx_per_s=round(s["tx_per_s"])) for s in timed],
               tx_per_s=a.rows / med, warmup_s=round(scans[0]["scan_s"], 4),
               diffs=[s["diff"] for s in scans if "diff" in s][:3])
    print(json.dumps(res))
    pt.close()


if __name__ == "__main__":
    main()
