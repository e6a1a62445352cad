"""Streaming-scan probe (measurement only): the same synthetic table scanned
(a) device-resident by cudasp_scan_device_batches (one k_scan_multi launch)
and (b) by the streaming scan from pinned host memory (cudasp_stream_*: one
persistent k_scan_stream), all batches published at once and, in the paced
form, with at most `--in-flight` batches out as the table-function host's
slot ring allows.  Flags of both must be identical.  One JSON line.

  python tools/stream_probe.py --rows 9400000 --labels 1
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "duckdb-cudasp-extension_amd"), os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=3_000_000)
    ap.add_argument("--batch", type=int, default=300_000)
    ap.add_argument("--labels", type=int, default=0)
    ap.add_argument("--kmax", type=int, default=0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--in-flight", type=int, default=8)
    ap.add_argument("--modes", default="all,paced")
    ap.add_argument("--device-inputs", action="store_true",
                    help="publish device copies of rows / offsets / lengths / outputs (a library built with "
                         "-DCUDASP_AB_STREAM_ANY_MEMORY): prices the zero-copy PCIe reads")
    ap.add_argument("--device-results", action="store_true",
                    help="match rows into device memory too (same build)")
    ap.add_argument("--gap-ms", type=float, default=0.0,
                    help="sleep this long (GPU idle) before every timed run of either kernel")
    ap.add_argument("--prewarm", action="store_true",
                    help="run k_scan_multi (untimed) right before every timed streaming run")
    ap.add_argument("--flags", action="store_true", help="also write per-row flags (the host path writes matches only)")
    a = ap.parse_args()
    import torch

    import bench
    import test_multi_batch_gpu as tm
    from cudasp_amd import Scanner, ScanStream, StreamBatch

    labels = bench.label_keys(a.labels) if a.labels else []
    sizes = [a.batch] * (a.rows // a.batch) + ([a.rows % a.batch] if a.rows % a.batch else [])
    t0 = time.time()
    batches = [tm.make_batch(torch, i * a.batch, n, kmax=a.kmax) for i, n in enumerate(sizes)]
    tm.plant(torch, batches, labels, every=1000)
    stage = []
    for b in batches:
        n = b["n"]
        xs = b["tweak_x"].cpu().numpy().view(np.uint32)
        ys = b["tweak_y"].cpu().numpy().view(np.uint32)
        rows = np.ascontiguousarray(np.concatenate([xs.T, ys.T], axis=1)).view(np.uint8).reshape(n, 64)
        stage.append(StreamBatch(rows, b["outputs"].cpu().numpy(), b["offsets"][:n].cpu().numpy().view(np.uint32),
                                 b["lengths"][:n].cpu().numpy().view(np.uint32), label_count=len(labels),
                                 want_flags=a.flags))
    setup_s = time.time() - t0
    out = dict(rows=a.rows, batch=a.batch, labels=a.labels, kmax=a.kmax, batches=len(sizes), setup_s=round(setup_s, 1))
    with Scanner(tm.SCAN, tm.SPEND, labels, max_rows=a.batch) as s:
        flags = [torch.zeros(max(b["n"], 1), dtype=torch.uint8, device="cuda") for b in batches]
        descs = [dict(tweak_x=b["tweak_x"], tweak_y=b["tweak_y"], outputs=b["outputs"], offsets=b["offsets"],
                      lengths=b["lengths"], flags=f[:b["n"]]) for b, f in zip(batches, flags)]
        s.scan_device_batches(descs)
        s.sync()
        times = []
        for _ in range(a.reps):
            torch.cuda.synchronize()
            if a.gap_ms:
                time.sleep(a.gap_ms / 1e3)
            t = time.perf_counter()
            s.scan_device_batches(descs)
            s.sync()
            times.append(time.perf_counter() - t)
        out["multi_ms"] = round(1e3 * min(times), 2)
        out["multi_tx_s"] = a.rows / min(times)
        want = [f[:b["n"]].cpu().numpy() for f, b in zip(flags, batches)]
        dev = []
        for b, sb in zip(batches, stage):
            d = {}
            if a.device_inputs:
                d["rows"] = torch.from_numpy(sb.rows.array.copy()).cuda()
                d["outputs"] = b["outputs"]
                d["offs"] = b["offsets"]
                d["lens"] = b["lengths"]
            if a.device_results:
                d["matches"] = torch.zeros(max(1, b["n"]), dtype=torch.int32, device="cuda")
            dev.append(d)
        torch.cuda.synchronize()
        with ScanStream(s) as st:
            for mode in a.modes.split(","):
                times = []
                for _ in range(a.reps + 1):
                    for sb in stage:
                        sb.reset()
                    if a.gap_ms:
                        time.sleep(a.gap_ms / 1e3)
                    if a.prewarm:
                        s.scan_device_batches(descs)
                        s.sync()
                    t = time.perf_counter()
                    seqs = []
                    for sb, d in zip(stage, dev):
                        if mode == "paced" and len(seqs) >= a.in_flight:
                            st.wait(seqs[-a.in_flight])
                        if a.device_inputs or a.device_results:
                            mr = d["matches"].data_ptr() if a.device_results else sb.match_rows
                            src = d if a.device_inputs else None
                            seqs.append(st.publish(src["rows"].data_ptr() if src else sb.rows,
                                                   src["outputs"].data_ptr() if src else sb.outputs,
                                                   src["offs"].data_ptr() if src else sb.offsets,
                                                   src["lens"].data_ptr() if src else sb.lengths,
                                                   sb.n, None, src["outputs"] if src else sb.mirror, mr))
                            sb.seq = seqs[-1]
                        else:
                            seqs.append(sb.publish(st))
                    st.close_input()
                    st.wait(seqs[-1])
                    for q in seqs:
                        st.wait(q)
                    times.append(time.perf_counter() - t)
                    for i, (sb, w) in enumerate(zip(stage, want)):
                        ok = True
                        if a.flags:
                            ok = (sb.result() == w).all()
                        else:  # match counts readable until finish
                            if a.device_results:
                                c = st.matches(sb.seq)
                                m = np.sort(dev[i]["matches"][:c].cpu().numpy().view(np.uint32))
                            else:
                                m = sb.matches(st)
                            ok = len(m) == int(w.sum()) and (m == np.nonzero(w)[0]).all()
                        if not ok:
                            out["mismatch"] = "%s batch %d" % (mode, i)
                    st.finish()
                    out["counters_%s" % mode] = st.counters()
                best = min(times[1:])
                out["stream_%s_ms" % mode] = round(1e3 * best, 2)
                out["stream_%s_tx_s" % mode] = a.rows / best
            out["stream_stats"] = st.stats()
        out["flags_equal"] = "mismatch" not in out
        out["found"] = int(sum(int(w.sum()) for w in want))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
