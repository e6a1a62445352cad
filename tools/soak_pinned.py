"""Randomized soak of cudasp_amd.PinnedTable and NativePinnedTable (the C
cudasp_pinned_* ABI, appended in random run sizes) on the GPU box (robustness only):
seeded random tables built from the golden random rows (planted base and label
matches; tests/golden/random_rows.json) -- replicated, shuffled, sliced, with
NULL txids / heights / tweaks / lists / list elements injected, binary or
fixed_size_binary tweaks, list or large_list outputs -- pinned with a random
batch_size over 1..3 logical GPUs and scanned several times with random key
sets (0..all labels, variants); every scan must equal cudasp_scan_arrow's rows
(the table-function host path, itself pinned to the oracle by the test suite).

  python tools/soak_pinned.py --minutes 10 --seed 1
"""
import argparse
import json
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "duckdb-cudasp-extension_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=10.0)
    ap.add_argument("--seed", type=int, default=1)
    a = ap.parse_args()
    import pyarrow as pa

    import golden_io
    from cudasp_amd import NativePinnedTable, PinnedTable, cudasp_scan_arrow
    rr = golden_io.load("random_rows.json")
    base = [(bytes.fromhex(x["tweak"]), x["outputs"]) for x in rr["rows"]]
    scan, spend = bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"])
    labels = [bytes.fromhex(l) for l in rr["label_keys"]]
    rng = random.Random(a.seed)
    t_end = time.time() + 60 * a.minutes
    runs = scans = rows_total = 0
    while time.time() < t_end:
        n = rng.choice([1, 50, 700, 3000, 9000])
        rows = []
        for i in range(n):
            tw, outs = base[rng.randrange(len(base))]
            outs = list(outs) if outs is not None else None
            if outs:
                rng.shuffle(outs)
            r = [i.to_bytes(32, "big"), 1000 + i, tw, outs]
            u = rng.random()
            if u < 0.02:
                r[rng.randrange(3)] = None
            elif u < 0.04:
                r[3] = None
            elif u < 0.06 and outs is not None:
                r[3] = outs + [None]
            rows.append(tuple(r))
        large = rng.random() < 0.3
        fixed = not large and rng.random() < 0.5
        tbl = pa.table({
            "txid": pa.array([r[0] for r in rows], pa.large_binary() if large else pa.binary()),
            "height": pa.array([r[1] for r in rows], pa.int32()),
            "tweak_key": pa.array([r[2] for r in rows], pa.binary(64) if fixed else
                                  (pa.large_binary() if large else pa.binary())),
            "outputs": pa.array([r[3] for r in rows], pa.large_list(pa.int64()) if large else pa.list_(pa.int64())),
        })
        if n > 10 and rng.random() < 0.3:
            s0 = rng.randrange(n // 2)
            tbl = tbl.slice(s0, rng.randrange(1, n - s0))
        bs = rng.choice([1, 7, 64, 500, 2048, 300000])
        devices = [0] * rng.choice([1, 1, 2, 3])
        native = rng.random() < 0.5
        kw = dict(piece_rows=rng.choice([1, 97, 65536]), placement=rng.choice(["pinned", "hbm"])) if native else {}
        with (NativePinnedTable if native else PinnedTable)(tbl, batch_size=bs, devices=devices, **kw) as pt:
            for _ in range(rng.choice([1, 2, 3])):
                L = labels[:rng.randrange(len(labels) + 1)]
                oc = rng.choice([None, None, 2, 7])
                neg = rng.choice([None, None, True])
                got = sorted(zip(*[c.to_pylist() for c in pt.scan(scan, spend, L, output_count=oc,
                                                                   label_negation=neg).columns]))
                want = sorted(zip(*[c.to_pylist() for c in cudasp_scan_arrow(tbl, scan, spend, L, batch_size=bs,
                                                                             output_count=oc,
                                                                             label_negation=neg).columns]))
                scans += 1
                if got != want:
                    print(json.dumps(dict(failed=True, run=runs, native=native, kw=str(kw), rows=tbl.num_rows,
                                          batch_size=bs,
                                          devices=devices,
                                          labels=len(L), output_count=oc, label_negation=neg, got=len(got),
                                          want=len(want))), flush=True)
                    sys.exit(1)
        runs += 1
        rows_total += tbl.num_rows
        if runs % 20 == 0:
            print(json.dumps(dict(runs=runs, scans=scans)), flush=True)
    print(json.dumps(dict(soak="ok", seed=a.seed, minutes=a.minutes, runs=runs, scans=scans, rows=rows_total)),
          flush=True)


if __name__ == "__main__":
    main()
