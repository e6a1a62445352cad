"""Repeatability stress of the small-launch value path (the bench's planter).

One reference launch computes t and the compare value of every row of a
synthetic table; then many small launches (gathered rows, like bench.py's
planting) recompute them and every difference is counted, split by stage
(t from stage A, value from stage B) and by the row's position group
j = k // ceil(n / 4) inside the launch (the 4-rows-per-thread slot).

    python tools/stress_values.py [--rows 30000] [--chunk 300] [--iters 300]

Run two copies at once on one GPU to test launches that share the device
with another process.
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "duckdb-cudasp-extension_amd"))
sys.path.insert(0, ROOT)

from cudasp_amd import Scanner, _native  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=30000)
    ap.add_argument("--chunk", type=int, default=300)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--tag", default="")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    lib = _native.load()
    n = args.rows
    tx = torch.empty((8, n), dtype=torch.int32, device=dev)
    ty = torch.empty((8, n), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()
    _native.check(lib.cudasp_synth_tweak_columns(0, bench.synth_s0(), 12345, n, tx.data_ptr(), ty.data_ptr(),
                                                 _native.stream_arg(st)))
    torch.cuda.synchronize()
    big = Scanner(bench.SCAN_KEY, bench.SPEND_KEY, [], max_rows=n, device=0)
    t_ref = torch.empty((8, n), dtype=torch.int32, device=dev)
    v_ref = torch.empty((1, n), dtype=torch.int64, device=dev)
    big.row_values_device(tx, ty, t_ref, v_ref)
    big.sync()
    small = Scanner(bench.SCAN_KEY, bench.SPEND_KEY, [], max_rows=2 * args.chunk + 2, device=0)
    g = torch.Generator().manual_seed(args.seed)
    m = args.chunk
    G = (m + 3) // 4
    bad_t = [0, 0, 0, 0]
    bad_v = [0, 0, 0, 0]
    bad_launches = 0
    for it in range(args.iters):
        idx = torch.randperm(n, generator=g)[:m].to(dev)
        gx = tx.index_select(1, idx).contiguous()
        gy = ty.index_select(1, idx).contiguous()
        t = torch.empty((8, m), dtype=torch.int32, device=dev)
        v = torch.empty((1, m), dtype=torch.int64, device=dev)
        small.row_values_device(gx, gy, t, v)
        small.sync()
        dt = (t != t_ref.index_select(1, idx)).any(0).cpu()
        dv = (v != v_ref.index_select(1, idx)).any(0).cpu()
        if dt.any() or dv.any():
            bad_launches += 1
            for k in range(m):
                if dt[k]:
                    bad_t[k // G] += 1
                if dv[k]:
                    bad_v[k // G] += 1
        if (it + 1) % 100 == 0:
            print(json.dumps(dict(tag=args.tag, iters=it + 1, bad_launches=bad_launches, bad_t_by_j=bad_t,
                                  bad_v_by_j=bad_v)), flush=True)
    small.close()
    big.close()


if __name__ == "__main__":
    main()
