"""Per-wave timeline of one k_scan_multi launch (measurement build only).

Build the library with -DCUDASP_MULTI_TRACE=1 (e.g. into
build_variants/trace/), then on the GPU box:

  CUDASP_LIB=build_variants/trace/libcudasp_amd.so python tools/multi_trace.py --rows 4200000

It scans a bench table of that many rows (round-robin share of rank 0 at
N = 1: --rows alone sets the table) once to warm up and once traced, and
prints, from every wave's start / end time and work: the launch span, how the
waves' start and end times spread, the wave-slot time left idle at the start
and in the drain (as a fraction of slots x span), pieces and wave-rows per
wave, and the mean end time per XCD (block i runs on XCD i mod 8).  From each
wave's placement (HW_ID, XCC_ID): the SIMDs' finish times and their idle
fraction in the drain, the waves per SIMD still busy when the counter ran
out, each SIMD's work by wave rank, and the shader clock (s_memtime ticks over
s_memrealtime).
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "duckdb-cudasp-extension_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4_200_000)
    ap.add_argument("--labels", type=int, default=0)
    ap.add_argument("--batch-size", type=int, default=300_000)
    ap.add_argument("--out", default="")
    ap.add_argument("--gap-ms", type=float, default=0.0,
                    help="host gap before the traced launch: -1 = queued right behind the previous launch "
                         "(no synchronize), 0 = synchronize only, > 0 = synchronize and sleep this long")
    ap.add_argument("--prior", type=int, default=1, help="launches before the traced one")
    a = ap.parse_args()
    os.environ.setdefault("CUDASP_FB_BITS", "26")
    import torch
    import bench
    from cudasp_amd import Scanner, _native, assign_gpu
    lib = _native.load()
    if not hasattr(lib, "cudasp_debug_multi_trace"):
        sys.exit("library built without CUDASP_MULTI_TRACE (set CUDASP_LIB to a trace build)")
    fn = lib.cudasp_debug_multi_trace
    fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int)]
    fn.restype = ctypes.c_int
    device = 0
    torch.cuda.set_device(device)
    labels = bench.label_keys(a.labels)
    gen = torch.cuda.Stream(device)
    batches = bench.rank_batches("roundrobin", a.rows, a.batch_size, 0, 1, assign_gpu)
    tab = bench.Table(lib, device, batches, a.batch_size, 2, labels, dev_stream=gen)
    scanner = Scanner(bench.SCAN_KEY, bench.SPEND_KEY, labels, max_rows=a.batch_size, device=device)
    scanner.set_fixed_base_bits(26)
    stream = torch.cuda.Stream(device)
    descs = bench.multi_descs(tab)
    bench.run_step_multi(tab, scanner, stream, descs)  # warm-up (builds the tables)
    torch.cuda.synchronize(device)
    for i in range(a.prior + 1):  # the prior launches, then the traced one
        if i == a.prior and a.gap_ms >= 0:
            torch.cuda.synchronize(device)
            if a.gap_ms > 0:
                import time
                time.sleep(a.gap_ms / 1e3)
        bench.run_step_multi(tab, scanner, stream, descs)
    torch.cuda.synchronize(device)
    found = int(tab.match_count.sum().item())
    W = 8
    buf = np.zeros(8192 * W, dtype=np.uint64)
    hz = ctypes.c_int(0)
    n = fn(buf.ctypes.data, 8192, ctypes.byref(hz))
    allrec = buf[: W * n].reshape(n, W)
    idx = np.nonzero(allrec[:, 1] > 0)[0]  # waves of the launch (the grid may be smaller than the buffer)
    rec = allrec[idx]
    waves = len(rec)
    t0 = rec[:, 0].min()
    ms = 1e3 / hz.value
    start = (rec[:, 0] - t0) * ms
    end = (rec[:, 1] - t0) * ms
    span = end.max()
    idle_start = start.sum() / (waves * span)
    idle_drain = (span - end).sum() / (waves * span)
    xcd = (idx // 4) % 8  # 4 waves per 256-thread block; block i on XCD i mod 8
    res = dict(rows=a.rows, labels=a.labels, gap_ms=a.gap_ms, prior=a.prior, batches=tab.nb, found=found, expected=tab.expected, waves=waves,
               clock_hz=hz.value, span_ms=round(float(span), 3),
               start_ms_p50_p99_max=[round(float(np.percentile(start, q)), 3) for q in (50, 99, 100)],
               end_ms_min_p1_p50_p99=[round(float(np.percentile(end, q)), 3) for q in (0, 1, 50, 99)],
               drain_ms_first_exit_to_last=round(float(span - end.min()), 3),
               idle_fraction_start=round(float(idle_start), 4), idle_fraction_drain=round(float(idle_drain), 4),
               pieces_per_wave_min_mean_max=[int(rec[:, 2].min()), round(float(rec[:, 2].mean()), 2), int(rec[:, 2].max())],
               wave_rows_per_wave_min_mean_max=[int(rec[:, 3].min()), round(float(rec[:, 3].mean()), 2),
                                                int(rec[:, 3].max())],
               mean_end_ms_per_xcd=[round(float(end[xcd == x].mean()), 3) for x in range(8)])
    # placement: HW_ID bits 4-5 SIMD, 8-11 CU, 12 SH, 13-15 SE; XCC_ID in the high word
    hw = rec[:, 4] & 0xFFFFFFFF
    xcc_hw = (rec[:, 4] >> 32) & 0xF
    simd_key = (xcc_hw << 16) | (((hw >> 8) & 0xFF) << 2) | ((hw >> 4) & 3)
    keys, inv = np.unique(simd_key, return_inverse=True)
    simd_end = np.zeros(len(keys))
    np.maximum.at(simd_end, inv, end)
    texh = (rec[:, 5].astype(np.int64) - int(t0)) * ms
    t_x = float(texh[rec[:, 5] > 0].min())  # the counter ran out
    busy_at_x = np.bincount(inv, weights=(end > t_x).astype(float), minlength=len(keys))
    ticks = rec[:, 6].astype(float)
    ta = (rec[:, 7].astype(np.int64) - int(t0)) * ms  # the wave's last stage-A row ended
    life_s = (end - start) / 1e3
    clock_mhz = ticks / life_s / 1e6
    # wave rank inside its SIMD by rows done (0 = the most)
    order = np.lexsort((-rec[:, 3].astype(np.int64), inv))
    rank = np.zeros(waves, dtype=int)
    first = np.r_[0, np.nonzero(np.diff(inv[order]))[0] + 1]
    for lo, hi in zip(first, np.r_[first[1:], waves]):
        rank[order[lo:hi]] = np.arange(hi - lo)
    res.update(simds=int(len(keys)), waves_per_simd=np.bincount(np.bincount(inv)).tolist(),
               simd_end_ms_min_p1_p50_p99=[round(float(np.percentile(simd_end, q)), 3) for q in (0, 1, 50, 99)],
               simd_idle_fraction_drain=round(float((span - simd_end).mean() / span), 4),
               counter_out_ms=round(t_x, 3),
               simds_by_busy_waves_at_counter_out=np.bincount(busy_at_x.astype(int), minlength=4).tolist(),
               rows_share_by_rank=[round(float(rec[rank == r, 3].sum() / rec[:, 3].sum()), 4) for r in range(int(rank.max()) + 1)],
               end_ms_mean_by_rank=[round(float(end[rank == r].mean()), 3) for r in range(int(rank.max()) + 1)],
               shader_clock_mhz_p1_p50_p99=[round(float(np.percentile(clock_mhz, q)), 1) for q in (1, 50, 99)],
               stage_a_end_ms_mean_by_rank=[round(float(ta[rank == r].mean()), 3) for r in range(int(rank.max()) + 1)])
    print(json.dumps(res))
    if a.out:
        np.savez(a.out, start=start, end=end, pieces=rec[:, 2], rows=rec[:, 3], xcd=xcd, simd=inv, rank=rank,
                 exhausted=texh, clock_mhz=clock_mhz, stage_a_end=ta)
    scanner.close()


if __name__ == "__main__":
    main()
