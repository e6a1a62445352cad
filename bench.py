#!/usr/bin/env python3
"""bench.py -- tx/s through cudasp_scan on a 32.7M-row synthetic tweak table.

Contract (see DESIGN.md "Measurement"):
  python bench.py [--gpus N] [--steps K] [--warmup W]
  N > 1 is launched by the driver as one process per GPU via
  torch.distributed.run; ranks read RANK / LOCAL_RANK / WORLD_SIZE.

Workload (BASELINE.json metric "tx/sec through cudasp_scan on 32M-row tweak
table at 1/2/4/8 MI355X", configs[3]): ONE 32.7M-row synthetic table and the
reference's default batch_size 300000 at every N (BASELINE.md section 3 row
4).  Every GPU scans its contiguous 1/N share of the rows, batched at
batch_size with one partial last batch (`--shard rows`): that is how batches
form per GPU in the reference (each executor thread batches the rows it is
handed, src/cudasp_extension.cu:416-418, and threads round-robin over the
GPUs, :523-529) and in the product's host (one device feed per GPU), so the
total work is fixed as N grows.  At N > 1 a secondary line cuts the same table
into global 300000-row batches dealt round-robin (batch b on rank b mod N,
cudasp_assign_gpu) and reports it as `value_roundrobin`, never as the
headline (`--shard roundrobin` makes it the headline; `--shard weak` gives
every rank its own table).  Each rank's batches are resident in HBM, tweak limbs
column-major per batch.  A step is one pass of the hot path over the rank's
batches: by default (`--launch multi`) one cudasp_scan_device_batches call
over all of them -- one persistent kernel (k_scan_multi) runs both stages
(stage A: d*T + tagged hash; stage B: t*G + B, labels, compare, flag + ballot
compaction) for every row, with per-batch flags and match lists; with
`--launch batches` every batch goes through cudasp_scan_device, round-robin
over `--streams` HIP streams (the reference's per-thread streams,
src/cudasp_gpu.cu:505).  No collective in the data path: torch.distributed
carries the bracketing barrier and the max of the elapsed time.  After the
timed steps, rank 0 also reports the PCIe-inclusive end-to-end rate of the
table-function host over all N GPUs (`e2e`: tools/host_e2e as a child
process, the same table shape in host memory, fed by executor threads through
the calls DuckDB makes; at N > 1 the other ranks wait at a CPU barrier) --
never the `value`.  `e2e` runs the host's default streaming feeds (one
persistent kernel per GPU reading the batch slots in place from pinned host
memory); `e2e_launch` the same child with per-slot
copies and launches (CUDASP_TF_MODE=launch).

Synthetic data: T_i = (s0 + g) G with s0 = SHA256("cudasp-synth-v1")
mod n and g the global row index; 2 splitmix64 outputs per row (seed
0xC0DA5EED); every 1000th row gets its true compare value planted, and with
L labels the next row gets label j's value, j cycling over all L labels, so the
expected match count is known exactly and checked after the run.

Only the CPU legs touch oracle/ (the C restatement: timed on a bounded sample
on this box's host cores as `cpu_baseline_port` and checked against the GPU
flags; it also recomputes the planted values of 256 planted rows spread over
the whole rank table, `planted_oracle_check`, and of a 256-row sample of the
end-to-end leg's planted and unplanted rows, `e2e.planted_oracle_check`).
With --pinned, the `pinned` leg scans the same table pinned once in host
memory, in place (the C pinned table cudasp_pinned_* driven by tools/host_e2e
--pinned, over all N GPUs, no host copy per query) and
the `resident` leg the same table kept in HBM by the same ABI
(CUDASP_TABLE_HBM); both are off by default (an API the reference's SQL
interface does not reach).
`cpu_baseline` itself is the strongest CPU stand-in the image allows:
`port-optimized` (tools/cpu_port, the product's row pipeline compiled for the
host) where it covers the options, else the oracle port.
"""
import argparse
import ctypes
import glob
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "duckdb-cudasp-extension_amd"))

sys.path.insert(0, os.path.join(ROOT, "tools"))

import codeobj  # noqa: E402
from cudasp_amd import Scanner, _native  # noqa: E402

METRIC = "tx/sec through cudasp_scan on 32M-row tweak table at 1/2/4/8 MI355X"
# Keys of the BIP-352 test vector as the reference's SQL test passes them
# (test/sql/cudasp.test:54): scan key LE, spend key LE x || y.
SCAN_KEY = bytes.fromhex("2c1f0cb94db3946522cc1487256535dd33a1f911946baff817a72880064e690f")
SPEND_KEY = bytes.fromhex(
    "36cf8fcd4d4890ab6c1083aeb5b50c260c20acda7839120e3575836f6d85c95c"
    "e0d705e31ff9fdcce67a8f3598871c6dfbe6bcde8a51cb7b48b0f95be0ea94de")
# Label key of test/sql/cudasp.test:104.
TEST_LABEL = bytes.fromhex(
    "cd63f9212a2deebde8a71e9ea23f6f958c47c41d2ed74b9617fe6fb554d1524e"
    "292fabddbdcbb643eafc328875c46d75a1d697b2b31c42d38aa93f85eab34bc1")
N_ORDER = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
P_FIELD = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
OUTPUT_SEED = 0xC0DA5EED
PLANT_EVERY = 1000
# Algorithmic HBM bytes per row: 64 tweak + 8 offset/length
# + 8 per output + 1 flag.
def bytes_per_row(k):
    return 73 + 8 * k


HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md, spec
# VALU issue peaks (wave-instructions/s per GPU):
#   nominal: 4 SIMD32 per CU, a wave64 VALU op every 2 cycles -> 2 per CU-cycle,
#            x 256 CUs x 2.4 GHz;
#   measured for VOP3 ops (v_mad_u64_u32, v_add3, v_lshl_add_u64: 37.1e12
#            lane-ops/s, profiles/r01_microbench_int.txt) -- half the nominal
#            rate; the scan kernels are ~80% VOP3.
VALU_WAVE_INSTR_PEAK = 2 * 256 * 2.4e9
VOP3_WAVE_INSTR_MEASURED = 37.1e12 / 64


def _ec_add(p, q):
    if p is None:
        return q
    if q is None:
        return p
    if p[0] == q[0]:
        if (p[1] + q[1]) % P_FIELD == 0:
            return None
        lam = 3 * p[0] * p[0] * pow(2 * p[1], -1, P_FIELD) % P_FIELD
    else:
        lam = (q[1] - p[1]) * pow(q[0] - p[0], -1, P_FIELD) % P_FIELD
    x = (lam * lam - p[0] - q[0]) % P_FIELD
    return (x, (lam * (p[0] - x) - p[1]) % P_FIELD)


def _ec_mul(k, p):
    r = None
    while k:
        if k & 1:
            r = _ec_add(r, p)
        p = _ec_add(p, p)
        k >>= 1
    return r


def label_keys(count):
    """Label keys: the SQL test's label, then L_j = (j+1) c G."""
    out = []
    if count >= 1:
        out.append(TEST_LABEL)
    c = int.from_bytes(hashlib.sha256(b"cudasp-label-v1").digest(), "big") % N_ORDER
    j = 1
    while len(out) < count:
        pt = _ec_mul((j + 1) * c % N_ORDER, (GX, GY))
        out.append(pt[0].to_bytes(32, "little") + pt[1].to_bytes(32, "little"))
        j += 1
    return out


def synth_s0():
    s0 = int.from_bytes(hashlib.sha256(b"cudasp-synth-v1").digest(), "big") % N_ORDER
    return s0.to_bytes(32, "little")


class Table:
    """One rank's resident share of the synthetic table, batch-major.

    batches: [(first global row, rows)] of the rank's batches (whole
    batch_size-row batches of the global table, the last one possibly short)."""

    def __init__(self, lib, device, batches, batch, k, labels, dev_stream, kmax=0):
        """k: fixed outputs per row; kmax > 0: variable lengths uniform in [1, kmax]."""
        self.batch, self.k, self.kmax = batch, k, kmax
        cap = kmax if kmax else k
        self.first = [g0 for g0, _ in batches]
        self.sizes = [m for _, m in batches]
        self.nb = len(batches)
        self.rows = sum(self.sizes)
        dev = torch.device("cuda", device)
        nb = max(1, self.nb)
        self.tx = torch.empty((nb, 8, batch), dtype=torch.int32, device=dev)
        self.ty = torch.empty((nb, 8, batch), dtype=torch.int32, device=dev)
        self.outs = torch.empty((nb, batch * cap), dtype=torch.int64, device=dev)
        self.offs = torch.empty((nb, batch), dtype=torch.int32, device=dev)
        self.lens = torch.empty((nb, batch), dtype=torch.int32, device=dev)
        self.flags = torch.zeros((nb, batch), dtype=torch.uint8, device=dev)
        self.match_rows = torch.zeros((nb, batch), dtype=torch.int32, device=dev)
        self.match_count = torch.zeros((nb,), dtype=torch.int32, device=dev)
        s0 = synth_s0()
        st = _native.stream_arg(dev_stream)
        for b in range(self.nb):
            m, g0 = self.sizes[b], self.first[b]
            _native.check(lib.cudasp_synth_tweak_columns(device, s0, g0, m, self.tx[b].data_ptr(),
                                                         self.ty[b].data_ptr(), st))
            if kmax:
                _native.check(lib.cudasp_synth_output_lengths(OUTPUT_SEED, g0, m, kmax, self.lens[b].data_ptr(), st))
                with torch.cuda.stream(dev_stream):
                    ln = self.lens[b][:m].to(torch.int64)
                    self.offs[b][:m] = (torch.cumsum(ln, 0) - ln).to(torch.int32)
                _native.check(lib.cudasp_synth_output_values(OUTPUT_SEED, g0, m, self.offs[b].data_ptr(),
                                                             self.lens[b].data_ptr(), self.outs[b].data_ptr(), st))
            else:
                _native.check(lib.cudasp_synth_outputs(OUTPUT_SEED, g0, m, k, self.outs[b].data_ptr(),
                                                       self.offs[b].data_ptr(), self.lens[b].data_ptr(), st))
        torch.cuda.synchronize(dev)
        # Plant true values (computed by the product's own stage outputs; the
        # test suite checks those against the oracle): the base value on every
        # global row g = 0 mod 1000 and, with L labels, label j's value on row
        # g = 1 mod 1000 with j = (g // 1000) mod L, so every label index of
        # the label loop (src/cudasp_gpu.cu:153-172) is planted and must be found.
        self.total_outputs = sum(int(self.lens[b][:self.sizes[b]].to(torch.int64).sum().item())
                                 for b in range(self.nb)) if kmax else self.rows * k
        self.expected = 0
        self.expected_per_batch = [0] * self.nb
        self.planted_labels = set()
        self.plant_log = []  # (batch, row in batch, values column: 0 = base, 1 + j = label j)
        L = len(labels)
        per_batch = 2 * ((batch + PLANT_EVERY - 1) // PLANT_EVERY) + 2
        planter = Scanner(SCAN_KEY, SPEND_KEY, labels, max_rows=per_batch, device=device)
        for b in range(self.nb):
            m, g0 = self.sizes[b], self.first[b]
            base_idx = [i for i in range((-g0) % PLANT_EVERY, m, PLANT_EVERY)]
            lab_idx = [i for i in range((1 - g0) % PLANT_EVERY, m, PLANT_EVERY)] if L else []
            idx = base_idx + lab_idx
            if not idx:
                continue
            it = torch.tensor(idx, dtype=torch.int64, device=dev)
            gx = self.cols(self.tx, b).index_select(1, it).contiguous()
            gy = self.cols(self.ty, b).index_select(1, it).contiguous()
            t = torch.empty((8, len(idx)), dtype=torch.int32, device=dev)
            vals = torch.empty((1 + L, len(idx)), dtype=torch.int64, device=dev)
            planter.row_values_device(gx, gy, t, vals)
            planter.sync()
            nbase = len(base_idx)
            pos = self.offs[b][:m].index_select(0, it).to(torch.int64)  # slot 0 of each planted list
            self.outs[b].index_copy_(0, pos[:nbase], vals[0, :nbase])
            if lab_idx:
                js = [((g0 + i) // PLANT_EVERY) % L for i in lab_idx]
                self.planted_labels.update(js)
                jt = torch.tensor(js, dtype=torch.int64, device=dev)
                cols = torch.arange(nbase, len(idx), dtype=torch.int64, device=dev)
                self.outs[b].index_copy_(0, pos[nbase:], vals[1 + jt, cols])
            self.expected += len(idx)
            self.expected_per_batch[b] = len(idx)
            self.plant_log += [(b, i, 0) for i in base_idx]
            if lab_idx:
                self.plant_log += [(b, i, 1 + j) for i, j in zip(lab_idx, js)]
        planter.close()
        torch.cuda.synchronize(dev)


def _cols(self, arr, b):
    """Batch b of a column array as its (8, m) column-major view (limb j of row
    i at j*m + i, the layout the kernels read)."""
    m = self.sizes[b]
    return arr[b].view(-1)[: 8 * m].view(8, m)


Table.cols = _cols


def aggregate(world, backend, total_s, found, flagged, expected):
    """Cross-rank reduction of one run: the job time is the MAX over ranks,
    match counts are summed.  Control plane only (no data-path collective)."""
    if world <= 1:
        return total_s, found, flagged, expected
    dev_t = "cuda" if backend == "nccl" else "cpu"
    tt = torch.tensor([total_s], dtype=torch.float64, device=dev_t)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    cnt = torch.tensor([found, flagged, expected], dtype=torch.int64, device=dev_t)
    dist.all_reduce(cnt, op=dist.ReduceOp.SUM)
    f, fl, e = (int(x) for x in cnt.tolist())
    return float(tt.item()), f, fl, e


def shard_first_row(rank, rows_per_rank):
    """Global index of a rank's first row (weak scaling: rank r owns rows
    [r * rows_per_rank, (r + 1) * rows_per_rank) of one conceptual table)."""
    return rank * rows_per_rank


def balanced_batch_size(rows, world, cap=300_000):
    """`--batch-size 0` (not the default): the largest
    size <= cap (the reference's default batch_size) whose batch count is a
    multiple of `world`, so that round-robin gives every rank the same number
    of batches.  At N = 1 this is cap itself (109 batches of 300000 rows);
    at N = 8 it is 112 batches of 291965 rows (14 per rank) instead of
    300000-row batches 14/13 per rank, whose largest share sets the job time.
    batch_size is the SQL function's own parameter (`batch_size := INTEGER`,
    src/cudasp_extension.cu:626-635); BASELINE configs[3] does not fix it."""
    if rows <= 0 or world <= 1:
        return cap  # N = 1: the reference's batches as configs[1]/[2] state them
    nb = -(-rows // cap)
    nb = -(-nb // world) * world
    return -(-rows // nb)


SHARD_DESC = dict(
    rows="every GPU scans its contiguous 1/N share of the rows in batch_size-row batches (BASELINE.json "
         "configs[3]; per-GPU batching as in the reference and the product host)",
    roundrobin="global batch_size-row batches dealt round-robin over the ranks (batch b on rank b mod N)",
    weak="every rank scans its own table (weak)")


def rank_rows(rows, rank, world):
    """A rank's contiguous share [first, last) of the table's rows (shares
    differ by at most one row)."""
    return rank * rows // world, (rank + 1) * rows // world


def rank_batches(shard, rows, batch, rank, world, assign):
    """The (first global row, rows) batches a rank scans.

    rows (config 4, the default): ONE table of `rows` rows; every GPU scans
    its contiguous 1/N share, batched at batch_size rows with one partial
    last batch.  That is how batches form per GPU both in the reference (each
    executor thread batches the rows it was handed, `>= batch_size` at
    src/cudasp_extension.cu:416-418, its remainder in the final call; threads
    round-robin over the GPUs, :523-529, and DuckDB deals the table's row
    groups over the threads) and in the product's host (one device feed per
    GPU; the threads' chunks round-robin over the GPUs), and it is SURVEY.md
    §8(e)'s "contiguous ranges".
    roundrobin: the same table cut into global batch_size-row batches; batch b
    goes to rank assign(b, world) (cudasp_assign_gpu: b mod N) -- whole
    batches, so the largest share (14 of 109 at N = 8) sets the job time.
    weak: every rank scans its own `rows`-row table (global rows
    [rank * rows, (rank + 1) * rows))."""
    if shard == "rows":
        first, last = rank_rows(rows, rank, world)
        return [(b, min(batch, last - b)) for b in range(first, last, batch)]
    if shard == "roundrobin":
        nb = (rows + batch - 1) // batch
        return [(b * batch, min(batch, rows - b * batch)) for b in range(nb) if assign(b, world) == rank]
    first = shard_first_row(rank, rows)
    return [(first + b * batch, min(batch, rows - b * batch)) for b in range((rows + batch - 1) // batch)]


def run_step(tab, scanners, streams, events=None, tail_rows=(0, 0)):
    """One pass over the rank's table.  Each batch is the two kernels of
    cudasp_scan_device (stage A then stage B on the batch's stream); when
    `events` is a list, HIP events bracket each launch on its stream (with
    several streams a launch's span includes the time it shares the GPU with
    the other streams' kernels)."""
    tab.match_count.zero_()
    cur = torch.cuda.current_stream()
    for st in streams:
        st.wait_stream(cur)  # the counters are zeroed before any batch counts into them
    tail_from = tab.nb - len(streams) if any(tail_rows) else tab.nb
    for b in range(tab.nb):
        s = b % len(scanners)
        st = streams[s]
        m = tab.sizes[b]
        if b >= tail_from:
            scanners[s].set_rows_per_thread(*tail_rows)  # the last round of launches: shorter drain
        with torch.cuda.stream(st):
            if events is not None:
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record(st)
            scanners[s].stage_shared_secret(tab.tx[b], tab.ty[b], m, st)
            if events is not None:
                e1.record(st)
            scanners[s].stage_match(tab.outs[b], tab.offs[b], tab.lens[b], m, tab.flags[b],
                                    tab.match_rows[b], tab.match_count[b:b + 1], st)
            if events is not None:
                e2.record(st)
                events.append((e0, e1, e2))
    if any(tail_rows):
        for sc in scanners:
            sc.set_rows_per_thread(0, 0)


def multi_descs(tab):
    """The rank's batches as cudasp_scan_device_batches descriptors, built
    once as the C array the call takes (Scanner.device_batches), so that a
    step spends no host time converting them."""
    from cudasp_amd import Scanner
    return Scanner.device_batches([dict(tweak_x=tab.cols(tab.tx, b), tweak_y=tab.cols(tab.ty, b), outputs=tab.outs[b], offsets=tab.offs[b],
                 lengths=tab.lens[b], flags=tab.flags[b][:tab.sizes[b]], match_rows=tab.match_rows[b],
                 match_count=tab.match_count[b:b + 1]) for b in range(tab.nb)])


def run_step_multi(tab, scanner, stream, descs, events=None):
    """One pass over the rank's table through cudasp_scan_device_batches: one
    persistent kernel runs both stages over every row of every batch, with
    per-batch flags and match lists (the results of run_step)."""
    tab.match_count.zero_()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        if events is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        scanner.scan_device_batches(descs, stream)
        if events is not None:
            e1.record(stream)
            events.append((e0, e1))


def exclusive_launches(tab, scanner, stream, max_batches):
    """Per-launch kernel durations with each launch ALONE on the GPU: after
    the timed steps, up to `max_batches` full batches go through one stream
    (so no two kernels overlap), HIP events recorded on that stream around
    each stage.  These are the durations a rocprofv3 kernel trace reports for
    the same dispatches (tools/prof_summary.py: `exclusive` = dispatches that
    overlap no other dispatch).  Also re-checks those batches' match counts."""
    full = [b for b in range(tab.nb) if tab.sizes[b] == tab.batch][:max_batches]
    ev = []
    tab.match_count.zero_()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        for b in full:
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record(stream)
            scanner.stage_shared_secret(tab.tx[b], tab.ty[b], tab.sizes[b], stream)
            e1.record(stream)
            scanner.stage_match(tab.outs[b], tab.offs[b], tab.lens[b], tab.sizes[b], tab.flags[b],
                                tab.match_rows[b], tab.match_count[b:b + 1], stream)
            e2.record(stream)
            ev.append((e0, e1, e2))
    stream.synchronize()
    counts = tab.match_count.tolist()
    ok = all(counts[b] == tab.expected_per_batch[b] for b in full)
    a = [e0.elapsed_time(e1) for e0, e1, _ in ev]
    m = [e1.elapsed_time(e2) for _, e1, e2 in ev]
    return dict(launches=len(full), stage_a_ms=float(np.mean(a)) if a else None,
                stage_b_ms=float(np.mean(m)) if m else None, matches_equal_planted=ok)


def layout_probe(lib, tab, reps=5):
    """HBM cost of the data layout alone: k_layout_probe (cudasp_layout_probe)
    over the whole rank table as one column-major launch, reading exactly the
    algorithmic bytes of every row with the kernels' thread
    mapping and no arithmetic.  Timed with HIP events on the current stream,
    after (and outside) the timed bench steps."""
    m = tab.sizes
    x = torch.cat([tab.cols(tab.tx, b) for b in range(tab.nb)], dim=1).contiguous()
    y = torch.cat([tab.cols(tab.ty, b) for b in range(tab.nb)], dim=1).contiguous()
    lens = torch.cat([tab.lens[b][:m[b]] for b in range(tab.nb)]).contiguous()
    per_batch_total = [int(tab.lens[b][:m[b]].to(torch.int64).sum().item()) for b in range(tab.nb)]
    outs = torch.cat([tab.outs[b][:per_batch_total[b]] for b in range(tab.nb)]).contiguous()
    base = 0
    offs_parts = []
    for b in range(tab.nb):
        offs_parts.append(tab.offs[b][:m[b]] + base)
        base += per_batch_total[b]
    offs = torch.cat(offs_parts).contiguous()
    n = x.shape[1]
    flags = torch.zeros(n, dtype=torch.uint8, device=x.device)
    st = _native.stream_arg(torch.cuda.current_stream())

    def launch():
        _native.check(lib.cudasp_layout_probe(x.data_ptr(), y.data_ptr(), n, outs.data_ptr(), offs.data_ptr(),
                                              lens.data_ptr(), flags.data_ptr(), st))
    launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nbytes = n * (64 + 8 + 1) + 8 * int(outs.numel())
    del x, y, lens, outs, offs, flags
    torch.cuda.empty_cache()
    gbs = nbytes / (ms * 1e-3) / 1e9
    return dict(kernel="k_layout_probe", rows=n, outputs_per_row=round(int(base) / n, 3),
                algorithmic_bytes=nbytes, ms=ms, achieved=gbs, peak=HBM_PEAK_GBS, unit="GB/s",
                frac=gbs / HBM_PEAK_GBS,
                note="the scan's algorithmic HBM bytes (73 + 8k per row) moved with the kernels' thread "
                     "mapping and no arithmetic: the layout's own HBM roofline, one launch over the rank table")


def cgroup_cpu_quota():
    """CPUs of this process's cgroup CPU quota (cgroup v2 cpu.max or v1
    cfs_quota_us / cfs_period_us), or None when there is no quota."""
    try:
        with open("/proc/self/cgroup") as f:
            lines = f.read().splitlines()
    except OSError:
        lines = []
    paths = []
    for ln in lines:
        parts = ln.split(":", 2)
        if len(parts) == 3 and (parts[0] == "0" or "cpu" in parts[1].split(",")):
            paths.append((parts[0] == "0", parts[2]))
    for v2, rel in paths + [(True, "/"), (False, "/")]:
        try:
            if v2:
                with open(os.path.join("/sys/fs/cgroup", rel.lstrip("/"), "cpu.max")) as f:
                    q, p = f.read().split()[:2]
                if q != "max":
                    return float(q) / float(p), "cgroup v2 cpu.max"
            else:
                base = os.path.join("/sys/fs/cgroup/cpu", rel.lstrip("/"))
                with open(os.path.join(base, "cpu.cfs_quota_us")) as f:
                    q = int(f.read())
                with open(os.path.join(base, "cpu.cfs_period_us")) as f:
                    p = int(f.read())
                if q > 0:
                    return q / p, "cgroup v1 cfs quota"
        except (OSError, ValueError):
            continue
    return None, None


def host_cores():
    """Host CPUs this process may use: the affinity mask, capped by the
    cgroup CPU quota when one is set; without a quota, by OMP_NUM_THREADS
    when the environment sets it (the GPU pool states the box's CPU share
    there while the mask shows the whole machine, and asks that worker pools
    stay within it).  Returns (cores, visible, source)."""
    visible = len(os.sched_getaffinity(0))
    quota, src = cgroup_cpu_quota()
    if quota is not None and quota < visible:
        return max(1, int(quota)), visible, src
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and 0 < int(omp) < visible:
        return int(omp), visible, "OMP_NUM_THREADS (no cgroup CPU quota; affinity shows %d CPUs)" % visible
    return visible, visible, "sched_getaffinity"


def pinned_leg(args, labels, world, hbm=False):
    """Zero-copy scans of the same table through the C pinned table
    (cudasp_pinned_*, include/cudasp_host.h):
    tools/host_e2e --pinned as a child process builds the table in host
    memory, appends it ONCE (Arrow runs) into pinned memory and scans it 4
    times in place over all `world` GPUs (batches round-robin, one streaming
    kernel per GPU, no host copy per query; each scan binds its keys like a
    query); the first scan warms the scanners and streams, the median of the
    other 3 is reported, and every scan must return exactly the planted rows.
    hbm=True: the same table resident in device memory instead
    (CUDASP_TABLE_HBM: each scan one k_scan_multi launch per GPU)."""
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "tools", "host_e2e")
    if not os.path.exists(exe):
        return dict(error="tools/host_e2e not built (make -C duckdb-cudasp-extension_amd)")
    devices = ",".join(str(r % max(1, torch.cuda.device_count())) for r in range(world))
    cmd = [exe, "--rows", str(args.rows), "--batch", str(args.batch_size), "--labels", str(len(labels)),
           "--reps", "3", "--pinned", devices] + (["--hbm"] if hbm else [])
    cmd += ["--outputs-max", str(args.outputs_max)] if args.outputs_max else ["--outputs", str(args.outputs_per_row)]
    lf = None
    if labels:
        lf = tempfile.NamedTemporaryFile(prefix="cudasp_labels_", suffix=".bin", delete=False)
        lf.write(b"".join(labels))
        lf.close()
        cmd += ["--labels-file", lf.name]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=args.e2e_timeout)
    except subprocess.TimeoutExpired:
        return dict(error="timed out after %d s" % args.e2e_timeout)
    finally:
        if lf is not None:
            os.unlink(lf.name)
    line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else ""
    try:
        res = json.loads(line)
    except ValueError:
        return dict(error="exit %d: %s" % (r.returncode, (r.stderr or r.stdout)[-400:]))
    res["exit_code"] = r.returncode
    res["args"] = " ".join(c if c != (lf.name if lf else None) else "<label keys>" for c in cmd[1:])
    if r.stderr.strip():
        res["stderr_tail"] = r.stderr.strip()[-300:]
    return res


def cold_start_leg(args, world, rows=1_000_000):
    """Cold start: config 2's 1M-row table written once
    by one tools/host_e2e child (--table-out), then fresh children whose first
    GPU work is the first query (--table-in; the process has only initialised
    the HIP runtime): `first_query_s` builds the fixed-base table, the feed
    and its pinned slots inside the query; `first_query_prewarmed_s` runs
    after cudasp_tf_prewarm (what the DuckDB extension starts at LOAD,
    `prewarm_s`).  Both against the same process's warm queries' median;
    every query must emit exactly the planted rows."""
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "tools", "host_e2e")
    if not os.path.exists(exe):
        return dict(error="tools/host_e2e not built (make -C duckdb-cudasp-extension_amd)")
    threads = max(1, min(8 * world, host_cores()[0]))
    fd, path = tempfile.mkstemp(prefix="cudasp_cold_", suffix=".bin")
    os.close(fd)
    base = [exe, "--rows", str(rows), "--threads", str(threads), "--batch", str(args.batch_size), "--outputs", "2"]

    def child(extra):
        try:
            r = subprocess.run(base + extra, capture_output=True, text=True, timeout=args.e2e_timeout)
        except subprocess.TimeoutExpired:
            return dict(error="timed out")
        try:
            d = json.loads(r.stdout.strip().splitlines()[-1])
        except (ValueError, IndexError):
            return dict(error="exit %d: %s" % (r.returncode, (r.stderr or r.stdout)[-300:]))
        d["exit_code"] = r.returncode
        return d

    try:
        gen = child(["--table-out", path])
        if "error" in gen:
            return dict(error="table: " + gen["error"])
        cold = child(["--table-in", path, "--reps", "5"])
        pw = child(["--table-in", path, "--reps", "5", "--prewarm"])
    finally:
        os.unlink(path)
    out = dict(rows=rows, threads=threads, batch_size=args.batch_size,
               note="fresh tools/host_e2e processes, first GPU work = the first query (HIP runtime initialised "
                    "before: hip_init_s); warm = the same process's next 5 queries' median")
    for name, d in (("cold", cold), ("prewarmed", pw)):
        if "error" in d:
            out[name + "_error"] = d["error"]
            continue
        out[name] = dict(first_query_s=d.get("first_query_s"), warm_query_s=d.get("seconds"),
                         ratio=(d["first_query_s"] / d["seconds"]) if d.get("seconds") else None,
                         hip_init_s=d.get("hip_init_s"), prewarm_s=d.get("prewarm_s"),
                         exact=bool(d.get("first_query_exact") and d.get("emitted_equal_planted")),
                         exit_code=d.get("exit_code"))
    out["first_query_s"] = out.get("cold", {}).get("first_query_s")
    out["first_query_prewarmed_s"] = out.get("prewarmed", {}).get("first_query_s")
    return out


def e2e_leg(args, labels, world, fb_bits, mode=None):
    """PCIe-inclusive end-to-end rate through the table-function host
    (include/cudasp_host.h, the calls DuckDB's executor makes) over all
    `world` GPUs: tools/host_e2e as a fresh child process (this process only
    waits for it), the same table shape in host memory -- rows, batch_size,
    label keys (bench.label_keys, passed as a file), outputs per row (fixed k,
    or 1..kmax from the same generators as the device legs) and planted base
    and label matches -- fed as DuckDB-style 2048-row chunks by executor
    threads.  Its first query warms the process (scanners, batch slots,
    fixed-base tables), then `reps` queries are timed and the median is
    reported; every query must emit exactly the planted rows.  The child runs
    with the environment's GPU_MAX_HW_QUEUES (HIP's default 4 unless
    --e2e-hw-queues sets one).  The host's default is its streaming feeds
    (one persistent kernel per device reading the slots in place, DESIGN.md
    section 7c); mode="launch" selects its per-slot launches
    (CUDASP_TF_MODE=launch).  Each query starts from an idle GPU, whose clock
    ramps up during the query; `reps` more queries start right after a 30 ms
    busy kernel (warm_tx_per_s: the host path at full clock)."""
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "tools", "host_e2e")
    if not os.path.exists(exe):
        return dict(error="tools/host_e2e not built (make -C duckdb-cudasp-extension_amd)")
    # 8 executor threads per GPU, but never more than the host cores this
    # process is allotted: oversubscribed threads collapse the host feed
    # (the cgroup's CPU quota throttles them; 64 threads on 16 cores run at
    # ~0.33 G rows/s against ~0.87 G for 16, profiles/r05_host_ceiling.txt)
    threads = args.e2e_threads or max(1, min(8 * world, host_cores()[0]))
    reps = args.e2e_reps or (5 if args.rows <= 2_000_000 else 3 if args.rows <= 10_000_000 else 1)
    env = dict(os.environ, CUDASP_FB_BITS=str(fb_bits))
    env.pop("CUDASP_TF_MODE", None)
    if mode:
        env["CUDASP_TF_MODE"] = mode
    if args.e2e_hw_queues:
        env["GPU_MAX_HW_QUEUES"] = str(args.e2e_hw_queues)
    lf = None
    sample = tempfile.NamedTemporaryFile(prefix="cudasp_e2e_sample_", suffix=".json", delete=False)
    sample.close()
    cmd = [exe, "--rows", str(args.rows), "--threads", str(threads), "--batch", str(args.batch_size),
           "--labels", str(len(labels)), "--input", args.e2e_input, "--reps", str(reps), "--warm-reps", str(reps),
           "--plant-sample", sample.name]
    if labels:
        lf = tempfile.NamedTemporaryFile(prefix="cudasp_labels_", suffix=".bin", delete=False)
        lf.write(b"".join(labels))
        lf.close()
        cmd += ["--labels-file", lf.name]
    cmd += ["--outputs-max", str(args.outputs_max)] if args.outputs_max else ["--outputs", str(args.outputs_per_row)]
    t0 = time.perf_counter()
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=args.e2e_timeout, env=env)
    except subprocess.TimeoutExpired:
        os.unlink(sample.name)
        return dict(error="timed out after %d s" % args.e2e_timeout, cmd=" ".join(cmd[1:]))
    finally:
        if lf is not None:
            os.unlink(lf.name)
    line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else ""
    try:
        res = json.loads(line)
    except ValueError:
        os.unlink(sample.name)
        return dict(error="exit %d: %s" % (r.returncode, (r.stderr or r.stdout)[-400:]), cmd=" ".join(cmd[1:]))
    # the planted values host_e2e wrote came from the GPU's own values path:
    # recompute a strided sample of planted and unplanted rows with the C
    # oracle (checker use of oracle/), so the e2e line's "emitted == planted"
    # is tied to the oracle, not only to the GPU
    try:
        with open(sample.name) as f:
            smp = json.load(f)
        sys.path.insert(0, ROOT)
        from oracle import oracle
        res["planted_oracle_check"] = oracle.check_planted_sample(smp, threads=min(16, host_cores()[0]))
        res["planted_oracle_check"]["note"] = ("host_e2e --plant-sample: 256 planted + 256 unplanted rows strided "
                                               "over the table, recomputed by oracle/cudasp_oracle.c (tweak = "
                                               "(s0 + g) G, planted value, flag, emitted)")
    except (OSError, ValueError, KeyError) as e:
        res["planted_oracle_check"] = dict(error=str(e))
    finally:
        os.unlink(sample.name)
    res["exit_code"] = r.returncode
    res["wall_s"] = round(time.perf_counter() - t0, 2)
    res["args"] = " ".join(c if c != (lf.name if lf else None) else "<label keys>" for c in cmd[1:])
    res["fixed_base_bits"] = fb_bits
    if r.stderr.strip():
        res["stderr_tail"] = r.stderr.strip()[-300:]
    return res


def cpu_sample(tab, sample_rows):
    """The first `sample_rows` rows of the rank table (whole batches, so
    several scanners/streams are covered) in host memory: tweak blobs, the
    outputs CSR and the GPU's flags of the last pass."""
    tw, outs, offs, lens, gflags = [], [], [], [], []
    base, m = 0, 0
    for b in range(tab.nb):
        if m >= sample_rows:
            break
        mb = min(tab.sizes[b], sample_rows - m)
        x = tab.cols(tab.tx, b)[:, :mb].cpu().numpy().view(np.uint32)
        y = tab.cols(tab.ty, b)[:, :mb].cpu().numpy().view(np.uint32)
        tw.append(np.ascontiguousarray(np.concatenate([x.T, y.T], axis=1).astype("<u4")).view(np.uint8).reshape(mb, 64))
        ln = tab.lens[b][:mb].cpu().numpy().view(np.uint32)
        of = tab.offs[b][:mb].cpu().numpy().view(np.uint32)
        used = int(of[-1]) + int(ln[-1]) if mb else 0
        outs.append(tab.outs[b][:used].cpu().numpy())
        offs.append(of + np.uint32(base))
        lens.append(ln)
        gflags.append(tab.flags[b][:mb].cpu().numpy())
        base += used
        m += mb
    return dict(tweaks=np.concatenate(tw), outs=np.concatenate(outs), offs=np.concatenate(offs),
                lens=np.concatenate(lens), gpu_flags=np.concatenate(gflags), rows=m, batches=len(tw))


def cpu_baseline(smp, labels, threads, output_count=1, label_negation=False):
    """The CPU oracle (oracle/cudasp_oracle.c, `port`: a plain restatement of
    the reference's algorithm -- 4x64-bit limbs, 4-bit Jacobian windows, no
    endomorphism) timed on this box's host cores over the sample, its flags
    compared row by row with the GPU's."""
    sys.path.insert(0, ROOT)
    from oracle import oracle  # the C restatement: baseline + checker only
    t0 = time.perf_counter()
    flags, _ = oracle.scan_ex(SCAN_KEY, SPEND_KEY, labels, smp["tweaks"], smp["outs"], smp["offs"], smp["lens"],
                              output_count=output_count, label_negation=label_negation, threads=threads)
    dt = time.perf_counter() - t0
    return dict(value=smp["rows"] / dt, unit="tx/s", cores=threads, kind="port",
                sample="first %d rows (%d batches) of the rank-0 table, %d labels, oracle/cudasp_oracle.c with %d "
                       "pthreads" % (smp["rows"], smp["batches"], len(labels), threads),
                seconds=round(dt, 3), flags_match_gpu=bool(np.array_equal(flags, smp["gpu_flags"])),
                sample_matches=int(flags.sum()))


def planted_oracle_check(tab, labels, threads, count=256):
    """The planted values (computed by the product's values path) of `count`
    planted rows spread over the whole rank table, recomputed by the C oracle:
    ties the full table's expected match count -- not only the CPU sample's
    first rows -- to the oracle.  Checker use of oracle/, in the CPU leg."""
    sys.path.insert(0, ROOT)
    from oracle import oracle
    log = tab.plant_log
    if not log:
        return dict(rows=0)
    pick = [log[int(i * len(log) / min(count, len(log)))] for i in range(min(count, len(log)))]
    tw, want_col, planted = [], [], []
    for b, i, col in pick:
        x = tab.cols(tab.tx, b)[:, i].cpu().numpy().view(np.uint32)
        y = tab.cols(tab.ty, b)[:, i].cpu().numpy().view(np.uint32)
        tw.append(np.concatenate([x, y]).astype("<u4").view(np.uint8))
        want_col.append(col)
        planted.append(int(tab.outs[b][int(tab.offs[b][i].item())].item()))
    _, vals = oracle.scan(SCAN_KEY, SPEND_KEY, labels, np.stack(tw), threads=threads, want_values=True)
    got = [int(vals[r, c]) for r, c in enumerate(want_col)]
    return dict(rows=len(pick), of_planted=len(log), equal=int(sum(g == p for g, p in zip(got, planted))),
                batches=len({b for b, _, _ in pick}), label_columns=sorted({c for c in want_col if c}),
                note="planted values of rows spread over every batch of the rank table, recomputed by "
                     "oracle/cudasp_oracle.c")


def cpu_baseline_optimized(smp, labels, threads):
    """`port-optimized`: the product's own row pipeline (GLV + wNAF, co-Z,
    shared inversions, one-compression SHA-256, batched label inversions)
    compiled for the host at -O3 (tools/cpu_port, 8-bit fixed-base windows
    sized for the CPU cache), timed on the same sample and cores; flags
    compared with the GPU's."""
    import ctypes
    lib_path = os.path.join(ROOT, "tools", "cpu_port", "libcudasp_cpu_port.so")
    if not os.path.exists(lib_path):
        return dict(error="tools/cpu_port not built")
    lib = ctypes.CDLL(lib_path)
    P = ctypes.c_void_p
    lib.cudasp_cpu_port_scan.argtypes = [P, P, P, ctypes.c_uint32, P, ctypes.c_uint32, P, P, P, P, ctypes.c_int]
    lib.cudasp_cpu_port_scan.restype = ctypes.c_int
    n = smp["rows"]
    flags = np.zeros(n, dtype=np.uint8)
    outs = np.ascontiguousarray(smp["outs"], dtype=np.int64)
    lab = b"".join(labels) if labels else None
    t0 = time.perf_counter()
    rc = lib.cudasp_cpu_port_scan(SCAN_KEY, SPEND_KEY, lab, len(labels), smp["tweaks"].ctypes.data, n,
                                  outs.ctypes.data if outs.size else None, smp["offs"].ctypes.data,
                                  smp["lens"].ctypes.data, flags.ctypes.data, threads)
    dt = time.perf_counter() - t0
    if rc != 0:
        return dict(error="cudasp_cpu_port_scan returned %d" % rc)
    return dict(value=n / dt, unit="tx/s", cores=threads, kind="port-optimized",
                sample="first %d rows (%d batches) of the rank-0 table, %d labels, the product's row pipeline "
                       "compiled for the host (tools/cpu_port) on %d threads" % (n, smp["batches"], len(labels),
                                                                                 threads),
                seconds=round(dt, 3), flags_match_gpu=bool(np.array_equal(flags, smp["gpu_flags"])),
                sample_matches=int(flags.sum()))


def cpu_baseline_openssl(smp, labels, threads, rows):
    """`openssl`: the reference's row pipeline on OpenSSL 3's secp256k1
    arithmetic (tools/cpu_openssl) -- the third-party library baseline
    SURVEY.md §8(d) names while libsecp256k1 is absent from the image --
    timed on the first `rows` rows of the sample and the same cores; flags
    compared with the GPU's.  OpenSSL's generic prime-field EC code is not
    libsecp256k1 (~10x slower per SURVEY.md §8(d)), hence the label."""
    import ctypes
    lib_path = os.path.join(ROOT, "tools", "cpu_openssl", "libcudasp_cpu_openssl.so")
    if not os.path.exists(lib_path):
        return dict(error="tools/cpu_openssl not built")
    lib = ctypes.CDLL(lib_path)
    P = ctypes.c_void_p
    lib.cudasp_cpu_openssl_scan.argtypes = [P, P, P, ctypes.c_uint32, P, ctypes.c_uint32, P, P, P, P, ctypes.c_int]
    lib.cudasp_cpu_openssl_scan.restype = ctypes.c_int
    n = min(rows, smp["rows"])
    used = int(smp["offs"][n - 1]) + int(smp["lens"][n - 1]) if n else 0
    flags = np.zeros(n, dtype=np.uint8)
    outs = np.ascontiguousarray(smp["outs"][:used], dtype=np.int64)
    lab = b"".join(labels) if labels else None
    t0 = time.perf_counter()
    rc = lib.cudasp_cpu_openssl_scan(SCAN_KEY, SPEND_KEY, lab, len(labels), smp["tweaks"].ctypes.data, n,
                                     outs.ctypes.data if outs.size else None, smp["offs"].ctypes.data,
                                     smp["lens"].ctypes.data, flags.ctypes.data, threads)
    dt = time.perf_counter() - t0
    if rc < 0:
        return dict(error="cudasp_cpu_openssl_scan returned %d" % rc)
    return dict(value=n / dt, unit="tx/s", cores=threads, kind="openssl",
                sample="first %d rows of the rank-0 table, %d labels, OpenSSL 3 EC_POINT_mul/EC_POINT_add "
                       "(NID_secp256k1) + EVP SHA-256 on %d threads (tools/cpu_openssl)" % (n, len(labels), threads),
                seconds=round(dt, 3), rows_refused=rc,
                flags_match_gpu=bool(np.array_equal(flags, smp["gpu_flags"][:n])), sample_matches=int(flags.sum()))


def cpu_port_sweep(smp, labels, cores, rows):
    """port-optimized at a few thread counts (cores/4, cores/2, cores; never
    more threads than the allotted cores) over the first `rows` rows of the
    sample: how the CPU bar scales with the host share."""
    sub = dict(smp)
    n = min(rows, smp["rows"])
    used = int(smp["offs"][n - 1]) + int(smp["lens"][n - 1]) if n else 0
    sub.update(tweaks=smp["tweaks"][:n], outs=smp["outs"][:used], offs=smp["offs"][:n], lens=smp["lens"][:n],
               gpu_flags=smp["gpu_flags"][:n], rows=n, batches=1)
    out = []
    for t in sorted({max(1, cores // 4), max(1, cores // 2), cores}):
        r = cpu_baseline_optimized(sub, labels, t)
        out.append(dict(threads=t, value=r.get("value"), seconds=r.get("seconds"),
                        flags_match_gpu=r.get("flags_match_gpu"), error=r.get("error")))
    return dict(rows=n, unit="tx/s", kind="port-optimized", points=out)


def stamped_summary(name, key, stamp):
    """The newest profiles/r0N_<name>.json measured on the machine code the
    process loaded: its `code_stamp[key]` (tools/pmc_summary.py --stamp-lib)
    must equal `stamp`, the loaded kernel's (tools/codeobj.py).  Counters of
    another build of the kernel are never used: (None, reason) instead."""
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "r0*_%s.json" % name)), reverse=True)
    seen = []
    for p in paths:
        with open(p) as f:
            d = json.load(f)
        st = ((d.get("code_stamp") or {}).get(key) or {}).get("sha256")
        if stamp and st == stamp:
            return p, d, None
        seen.append("%s: %s" % (os.path.relpath(p, ROOT), st or "unstamped"))
    return None, None, ("no %s summary measured on the loaded %s (stamp %s); on file: %s"
                        % (name, key, stamp, "; ".join(seen) or "none"))


def sq_profile_name(args):
    """The PMC instruction-count summary name matching this run's shape (launch
    mode, labels, outputs per row, fixed-base width, variants):
    pmc_sq_[multi_]L<labels>_k<outputs>_w<bits>[_neg][_K<k>]."""
    kdesc = "1-%d" % args.outputs_max if args.outputs_max else str(args.outputs_per_row)
    name = "pmc_sq_%sL%d_k%s_w%d" % ("multi_" if args.launch == "multi" else "", args.labels, kdesc, args.fb_bits)
    if args.label_negation:
        name += "_neg"
    if args.output_count != 1:
        name += "_K%d" % args.output_count
    return name


def alu_roofline(sq, path, value_per_gpu, multi=False, clock_mhz=None, stamp=None, labels=0):
    """Integer-VALU roofline of the whole path: VALU wave-instructions per row
    (rocprofv3 SQ_INSTS_VALU of a run of the same shape on the same machine
    code, profiles/: k_scan_multi per row with --launch multi, both stage
    kernels per batch otherwise) x rows/s per GPU, against the nominal VALU
    issue rate, the measured VOP3 rate and the kernel's own mix ceiling."""
    per = sq["per_kernel"]
    if multi:
        m = per.get("k_scan_multi", {}).get("SQ_INSTS_VALU")
        rows = sq.get("multi_rows_per_launch")
        if not (m and rows):
            return dict(error="%s lacks k_scan_multi" % os.path.relpath(path, ROOT))
        wi_per_row = m / float(rows)
        per64 = dict(k_scan_multi=wi_per_row * 64)
        g = per.get("k_scan_multi", {}).get("GRBM_GUI_ACTIVE")
        # issue rate in the profiled launch itself: VALU wave-instructions per
        # 4 SIMD cycles (GRBM_GUI_ACTIVE sums the 8 XCDs), clock-independent
        kernel_u = 4 * m / (g / 8 * 1024) if g else None
    else:
        rpl = float(sq.get("rows_per_launch", 300000))
        a = per.get("k_shared_secret", {}).get("SQ_INSTS_VALU")
        bm = per.get("void k_match<false>", {}).get("SQ_INSTS_VALU")
        if not (a and bm):
            return dict(error="%s lacks the stage kernels" % os.path.relpath(path, ROOT))
        wi_per_row = (a + bm) / rpl
        per64 = dict(k_shared_secret=a / rpl * 64, k_match=bm / rpl * 64)
        kernel_u = None
    achieved_wi = wi_per_row * value_per_gpu
    out = dict(bound="valu", unit="wave-instr/s per GPU", achieved=achieved_wi, peak=VALU_WAVE_INSTR_PEAK,
               frac=achieved_wi / VALU_WAVE_INSTR_PEAK, measured_vop3_issue_rate=VOP3_WAVE_INSTR_MEASURED,
               frac_of_measured_vop3_rate=achieved_wi / VOP3_WAVE_INSTR_MEASURED,
               valu_wave_instr_per_64_rows=per64, kernel_U_profiled=kernel_u,
               source=os.path.relpath(path, ROOT), code_stamp=stamp,
               note="SQ_INSTS_VALU per row of a run of this shape on this machine code (%s); peak = nominal VALU "
                    "issue rate; measured_vop3_issue_rate = 8-byte-encoded (VOP3) integer ops alone at 2.4 GHz, "
                    "about half of it -- the kernel's 4-byte VOP2 ops issue faster, so it can exceed 1; "
                    "mix_ceiling is the bound of the kernel's own mix" % sq.get("shape", "see source"))
    if multi:
        mix = mix_ceiling(achieved_wi, clock_mhz, stamp, kernel_u, labels)
        if mix:
            out["mix_ceiling"] = mix
    return out


def mix_ceiling(achieved_wi, clock_mhz, stamp, kernel_u, labels=0):
    """The issue ceiling of the scan's own instruction mix (tools/valu_ceiling.py,
    profiles/r0N_valu_ceiling.json, stamped like the counters).  The stage-A
    ladder's own operations (the Yh-form doubling and addition), run as
    register-resident loops at the kernel's 3 waves per SIMD, issue U_ladder
    VALU wave-instructions per 4 SIMD cycles; they are the ladder's share of
    the kernel's VALU per row (82% at 0 labels, the bench key's 126 doublings
    and 39 additions); the rest issues at most at the 4-byte VOP2 rate (the
    fastest one-opcode loop).  U_max = 1 / (share / U_ladder + (1 - share) /
    U_vop2) bounds the whole mix, and U_max x 1024 SIMDs x f / 4 is the rate
    at clock f -- the timed launch's own shader clock (`clock`), else the
    2.4 GHz peak.  The clock-free form is the profiled launch's U over U_max."""
    path, vc, why = stamped_summary("valu_ceiling", "k_scan_multi", stamp)
    if vc is None:
        return dict(error=why)
    shape = vc.get("k_scan_multi_L%d" % labels) or {}
    u_max = shape.get("mix_U_upper_bound")
    if not u_max:
        return dict(error="%s has no mix bound for %d labels" % (os.path.relpath(path, ROOT), labels))
    f = clock_mhz * 1e6 if clock_mhz else 2.4e9
    ceiling = u_max * 1024 * f / 4
    return dict(mix_U_upper_bound=u_max, ladder_U=vc.get("ladder_mix_U"), ladder_ops=vc.get("ladder_ops"),
                ladder_share=shape.get("ladder_share"), vop2_U=vc.get("vop2_U"), clock_hz=f,
                clock_source="timed launch" if clock_mhz else "peak (no clock read)",
                ceiling_wave_instr_per_s=ceiling, frac=achieved_wi / ceiling,
                kernel_U_profiled=kernel_u, kernel_frac_of_mix_bound_profiled=(kernel_u / u_max) if kernel_u else None,
                source=os.path.relpath(path, ROOT),
                note="U = VALU wave-instructions per 4 SIMD cycles (PMC); U_max = 1 / (share / U_ladder + (1 - share) "
                     "/ U_vop2): the ladder's ops at their measured loop rate, the rest at most at the VOP2 rate; frac "
                     "= achieved / (U_max x SIMDs x clock / 4)")


def timed_steps(step, steps, warmup, device, barrier, counter=None):
    """W untimed then K timed steps, each bracketed by barrier + synchronize;
    returns (per-step seconds, found per step)."""
    found = []
    for _ in range(warmup):
        step()
        torch.cuda.synchronize(device)
        if counter is not None:
            found.append(counter())
    times = []
    events = []
    for _ in range(steps):
        barrier()
        torch.cuda.synchronize(device)
        t0 = time.perf_counter()
        step(events)
        torch.cuda.synchronize(device)
        barrier()
        times.append(time.perf_counter() - t0)
        if counter is not None:
            found.append(counter())
    return times, events, found


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rows", type=int, default=32_700_000,
                    help="rows of the table (rows, roundrobin) or of each rank's table (weak)")
    ap.add_argument("--shard", choices=["rows", "roundrobin", "weak"], default="rows",
                    help="rows: ONE table, every GPU scans its contiguous 1/N share in batch_size-row batches "
                         "(BASELINE configs[3], strong scaling; the reference's and the host's per-GPU batching); "
                         "roundrobin: ONE table cut into global batches, batch b on rank b mod N; "
                         "weak: every rank scans its own table")
    ap.add_argument("--batch-size", type=int, default=300_000,
                    help="rows per batch (the reference's default 300000, BASELINE.md section 3, at every N); "
                         "0 = balanced: the largest size <= 300000 giving every rank the same batch count")
    ap.add_argument("--no-secondary", "--no-balanced", dest="no_secondary", action="store_true",
                    help="at N > 1, skip the secondary value_roundrobin line (whole global batches dealt b mod N)")
    ap.add_argument("--labels", type=int, default=0)
    ap.add_argument("--output-count", type=int, default=1,
                    help="protocol variant: output indices k = 0..K-1 per row (1 = the reference)")
    ap.add_argument("--label-negation", action="store_true", help="protocol variant: labels also negated")
    ap.add_argument("--outputs-per-row", type=int, default=2)
    ap.add_argument("--outputs-max", type=int, default=0,
                    help="variable outputs per row, uniform in [1, N] (15 -> mean 8, config 5); 0 = fixed")
    ap.add_argument("--fb-bits", type=int, default=0, choices=[0, 7, 22, 26],
                    help="fixed-base window width; 0 = the product default (cudasp_default_fixed_base_bits: 26 "
                         "on MI355X, 21.5 GB HBM table; 22: 1.5 GiB; 7: 151.5 KB staged in LDS; same results)")
    ap.add_argument("--launch", choices=["multi", "batches"], default="multi",
                    help="multi: the rank's batches in one cudasp_scan_device_batches call (one persistent kernel "
                         "for both stages); batches: cudasp_scan_device per batch, round-robin over --streams")
    ap.add_argument("--streams", type=int, default=4)
    ap.add_argument("--tail-rows-a", type=int, default=0, help="stage-A rows per thread of the last round of "
                    "launches (one per stream); 0 = automatic")
    ap.add_argument("--tail-rows-b", type=int, default=0)
    ap.add_argument("--exclusive-batches", type=int, default=16,
                    help="full batches timed alone on one stream after the timed steps (roofline kernel_ms)")
    ap.add_argument("--cpu-rows", type=int, default=1200000)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every host core this process may use")
    ap.add_argument("--cpu-sweep-rows", type=int, default=200000,
                    help="rows of the port-optimized thread sweep (0 = no sweep)")
    ap.add_argument("--cpu-openssl-rows", type=int, default=100000,
                    help="rows of the OpenSSL baseline (about 1 ms per row per thread; 0 = skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-layout-probe", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--pinned", action="store_true",
                    help="also run the pinned and resident table legs (cudasp_pinned_*, tools/host_e2e --pinned; "
                         "an API beside the reference's interface, off by default)")
    ap.add_argument("--no-pinned", action="store_true", help=argparse.SUPPRESS)  # the default since round 6
    ap.add_argument("--no-cold-start", action="store_true",
                    help="skip the cold-start leg (fresh processes' first 1M-row query, with and without prewarm)")
    ap.add_argument("--no-e2e-launch", action="store_true",
                    help="skip the second end-to-end leg with the host's per-slot launches (CUDASP_TF_MODE=launch)")
    ap.add_argument("--e2e-threads", type=int, default=0,
                    help="executor threads of the e2e leg; 0 = 8 per GPU, at most the allotted host cores")
    ap.add_argument("--e2e-reps", type=int, default=0, help="timed e2e queries (median); 0 = by table size")
    ap.add_argument("--e2e-input", choices=["rows", "columns", "vectors"], default="rows",
                    help="how the e2e child hands chunks to the host: per-row pointers, Arrow columns, or DuckDB vectors "
                         "(the extension's pass-through form)")
    ap.add_argument("--e2e-hw-queues", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES for the e2e child; 0 = the environment's (HIP default 4)")
    ap.add_argument("--e2e-timeout", type=int, default=600)
    ap.add_argument("--idle-samples", type=int, default=3,
                    help="device-resident steps each after 100 ms of GPU idle (device_after_idle); 0 = none")
    ap.add_argument("--pmc-summary", default="",
                    help="HBM traffic summary (default: the newest profiles/r0N_pmc_hbm_multi.json measured on the "
                         "loaded kernel's machine code); a summary of other machine code is never used")
    ap.add_argument("--pmc-sq", default="", help="SQ counter summary (default: the newest file matching this run's "
                    "shape and the loaded kernel's machine code)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL) for the barrier/max; gloo to rehearse "
                    "several ranks on one GPU")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.batch_size <= 0:
        args.batch_size = balanced_batch_size(args.rows, world) if args.shard != "weak" else 300_000
    if args.fb_bits in (22, 26):
        # the process default for every scanner and the synthetic-table
        # generator (read once by the library); 0 keeps the product default
        os.environ["CUDASP_FB_BITS"] = str(args.fb_bits)
    device = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(device)
    cpu_group = None
    if world > 1:
        import datetime
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(args.dist_backend)
        # host-side waits (the e2e leg) on a CPU group: no collective kernel
        # spins on the other ranks' GPUs meanwhile
        cpu_group = dist.new_group(backend="gloo", timeout=datetime.timedelta(minutes=30))
    lib = _native.load()
    from cudasp_amd import assign_gpu
    product_fb_bits = int(lib.cudasp_default_fixed_base_bits())
    if args.fb_bits == 0:
        args.fb_bits = product_fb_bits

    labels = label_keys(args.labels)
    gen_stream = torch.cuda.Stream(device)
    t_setup = time.perf_counter()
    batches = rank_batches(args.shard, args.rows, args.batch_size, rank, world, assign_gpu)
    tab = Table(lib, device, batches, args.batch_size, args.outputs_per_row, labels, dev_stream=gen_stream,
                kmax=args.outputs_max)
    streams = [torch.cuda.Stream(device) for _ in range(args.streams)]
    scanners = [Scanner(SCAN_KEY, SPEND_KEY, labels, max_rows=args.batch_size, device=device)
                for _ in range(args.streams)]
    for s in scanners:
        s.set_fixed_base_bits(args.fb_bits)
        if args.output_count != 1 or args.label_negation:
            s.set_options(args.output_count, args.label_negation)
    setup_s = time.perf_counter() - t_setup

    def barrier():
        if world > 1:
            dist.barrier()

    multi = args.launch == "multi"
    descs = multi_descs(tab) if multi else None

    def step(events=None):
        if multi:
            run_step_multi(tab, scanners[0], streams[0], descs, events)
        else:
            run_step(tab, scanners, streams, events=events, tail_rows=(args.tail_rows_a, args.tail_rows_b))

    times, events, step_found = timed_steps(step, args.steps, args.warmup, device, barrier,
                                            lambda: int(tab.match_count.sum().item()))
    total_s = float(np.sum(times))
    found = int(tab.match_count.sum().item())
    flagged = int(tab.flags.sum().item())
    if found != tab.expected or flagged != tab.expected:
        per = tab.match_count.tolist()
        bad = [(b, per[b], tab.expected_per_batch[b]) for b in range(tab.nb) if per[b] != tab.expected_per_batch[b]]
        # Diagnostic only: the reported `matches` are the timed steps' counts above.
        print("rank %d: %d found, %d flagged, %d planted; found per step %s; batches (index, found, planted) "
              "that differ: %s" % (rank, found, flagged, tab.expected, step_found, bad[:16]), file=sys.stderr, flush=True)
    # the shader clock of the last timed launch (the grid's first wave's
    # s_memtime over s_memrealtime; boxes of the pool differ by a few percent)
    clock = None
    if multi:
        mhz, secs = ctypes.c_double(0), ctypes.c_double(0)
        if lib.cudasp_debug_multi_clock(device, ctypes.byref(mhz), ctypes.byref(secs)) == 0:
            clock = dict(shader_mhz=round(mhz.value, 1), wave_s=round(secs.value, 4),
                         note="last timed k_scan_multi launch: its first wave's s_memtime ticks over s_memrealtime")
    total_s, found, flagged, expected = aggregate(world, args.dist_backend, total_s, found, flagged, tab.expected)
    after_idle = None
    if multi and world == 1 and args.idle_samples:
        # The same step started after 100 ms of GPU idle, as every end-to-end
        # query starts (the clock ramps up within it): the device rate to set
        # the e2e leg against.  After the timed region; never the value.
        idle_s = []
        for _ in range(args.idle_samples):
            torch.cuda.synchronize(device)
            time.sleep(0.1)
            t0 = time.perf_counter()
            step()
            torch.cuda.synchronize(device)
            idle_s.append(time.perf_counter() - t0)
        med = float(np.median(idle_s))
        after_idle = dict(tx_s=args.rows / med, ms=med * 1e3, samples=[round(x * 1e3, 3) for x in idle_s],
                          note="one device-resident step after 100 ms of GPU idle, median of the samples")

    # Per-launch kernel durations.  multi: the step is ONE k_scan_multi launch,
    # timed by the HIP events around it on its stream (it runs alone), so
    # kernel_ms is that launch's duration.  batches: the timed steps run 4
    # streams at once, so a launch's event span there includes time shared with
    # the other streams' kernels (launch_span_ms_concurrent); kernel_ms is the
    # duration of a stage-A launch alone on the GPU (exclusive_launches, after
    # the timed region).  Both modes also report the per-batch kernels alone.
    excl = exclusive_launches(tab, scanners[0], streams[0], args.exclusive_batches)
    mean_k = tab.total_outputs / max(1, tab.rows)
    # Counters are read only from summaries stamped with the machine code of
    # the kernel this process loaded (tools/codeobj.py): the timed kernel's
    # instance, k_scan_multi<fb_bits, pipelined> or stage A's k_shared_secret<4>.
    lib_path = os.environ.get("CUDASP_LIB") or _native.LIB_PATH
    skey = "k_scan_multi" if multi else "k_shared_secret"
    spat = codeobj.multi_pattern(args.fb_bits) if multi else r"^_Z15k_shared_secretILi4EE"
    try:
        stamp = codeobj.kernel_stamp(lib_path, spat)["sha256"]
        probe_stamp = codeobj.kernel_stamp(lib_path, codeobj.K_LAYOUT_PROBE)["sha256"]
    except (OSError, ValueError) as e:
        stamp = probe_stamp = None
        print("bench: no code stamp (%s): counters unused" % e, file=sys.stderr)

    def summary(explicit, name):
        if explicit:
            with open(explicit) as f:
                d = json.load(f)
            st = ((d.get("code_stamp") or {}).get(skey) or {}).get("sha256")
            if stamp and st == stamp:
                return explicit, d, None
            return None, None, "%s: stamp %s, loaded %s %s" % (explicit, st or "none", skey, stamp)
        return stamped_summary(name, skey, stamp)

    hbm_path, pmc, traffic_why = summary(args.pmc_summary, "pmc_hbm_multi" if multi else "pmc_hbm_k_shared_secret")
    if pmc and not args.pmc_summary and (args.labels or args.outputs_max or args.outputs_per_row != 2 or
                                         args.output_count != 1 or args.label_negation):
        # the HBM passes profile config 4's row shape (0 labels, 2 outputs per row)
        hbm_path, pmc, traffic_why = None, None, "HBM counters are measured at config 4's row shape only " \
                                                 "(0 labels, 2 outputs/row)"
    pmc = pmc or {}
    traffic = None
    if multi:
        spans = [e0.elapsed_time(e1) for e0, e1 in events]
        kernel, kernel_ms, rows_per_launch, launches = "k_scan_multi", float(np.mean(spans)), float(tab.rows), 1
        kernel_ms_how = ("the step's one k_scan_multi launch (both stages, all %d batches), HIP events on its stream "
                         "around each timed step's call (descriptor upload and counter reset included)" % tab.nb)
        per_row = pmc.get("multi_hbm_bytes_per_row")
        traffic = per_row * rows_per_launch if per_row else None
        extra = dict(per_batch_stage_a_ms_alone=excl["stage_a_ms"], per_batch_stage_b_ms_alone=excl["stage_b_ms"])
    else:
        ka = [e0.elapsed_time(e1) for e0, e1, _ in events]
        kb = [e1.elapsed_time(e2) for _, e1, e2 in events]
        kernel, rows_per_launch, launches = "k_shared_secret", float(args.batch_size), tab.nb
        kernel_ms = excl["stage_a_ms"] or float(np.mean(ka))
        kernel_ms_how = ("stage-A launch alone on the GPU: %d full batches on one stream after the timed steps, HIP "
                         "events on that stream" % excl["launches"])
        traffic = pmc.get("hbm_bytes_per_launch")
        extra = dict(match_kernel_ms=excl["stage_b_ms"],
                     launch_span_ms_concurrent=float(np.mean(ka)) if ka else None,
                     match_launch_span_ms_concurrent=float(np.mean(kb)) if kb else None, streams=args.streams)
    algo_bytes = bytes_per_row(mean_k) * rows_per_launch
    achieved_gbs = algo_bytes / (kernel_ms * 1e-3) / 1e9

    rows_job = args.rows * (world if args.shard == "weak" else 1)  # rows all ranks scan per step
    value = rows_job * args.steps / total_s
    ms_per_step = total_s / args.steps * 1e3
    rows_gpu_step = rows_job / world
    step_gbs = bytes_per_row(mean_k) * rows_gpu_step / (ms_per_step * 1e-3) / 1e9
    sq_path, sq, sq_why = summary(args.pmc_sq, sq_profile_name(args))
    if sq is None:
        alu = dict(bound="valu", error=sq_why, code_stamp=stamp)
    else:
        alu = alu_roofline(sq, sq_path, value / world, multi, clock["shader_mhz"] if clock else None, stamp,
                           args.labels)

    result = dict(
        metric=METRIC, value=value, unit="tx/s", n_gpus=world, steps=args.steps, warmup=args.warmup,
        ms_per_step=ms_per_step, higher_is_better=True,
        scaling="weak" if args.shard == "weak" else "strong", vs_baseline=None,
        dtype="u32", data="synthetic",
        config=dict(workload="%.1fM-row synthetic tweak table%s, %d labels, %s outputs/row, batch_size %d, "
                             "device-resident; %s" % (
                                 args.rows / 1e6, " per rank" if args.shard == "weak" else "", args.labels,
                                 ("1..%d (mean %.2f)" % (args.outputs_max, mean_k)) if args.outputs_max
                                 else str(args.outputs_per_row), args.batch_size,
                                 SHARD_DESC[args.shard]),
                    rows=args.rows, shard=args.shard, batch_size=args.batch_size, labels=args.labels,
                    output_count=args.output_count, label_negation=args.label_negation,
                    outputs_per_row=round(mean_k, 3), fixed_base_bits=args.fb_bits,
                    fixed_base_bits_product_default=product_fb_bits, spend_key_folded=scanners[0].spend_folded,
                    launch=args.launch,
                    streams=1 if multi else args.streams, batches_rank0=tab.nb, parallelism="dp%d" % world),
        roofline=dict(bound="hbm", achieved=achieved_gbs, peak=HBM_PEAK_GBS, unit="GB/s",
                      frac=achieved_gbs / HBM_PEAK_GBS, traffic=traffic,
                      traffic_ratio=(traffic / algo_bytes) if traffic else None,
                      traffic_source=os.path.relpath(hbm_path, ROOT) if hbm_path else None,
                      traffic_null_reason=None if traffic else traffic_why, code_stamp=stamp,
                      traffic_counts=("2 x FETCH_SIZE + WRITE_SIZE (rocprofv3 --pmc derived counters, the "
                                      "MI355X_MICROARCH.md gfx950 correction) per launch: L2-to-fabric traffic, so "
                                      "MALL (Infinity Cache) hits are included -- an upper bound on HBM bytes; the "
                                      "excess over the algorithmic bytes is the per-thread scratch (odd-multiple "
                                      "tables, pending rows) leaving L2, DESIGN.md section 5"
                                      if traffic else None),
                      kernel=kernel, kernel_ms=kernel_ms, kernel_ms_how=kernel_ms_how,
                      algorithmic_bytes_per_launch=algo_bytes, rows_per_launch=rows_per_launch,
                      launches_per_step_rank0=launches,
                      step_achieved=step_gbs, step_frac=step_gbs / HBM_PEAK_GBS,
                      step_note="whole step: rows x (73 + 8k) B per GPU / ms_per_step",
                      note="integer-VALU-bound path; see alu_roofline", **extra),
        alu_roofline=alu,
        matches=dict(found=found, flagged=flagged, expected_planted=expected,
                     label_indices_planted=sorted(tab.planted_labels) if labels else [],
                     exclusive_pass_matches_equal_planted=excl["matches_equal_planted"]),
        setup_s=round(setup_s, 2),
    )
    if after_idle:
        result["device_after_idle"] = after_idle
    if clock:
        result["clock"] = clock
    if not args.no_layout_probe:
        result["layout_probe"] = layout_probe(lib, tab)
        probe_ok = ((pmc.get("code_stamp") or {}).get("k_layout_probe") or {}).get("sha256") == probe_stamp
        if pmc and probe_ok and not args.outputs_max and args.outputs_per_row == 2:
            # the PMC pass profiles the probe at 2 outputs per row (tools/recipes/pmc.sh)
            probe_traffic = pmc.get("probe_hbm_bytes_per_row")
            if probe_traffic:
                result["layout_probe"]["traffic_per_row"] = probe_traffic
                result["layout_probe"]["traffic_ratio"] = probe_traffic / (result["layout_probe"]["algorithmic_bytes"]
                                                                           / result["layout_probe"]["rows"])
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        use, visible, source = host_cores()
        threads = args.cpu_threads or use
        smp = cpu_sample(tab, args.cpu_rows)
        result["host_cores_allotted"] = dict(cores=use, source=source, visible=visible,
                                             omp_num_threads=os.environ.get("OMP_NUM_THREADS"))
        # cpu_baseline is the strongest CPU restatement the image allows:
        # port-optimized (the product's GLV/wNAF/co-Z row pipeline compiled
        # for the host) where it covers the options, else the oracle port;
        # the oracle port is kept beside it as cpu_baseline_port
        port = cpu_baseline(smp, labels, threads, args.output_count, args.label_negation)
        port["host_cpus_visible"] = visible
        result["cpu_baseline"] = port
        result["planted_oracle_check"] = planted_oracle_check(tab, labels, threads)
        if args.output_count == 1 and not args.label_negation:
            opt = cpu_baseline_optimized(smp, labels, threads)
            if "value" in opt:
                opt["host_cpus_visible"] = visible
                result["cpu_baseline"] = opt
                result["cpu_baseline_port"] = port
            else:
                result["cpu_baseline_optimized_error"] = opt.get("error")
            if args.cpu_sweep_rows:
                result["cpu_baseline_optimized_sweep"] = cpu_port_sweep(smp, labels, use, args.cpu_sweep_rows)
            if args.cpu_openssl_rows:
                result["cpu_baseline_openssl"] = cpu_baseline_openssl(smp, labels, threads, args.cpu_openssl_rows)
        del smp

    # Secondary line at N > 1: the same table and batch_size, cut into global
    # batches dealt round-robin (whole batches: the largest share sets the
    # job time).  Never the headline.
    if world > 1 and args.shard == "rows" and multi and not args.no_secondary:
        del descs, tab
        torch.cuda.empty_cache()
        rtab = Table(lib, device, rank_batches("roundrobin", args.rows, args.batch_size, rank, world, assign_gpu),
                     args.batch_size, args.outputs_per_row, labels, dev_stream=gen_stream, kmax=args.outputs_max)
        rdescs = multi_descs(rtab)
        rtimes, _, _ = timed_steps(lambda ev=None: run_step_multi(rtab, scanners[0], streams[0], rdescs, ev),
                                   args.steps, args.warmup, device, barrier)
        rfound = int(rtab.match_count.sum().item())
        rt, rfound, _, rexp = aggregate(world, args.dist_backend, float(np.sum(rtimes)), rfound, 0, rtab.expected)
        result["value_roundrobin"] = args.rows * args.steps / rt
        result["roundrobin"] = dict(batch_size=args.batch_size, batches=-(-args.rows // args.batch_size),
                                    batches_rank0=rtab.nb, ms_per_step=rt / args.steps * 1e3, found=rfound,
                                    expected_planted=rexp, note="secondary: " + SHARD_DESC["roundrobin"])
        del rdescs, rtab
        torch.cuda.empty_cache()
    else:
        del descs, tab
        torch.cuda.empty_cache()
    for s in scanners:
        s.close()

    if not args.no_e2e and args.output_count == 1 and not args.label_negation:
        # After the device-resident legs: rank 0 starts the end-to-end child
        # over all N GPUs while the other ranks wait at a CPU barrier.
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier(group=cpu_group)
        if rank == 0:
            e2e = e2e_leg(args, labels, world, args.fb_bits)
            result["e2e"] = e2e
            result["e2e_tx_s"] = e2e.get("tx_per_s")
            result["e2e_warm_tx_s"] = e2e.get("warm_tx_per_s")
            if after_idle and e2e.get("tx_per_s"):
                # like for like: both start from an idle GPU / both at full clock
                result["e2e_vs_device"] = dict(
                    cold=e2e["tx_per_s"] / after_idle["tx_s"],
                    warm=(e2e.get("warm_tx_per_s") or 0) / value,
                    note="e2e_tx_s / device_after_idle.tx_s, and e2e_warm_tx_s / value (back-to-back steps)")
            if not args.no_e2e_launch:
                # the same child with the host's per-slot launches (each slot
                # copied to the device and scanned by its own k_scan_multi)
                el = e2e_leg(args, labels, world, args.fb_bits, mode="launch")
                result["e2e_launch"] = el
                result["e2e_launch_tx_s"] = el.get("tx_per_s")
            if not args.no_cold_start and args.fb_bits == product_fb_bits:
                result["cold_start"] = cold_start_leg(args, world)
            if args.pinned and args.fb_bits in (0, 26) and args.rows <= 40_000_000:
                # (the child rebuilds the table in host memory: bounded to config-4 sizes)
                # the table pinned once and scanned in place: no host copy per query
                pn = pinned_leg(args, labels, world)
                result["pinned"] = pn
                result["pinned_tx_s"] = pn.get("tx_per_s")
                rs = pinned_leg(args, labels, world, hbm=True)
                result["resident"] = rs
                result["resident_tx_s"] = rs.get("tx_per_s")
        if world > 1:
            dist.barrier(group=cpu_group)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
