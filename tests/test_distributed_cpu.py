"""CPU, world_size 2 over gloo: the benchmark's multi-GPU sharding and
cross-rank reduction, with the C oracle standing in for each rank's GPU scan.

* rows (BASELINE configs[3], the bench default): ONE table, every rank scans
  its contiguous 1/N share of the rows in batch_size-row batches (a partial
  last batch per rank) -- the per-GPU batching of the reference's executor
  threads and of the product host's device feeds.  The ranks' rows must
  partition the table and the union of their matches equal a single scan.
* roundrobin (the N > 1 secondary line): ONE table cut into
  batch_size-row batches, batch b scanned by rank cudasp_assign_gpu(b, N) --
  the product's own assignment function from libcudasp_amd.so (host-only
  code, the round-robin of src/cudasp_extension.cu:523-529).  The ranks'
  batches must partition the table, and the union of their matches must equal
  a single-process scan of the whole table.
* weak: every rank scans its own table (bench.shard_first_row).
The job time is the max over ranks, match counts the sum (bench.aggregate)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "duckdb-cudasp-extension_amd")
ROWS = 46          # global table (roundrobin): 6 batches of 8, the last one short
BATCH = 8
ROWS_PER_RANK = 24  # weak


def _paths():
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)


def _scan_rows(global_rows):
    """Oracle scan of the given global row indices of the synthetic table:
    every 5th global row carries its true value.  -> (flags, planted)."""
    _paths()
    import bench
    from oracle import oracle
    s0 = bench.synth_s0()
    n = len(global_rows)
    if n == 0:
        return np.zeros(0, dtype=np.uint8), 0
    tweaks = np.frombuffer(b"".join(oracle.synth_tweak(s0, g) for g in global_rows),
                           dtype=np.uint8).reshape(n, 64)
    _, vals = oracle.scan(bench.SCAN_KEY, bench.SPEND_KEY, [], tweaks, want_values=True)
    outs = np.array([[g * 7 + 1, 0] for g in global_rows], dtype=np.int64)
    planted = [i for i, g in enumerate(global_rows) if g % 5 == 0]
    for i in planted:
        outs[i, 1] = vals[i, 0]
    flags, _ = oracle.scan(bench.SCAN_KEY, bench.SPEND_KEY, [], tweaks, outs.reshape(-1),
                           np.arange(n, dtype=np.uint32) * 2, np.full(n, 2, dtype=np.uint32))
    return flags, len(planted)


def _worker(rank, world, port, shard, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _paths()
    import bench
    from cudasp_amd import assign_gpu
    rows = ROWS_PER_RANK if shard == "weak" else ROWS
    batches = bench.rank_batches(shard, rows, BATCH, rank, world, assign_gpu)
    global_rows = [g0 + i for g0, m in batches for i in range(m)]
    flags, planted = _scan_rows(global_rows)
    t, found, flagged, expected = bench.aggregate(world, "gloo", 1.0 + rank, int(flags.sum()), int(flags.sum()),
                                                  planted)
    gathered = [None] * world
    dist.all_gather_object(gathered, global_rows)
    if rank == 0:
        q.put((t, found, flagged, expected, gathered))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(shard, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, shard, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    return q.get(timeout=5)


def test_assignment_is_round_robin():
    _paths()
    from cudasp_amd import assign_gpu
    assert [assign_gpu(b, 3) for b in range(7)] == [0, 1, 2, 0, 1, 2, 0]
    assert [assign_gpu(b, 1) for b in range(3)] == [0, 0, 0]
    assert assign_gpu(2**40 + 5, 8) == 5


def test_two_rank_roundrobin_equals_single_scan():
    t, found, flagged, expected, gathered = _run("roundrobin")
    # the ranks' batches partition the one table: rank r holds batches b = r mod 2
    assert sorted(r for rows in gathered for r in rows) == list(range(ROWS))
    assert gathered[0][:BATCH] == list(range(0, BATCH)) and gathered[1][:BATCH] == list(range(BATCH, 2 * BATCH))
    flags_all, planted_all = _scan_rows(list(range(ROWS)))
    assert t == 2.0  # max over ranks
    assert found == flagged == int(flags_all.sum()) == planted_all == expected


def test_two_rank_row_shares_equal_single_scan():
    t, found, flagged, expected, gathered = _run("rows")
    assert gathered[0] == list(range(ROWS // 2)) and gathered[1] == list(range(ROWS // 2, ROWS))
    flags_all, planted_all = _scan_rows(list(range(ROWS)))
    assert t == 2.0
    assert found == flagged == int(flags_all.sum()) == planted_all == expected


def test_row_shares_cover_config4_table():
    """The default bench shape: 32.7M rows over 1, 2, 4 and 8 ranks with
    batch_size 300000 at every N: contiguous shares partition the table,
    differ by at most one row, and every batch holds <= 300000 rows with only
    each rank's last batch short; at N = 1 the batches are the round-robin
    cut's (109 full batches)."""
    _paths()
    import bench
    from cudasp_amd import assign_gpu
    rows, batch = 32_700_000, 300_000
    assert bench.rank_batches("rows", rows, batch, 0, 1, assign_gpu) == \
        bench.rank_batches("roundrobin", rows, batch, 0, 1, assign_gpu)
    for world in (1, 2, 3, 4, 8):
        per = [bench.rank_batches("rows", rows, batch, r, world, assign_gpu) for r in range(world)]
        covered = []
        for p in per:
            assert all(m == batch for _, m in p[:-1]) and 0 < p[-1][1] <= batch
            for (g0, m), (g1, _) in zip(p, p[1:]):
                assert g1 == g0 + m
            covered.append((p[0][0], p[-1][0] + p[-1][1]))
        assert covered[0][0] == 0 and covered[-1][1] == rows
        assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))
        shares = [e - b for b, e in covered]
        assert max(shares) - min(shares) <= 1
    # N = 8: 4,087,500 rows per GPU = 13 full batches + 187,500
    p = bench.rank_batches("rows", rows, batch, 7, 8, assign_gpu)
    assert len(p) == 14 and p[-1][1] == 187_500


def test_two_rank_weak_shards_equal_single_scan():
    t, found, flagged, expected, gathered = _run("weak")
    assert gathered[0] == list(range(ROWS_PER_RANK))
    assert gathered[1] == list(range(ROWS_PER_RANK, 2 * ROWS_PER_RANK))
    flags_all, planted_all = _scan_rows(list(range(2 * ROWS_PER_RANK)))
    assert t == 2.0
    assert found == flagged == int(flags_all.sum()) == planted_all == expected


def test_rank_batches_cover_config4_table():
    """The default bench shape: 32.7M rows in 300000-row batches (109 full
    batches) over 1, 2, 4 and 8 ranks: every batch on exactly one rank, rank
    loads differ by at most one batch."""
    _paths()
    import bench
    from cudasp_amd import assign_gpu
    rows, batch = 32_700_000, 300_000
    for world in (1, 2, 4, 8):
        per = [bench.rank_batches("roundrobin", rows, batch, r, world, assign_gpu) for r in range(world)]
        firsts = sorted(g0 for p in per for g0, _ in p)
        assert firsts == list(range(0, rows, batch))
        assert sum(m for p in per for _, m in p) == rows
        loads = [len(p) for p in per]
        assert max(loads) - min(loads) <= 1


def test_balanced_batch_size_equal_rank_shares():
    """`--batch-size 0` (balanced): 300000 at N = 1 (the reference's
    default); at N = 2/4/8 every rank gets the same number of batches, the
    batches cover the table exactly, and rank row counts differ by less than
    one batch (only the short last batch differs)."""
    _paths()
    import bench
    from cudasp_amd import assign_gpu
    rows = 32_700_000
    assert bench.balanced_batch_size(rows, 1) == 300_000
    assert bench.balanced_batch_size(rows, 8) == 291_965
    # configs[1]/[2] state batch_size=300000: one GPU keeps it whatever the rows
    for r in (1_000_000, 9_400_000, 100_000_000):
        assert bench.balanced_batch_size(r, 1) == 300_000
    for world in (1, 2, 3, 4, 8):
        batch = bench.balanced_batch_size(rows, world)
        assert batch <= 300_000
        per = [bench.rank_batches("roundrobin", rows, batch, r, world, assign_gpu) for r in range(world)]
        assert len({len(p) for p in per}) == 1
        firsts = sorted(g0 for p in per for g0, _ in p)
        assert firsts == list(range(0, rows, batch))
        shares = [sum(m for _, m in p) for p in per]
        assert sum(shares) == rows
        assert max(shares) - min(shares) < batch
    for rows in (1, 1000, 299_999, 300_001, 1_000_000):
        for world in (1, 2, 8):
            batch = bench.balanced_batch_size(rows, world)
            assert 0 < batch <= 300_000
            assert -(-rows // batch) <= -(-(-(-rows // 300_000)) // world) * world
