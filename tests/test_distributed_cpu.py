"""CPU, world_size 2 over gloo: the benchmark's sharding and cross-rank
reduction (bench.shard_first_row / bench.aggregate), with the C oracle standing
in for the GPU scan of each rank's shard.  The union of the shards must equal a
single-process scan of the whole table, and the job time must be the max."""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
ROWS_PER_RANK = 24


def _table(first, rows):
    import sys
    sys.path.insert(0, ROOT)
    import bench
    from oracle import oracle
    s0 = bench.synth_s0()
    tweaks = np.frombuffer(b"".join(oracle.synth_tweak(s0, first + i) for i in range(rows)),
                           dtype=np.uint8).reshape(rows, 64)
    _, vals = oracle.scan(bench.SCAN_KEY, bench.SPEND_KEY, [], tweaks, want_values=True)
    outs = np.array([[i * 7 + 1, 0] for i in range(rows)], dtype=np.int64)
    planted = [i for i in range(rows) if (first + i) % 5 == 0]
    for i in planted:
        outs[i, 1] = vals[i, 0]
    flags, _ = oracle.scan(bench.SCAN_KEY, bench.SPEND_KEY, [], tweaks, outs.reshape(-1),
                           np.arange(rows, dtype=np.uint32) * 2, np.full(rows, 2, dtype=np.uint32))
    return flags, len(planted)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    sys.path.insert(0, ROOT)
    import bench
    first = bench.shard_first_row(rank, ROWS_PER_RANK)
    flags, planted = _table(first, ROWS_PER_RANK)
    t, found, flagged, expected = bench.aggregate(world, "gloo", 1.0 + rank, int(flags.sum()), int(flags.sum()),
                                                  planted)
    if rank == 0:
        q.put((t, found, flagged, expected))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_shards_equal_single_scan():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs)
    t, found, flagged, expected = q.get(timeout=5)
    flags_all, planted_all = _table(0, world * ROWS_PER_RANK)
    assert t == 2.0  # max over ranks
    assert found == flagged == int(flags_all.sum()) == planted_all == expected

