"""CPU: the work distribution of the multi-batch persistent kernel (k_scan_multi,
duckdb-cudasp-extension_amd/csrc/scan_multi.hpp) replayed on the host with the
kernel's own helpers.  Whatever the interleaving of the waves' counter reads and
adds, every row of every batch is scanned by exactly one active lane, padding
lanes stay inactive, and the guided schedule ends on one-row pieces."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
RMAX = 6  # CUDASP_MULTI_RMAX


@pytest.fixture(scope="module")
def emu():
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "native")])
    lib = ctypes.CDLL(os.path.join(HERE, "native", "libcudasp_emu29.so"))
    V, U = ctypes.c_void_p, ctypes.c_uint32
    lib.emu_multi_schedule.argtypes = [V, U, U, U, U, U, ctypes.c_uint64, V, V]
    return lib


def schedule(emu, sizes, waves, g1, g2, rmax=RMAX, seed=1):
    sizes = np.asarray(sizes, dtype=np.uint32)
    cover = np.zeros(max(1, int(sizes.sum())), dtype=np.uint32)
    stats = np.zeros(5, dtype=np.uint64)
    rc = emu.emu_multi_schedule(sizes.ctypes.data, len(sizes), waves, g1, g2, rmax, seed,
                                cover.ctypes.data, stats.ctypes.data)
    assert rc == 0
    return cover[: int(sizes.sum())], stats


# the GPU test's ragged batch set (tests/test_multi_batch_gpu.py), bench-like
# batches, and a single fused batch (g1 = g2 = 0)
CASES = [
    ([3001, 64, 1, 0, 129, 70000, 65, 2047], 48, 72, 192),
    ([300000] * 5, 3072, 4608, 12288),
    ([0, 0, 7], 12, 18, 48),
    ([1] * 300, 12, 18, 48),
    ([65536 + 63, 64 * 1000 + 1], 768, 1152, 3072),
    ([300000], 294, 0, 0),
]


@pytest.mark.parametrize("sizes,waves,g1,g2", CASES)
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_every_row_once(emu, sizes, waves, g1, g2, seed):
    cover, stats = schedule(emu, sizes, waves, g1, g2, seed=seed)
    assert cover.size == sum(sizes)
    assert np.all(cover == 1)
    wr = sum((n + 63) // 64 for n in sizes)
    assert stats[3] == stats[0] + stats[1] + stats[2]
    # pieces past the end only at the tail: at most one per wave
    assert stats[4] <= waves
    assert stats[0] * RMAX + stats[1] * 2 + stats[2] >= wr


def test_guided_tail(emu):
    """With the bench's thresholds the bulk runs RMAX rows per thread and the tail
    goes in 2- and 1-row pieces.  The replay lets a wave size its piece from a
    counter value up to a whole round of the other waves old (on the GPU the
    read and the add are back to back), so only the shape is checked."""
    waves, g1, g2 = 3072, 4608, 12288
    sizes = [300000] * 20
    cover, stats = schedule(emu, sizes, waves, g1, g2)
    assert np.all(cover == 1)
    wr = sum((n + 63) // 64 for n in sizes)
    assert stats[0] * RMAX >= wr - g2 - RMAX * waves  # bulk in rmax pieces (stale reads aside)
    assert stats[1] > 0 and stats[2] > 0


def test_fixed_pieces(emu):
    """g1 = g2 = 0 (the fused single-batch launch): every piece has rmax rows."""
    cover, stats = schedule(emu, [100000], 300, 0, 0)
    assert np.all(cover == 1)
    assert stats[1] == 0 and stats[2] == 0
    assert stats[0] == -(-((100000 + 63) // 64) // RMAX)


def test_empty(emu):
    cover, stats = schedule(emu, [0, 0], 12, 18, 48)
    assert cover.size == 0 and stats[3] == 0
