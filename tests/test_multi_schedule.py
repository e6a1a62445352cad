"""CPU: the work distribution of the multi-batch persistent kernel (k_scan_multi,
duckdb-cudasp-extension_amd/csrc/scan_multi.hpp) replayed on the host with the
kernel's own helpers.  Whatever the interleaving of the waves' counter reads and
adds, every row of every batch is scanned by exactly one active lane and padding
lanes stay inactive; the guided rule sizes pieces by the work left."""
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
    lib.emu_multi_schedule.argtypes = [V, U, U, U, U, U, U, U, ctypes.c_uint64, V, V]
    return lib


NO_YOUNG = 0xFFFFFFFF


def schedule(emu, sizes, waves, g1, g2, rmax=RMAX, seed=1, adaptive=0, young_from=NO_YOUNG):
    """cover per row; stats: pieces by size (index r - 1), total, past the end,
    waves that left without claiming (waves >= young_from are the SIMDs'
    youngest)."""
    sizes = np.asarray(sizes, dtype=np.uint32)
    cover = np.zeros(max(1, int(sizes.sum())), dtype=np.uint32)
    stats = np.zeros(19, dtype=np.uint64)
    rc = emu.emu_multi_schedule(sizes.ctypes.data, len(sizes), waves, g1, g2, rmax, adaptive, young_from, seed,
                                cover.ctypes.data, stats.ctypes.data)
    assert rc == 0
    return cover[: int(sizes.sum())], stats


def wave_rows(sizes):
    return sum((n + 63) // 64 for n in sizes)


# the GPU test's ragged batch set (tests/test_multi_batch_gpu.py), bench-like
# batches, and a single fused batch (g1 = 0); g1 = waves is the default rule,
# g2 > 0 adds a leading rmax phase
CASES = [
    ([3001, 64, 1, 0, 129, 70000, 65, 2047], 48, 48, 0),
    ([3001, 64, 1, 0, 129, 70000, 65, 2047], 48, 72, 192),
    ([300000] * 5, 3072, 3072, 0),
    ([0, 0, 7], 12, 12, 0),
    ([1] * 300, 12, 12, 0),
    ([65536 + 63, 64 * 1000 + 1], 768, 768, 0),
    ([300000], 294, 0, 0),
]


@pytest.mark.parametrize("sizes,waves,g1,g2", CASES)
@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("adaptive", [0, 1])
def test_every_row_once(emu, sizes, waves, g1, g2, seed, adaptive):
    cover, stats = schedule(emu, sizes, waves, g1, g2, seed=seed, adaptive=adaptive)
    assert cover.size == sum(sizes)
    assert np.all(cover == 1)
    assert stats[16] == stats[:16].sum()
    # pieces past the end only at the tail: at most one per wave
    assert stats[17] <= waves
    assert sum((r + 1) * int(stats[r]) for r in range(16)) >= wave_rows(sizes)
    assert stats[RMAX:16].sum() == 0  # never more than rmax rows


def test_guided_rule_sizes(emu):
    """The default rule (g1 = waves): most of a long step in rmax pieces, then
    every size down to 1 as the work runs out.  The replay lets a wave size its
    piece from a counter value up to a whole round of the other waves old (on
    the GPU the read and the add are back to back), so only the shape is
    checked."""
    waves = 3072
    sizes = [300000] * 20
    cover, stats = schedule(emu, sizes, waves, waves, 0)
    assert np.all(cover == 1)
    wr = wave_rows(sizes)
    assert RMAX * int(stats[RMAX - 1]) >= wr - RMAX * RMAX * 2 * waves  # the bulk in rmax pieces
    assert all(stats[r] > 0 for r in range(RMAX))  # sizes 1 .. rmax all occur


def test_piece_rows_rule(emu):
    """multi_piece_rows itself, through one wave (no interleaving): a piece
    with rem wave-rows left has min(rmax, max(1, rem // g1)) rows."""
    waves, g1 = 1, 10
    sizes = [64 * 100]
    _, stats = schedule(emu, sizes, waves, g1, 0)
    rem, want = 100, np.zeros(19, dtype=np.uint64)
    while rem > 0:
        r = min(RMAX, max(1, rem // g1))
        want[r - 1] += 1
        want[16] += 1
        if r > rem:
            want[17] += 1
        rem -= r
    assert (stats == want).all()


def test_fixed_pieces(emu):
    """g1 = 0 (the fused single-batch launch): every piece has rmax rows."""
    cover, stats = schedule(emu, [100000], 300, 0, 0)
    assert np.all(cover == 1)
    assert stats[16] == stats[RMAX - 1]
    assert stats[RMAX - 1] == -(-((100000 + 63) // 64) // RMAX)


def test_empty(emu):
    cover, stats = schedule(emu, [0, 0], 12, 12, 0)
    assert cover.size == 0 and stats[16] == 0


def test_adaptive_rule(emu):
    """The default sizing (multi_piece_rows_adaptive) through one wave: the
    first piece is one wave-row; then the wave's share of the claimed work is
    all of it, so pieces are min(rmax, rem) rows: 100 = 1 + 16 x 6 + 3."""
    _, stats = schedule(emu, [64 * 100], 1, 1, 0, adaptive=1)
    want = np.zeros(19, dtype=np.uint64)
    want[0] = 1
    want[RMAX - 1] = 16
    want[2] = 1
    want[16] = want[:16].sum()
    assert (stats == want).all()


def test_adaptive_long_step(emu):
    """Bench-like step with the adaptive sizing: the bulk still runs in rmax
    pieces (each wave's first piece is one wave-row)."""
    waves = 3072
    sizes = [300000] * 20
    cover, stats = schedule(emu, sizes, waves, waves, 0, adaptive=1)
    assert np.all(cover == 1)
    assert RMAX * int(stats[RMAX - 1]) >= 0.8 * wave_rows(sizes)


@pytest.mark.parametrize("rows,young_idle", [(1_000_000, True), (4_087_500, False), (300_000 * 20, False)])
@pytest.mark.parametrize("seed", [1, 2])
def test_young_waves(emu, rows, young_idle, seed):
    """The persistent grid's youngest third (waves >= 2048 of 3072) claims
    nothing in a launch under 10 x 3072 wave-rows (1M rows), and works as the
    others do in a larger one.  Every row is still claimed exactly once."""
    waves = 3072
    sizes = [300000] * (rows // 300000) + ([rows % 300000] if rows % 300000 else [])
    cover, stats = schedule(emu, sizes, waves, waves, 0, seed=seed, adaptive=1, young_from=2048)
    assert np.all(cover == 1)
    assert stats[16] == stats[:16].sum()
    if young_idle:
        assert stats[18] == waves - 2048  # every young wave left at once
    else:
        # young waves work; only one whose first read comes late (under 10 x g1
        # wave-rows left by then, in this random interleaving) leaves at once
        assert stats[18] < (waves - 2048) // 10
