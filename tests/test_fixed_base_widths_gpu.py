"""GPU: stage B's fixed-base window widths give identical results.

The width of the t*G table is a per-scanner runtime choice
(cudasp_scanner_set_fixed_base_bits): 22-bit windows (1.5 GiB HBM table),
26-bit (21.5 GB HBM, the default on MI355X) and 7-bit staged into LDS
(k_match_lds).  All must produce the oracle's compare values and flags
bit for bit, with labels and at a launch large enough to use the 6-rows-per-
thread shapes."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def test_widths_equal_oracle(torch):
    from test_labels16_gpu import rows_of, synth_var
    from cudasp_amd import Scanner
    from oracle import oracle
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    labels = bench.label_keys(3)
    n = 5003
    x, y, outs, offs, lens = synth_var(torch, 123456, n)
    rows = rows_of(x, y)
    _, ov = oracle.scan(bench.SCAN_KEY, bench.SPEND_KEY, labels, rows, threads=16, want_values=True)
    o = outs.cpu().numpy()
    of = offs.cpu().numpy().view(np.uint32)
    for i in range(0, n, 5):
        o[of[i]] = ov[i, (i // 5) % 4]
    od = torch.from_numpy(o).cuda()
    want, _ = oracle.scan(bench.SCAN_KEY, bench.SPEND_KEY, labels, rows, o, of, lens.cpu().numpy().view(np.uint32),
                          threads=16)
    with Scanner(bench.SCAN_KEY, bench.SPEND_KEY, labels, max_rows=n) as s:
        assert s.fixed_base_bits in (22, 26)
        for bits in (22, 26, 7):
            s.set_fixed_base_bits(bits)
            assert s.fixed_base_bits == bits
            t = torch.empty((8, n), dtype=torch.int32, device="cuda")
            v = torch.empty((4, n), dtype=torch.int64, device="cuda")
            s.row_values_device(x, y, t, v)
            flags = torch.zeros(n, dtype=torch.uint8, device="cuda")
            s.scan_device(x, y, od, offs, lens, flags)
            s.sync()
            assert (v.cpu().numpy().T == ov).all(), bits
            assert (flags.cpu().numpy() == want).all(), bits
        with pytest.raises(Exception):
            s.set_fixed_base_bits(24)


def test_lds_width_full_batch(torch):
    """A full 300000-row batch through the LDS-staged stage B equals the
    default width's flags and compacted rows (both 2- and 6-row shapes)."""
    from test_gpu_synth import _plant, synth
    from cudasp_amd import Scanner
    import bench
    n = 300000
    x, y, outs, offs, lens = synth(torch, 42, n)
    planted = _plant(torch, x, y, outs, [])
    res = []
    with Scanner(bench.SCAN_KEY, bench.SPEND_KEY, [], max_rows=n) as s:
        for bits, rb in ((22, 0), (7, 0), (7, 6), (7, 2)):
            s.set_fixed_base_bits(bits)
            s.set_rows_per_thread(0, rb)
            flags = torch.zeros(n, dtype=torch.uint8, device="cuda")
            rows = torch.zeros(n, dtype=torch.int32, device="cuda")
            cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
            s.scan_device(x, y, outs, offs, lens, flags, rows, cnt)
            s.sync()
            c = int(cnt.item())
            assert sorted(rows[:c].cpu().tolist()) == planted.cpu().tolist()
            res.append(flags.cpu().numpy())
    for r in res[1:]:
        assert (r == res[0]).all()


@pytest.mark.parametrize("max_rows", [300, 2000])
def test_lds_width_small_scanner(torch, max_rows):
    """A scanner too small for one 768-thread LDS workgroup at 6 rows per
    thread (its label scratch holds 256 / 512 slots at max_rows 300 / 2000;
    one workgroup needs 768): the launch takes 2 rows per thread, whose slots are
    smaller, instead of writing past the scratch.  Flags equal the HBM
    width's; also with 6 rows per thread forced."""
    from test_gpu_synth import _plant, synth
    from cudasp_amd import Scanner
    import bench
    n = max_rows
    x, y, outs, offs, lens = synth(torch, 9001, n)
    planted = _plant(torch, x, y, outs, [], every=50)
    res = []
    with Scanner(bench.SCAN_KEY, bench.SPEND_KEY, [bench.TEST_LABEL], max_rows=n) as s:
        for bits, rb in ((22, 0), (7, 6), (7, 0)):
            s.set_fixed_base_bits(bits)
            s.set_rows_per_thread(0, rb)
            flags = torch.zeros(n, dtype=torch.uint8, device="cuda")
            s.scan_device(x, y, outs, offs, lens, flags)
            s.sync()
            res.append(flags.cpu().numpy())
    assert sorted(np.nonzero(res[0])[0].tolist()) == planted.cpu().tolist()
    for r in res[1:]:
        assert (r == res[0]).all()


def test_spend_fold_equals_separate_addition(torch):
    """The spend key folded into the top window (cudasp_scanner_set_spend_fold,
    on by default for an on-curve key at an HBM width): compare values and
    flags through the stage kernels, the fused single-batch kernel and the
    multi-batch kernel equal the oracle's with the fold and without it, at 22
    and 26 bits; an off-curve spend key (the SQL test's "wrong keys" query
    passes one) is never folded."""
    from test_labels16_gpu import rows_of, synth_var
    from cudasp_amd import Scanner
    from oracle import oracle
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    labels = bench.label_keys(2)
    n = 4099
    x, y, outs, offs, lens = synth_var(torch, 987654, n)
    rows = rows_of(x, y)
    _, ov = oracle.scan(bench.SCAN_KEY, bench.SPEND_KEY, labels, rows, threads=16, want_values=True)
    o = outs.cpu().numpy()
    of = offs.cpu().numpy().view(np.uint32)
    for i in range(0, n, 3):
        o[of[i]] = ov[i, (i // 3) % 3]
    od = torch.from_numpy(o).cuda()
    want, _ = oracle.scan(bench.SCAN_KEY, bench.SPEND_KEY, labels, rows, o, of, lens.cpu().numpy().view(np.uint32),
                          threads=16)
    with Scanner(bench.SCAN_KEY, bench.SPEND_KEY, labels, max_rows=n) as s:
        for bits in (22, 26):
            s.set_fixed_base_bits(bits)
            for fold in (True, False):
                s.set_spend_fold(fold)
                assert s.spend_folded == fold, (bits, fold)
                t = torch.empty((8, n), dtype=torch.int32, device="cuda")
                v = torch.empty((3, n), dtype=torch.int64, device="cuda")
                s.row_values_device(x, y, t, v)
                f1 = torch.zeros(n, dtype=torch.uint8, device="cuda")
                s.scan_device(x, y, od, offs, lens, f1)
                f2 = torch.zeros(n, dtype=torch.uint8, device="cuda")
                s.scan_device_batches([dict(tweak_x=x, tweak_y=y, outputs=od, offsets=offs, lengths=lens, flags=f2)])
                s.sync()
                assert (v.cpu().numpy().T == ov).all(), (bits, fold)
                assert (f1.cpu().numpy() == want).all(), (bits, fold)
                assert (f2.cpu().numpy() == want).all(), (bits, fold)
        s.set_spend_fold(True)
        off_curve = bench.SPEND_KEY[:32] + bytes([bench.SPEND_KEY[32] ^ 1]) + bench.SPEND_KEY[33:]
        s.set_keys(bench.SCAN_KEY, off_curve, labels)
        assert not s.spend_folded
        s.set_keys(bench.SCAN_KEY, bench.SPEND_KEY, labels)
        assert s.spend_folded


@pytest.mark.parametrize("bits,stride", [(22, 1), (26, 7), (7, 1)])
def test_table_built_in_runs_equals_entries_built_alone(torch, bits, stride):
    """The fixed-base tables are built in runs of consecutive odd multiples
    with one batched inversion per run (k_fb_build_runs); every stride-th
    entry (all of them at 22 and 7 bits; at 26 bits stride 7, which visits
    every position of a 128-entry run) equals the entry computed on its own
    by double-and-add and its own inversion (k_fb_check)."""
    import ctypes
    from cudasp_amd import _native
    lib = _native.load()
    checked, bad = ctypes.c_uint64(), ctypes.c_uint64()
    _native.check(lib.cudasp_debug_fb_check(0, bits, stride, ctypes.byref(checked), ctypes.byref(bad)))
    windows, entries = (256 + bits - 1) // bits, 1 << (bits - 1)
    assert checked.value == -(-windows * entries // stride)
    assert bad.value == 0, (bits, bad.value)
    secs = ctypes.c_double(-1)
    _native.check(lib.cudasp_fixed_base_prepare(0, bits, ctypes.byref(secs)))
    assert secs.value == 0  # already built: nothing to do


@pytest.mark.parametrize("bits,stride", [(22, 1), (26, 3)])
def test_fold_table_built_in_runs_equals_entries_built_alone(torch, bits, stride):
    """The spend-key fold table (top window + B and - B) is built with one
    batched inversion per run of 16 entries (k_fb_fold); every stride-th
    entry's two halves (all of them at 22 bits; at 26 bits stride 3, which
    visits every position of a run) equal fb_fold_entry's, one inversion per
    entry (k_fold_check)."""
    import ctypes
    from cudasp_amd import _native
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    lib = _native.load()
    checked, bad = ctypes.c_uint64(), ctypes.c_uint64()
    _native.check(lib.cudasp_debug_fold_check(0, bits, bench.SPEND_KEY, stride, ctypes.byref(checked),
                                              ctypes.byref(bad)))
    top = 1 << (255 - bits * ((256 + bits - 1) // bits - 1))
    assert checked.value == -(-top // stride)
    assert bad.value == 0, (bits, bad.value)
