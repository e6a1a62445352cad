"""GPU: the 16-label configuration (BASELINE.json configs[4]: 16 label keys,
1..15 outputs per row) against the C oracle, bit for bit.

The reference tests every label in order after the base output and stops at
the first hit (src/cudasp_gpu.cu:153-172); the kernels test all labels of a
thread's rows with one batched inversion (match_labels_rows), so every label
index is exercised here, with and without label negation (32 label entries),
at a few thousand rows for the values and at a full 300000-row batch for the
flags, with planted matches rotating over all 16 label indices."""
import hashlib
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
SEED = 0xC0DA5EED


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def keys():
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    return bench.SCAN_KEY, bench.SPEND_KEY, bench.label_keys(16)


def s0():
    return (int.from_bytes(hashlib.sha256(b"cudasp-synth-v1").digest(), "big") % N).to_bytes(32, "little")


def synth_var(torch, first, n, kmax=15):
    """Synthetic rows with variable-length outputs lists (uniform 1..kmax,
    mean 8 for kmax = 15: the config-5 shape), generated on the device."""
    from cudasp_amd import _native
    lib = _native.load()
    x = torch.empty((8, n), dtype=torch.int32, device="cuda")
    y = torch.empty((8, n), dtype=torch.int32, device="cuda")
    lens = torch.empty((n,), dtype=torch.int32, device="cuda")
    _native.check(lib.cudasp_synth_tweak_columns(0, s0(), first, n, x.data_ptr(), y.data_ptr(), None))
    _native.check(lib.cudasp_synth_output_lengths(SEED, first, n, kmax, lens.data_ptr(), None))
    torch.cuda.synchronize()
    ln = lens.to(torch.int64)
    offs = (torch.cumsum(ln, 0) - ln).to(torch.int32)
    outs = torch.empty((int(ln.sum().item()),), dtype=torch.int64, device="cuda")
    _native.check(lib.cudasp_synth_output_values(SEED, first, n, offs.data_ptr(), lens.data_ptr(), outs.data_ptr(),
                                                 None))
    torch.cuda.synchronize()
    return x, y, outs, offs, lens


def rows_of(x, y):
    xs = x.cpu().numpy().view(np.uint32)
    ys = y.cpu().numpy().view(np.uint32)
    return np.ascontiguousarray(np.concatenate([xs.T, ys.T], axis=1).astype("<u4")).view(np.uint8).reshape(-1, 64)


def plant_rotating(outs, offs, vals, L, every=1000, first=0):
    """Base value on rows g = 0 mod `every`; label j = (g // every) mod L on
    rows g = 1 mod `every` (g = first + row), in the list's last slot.
    vals: [n, 1 + L] host values.  Returns (outs, planted rows, label indices)."""
    o = outs.copy()
    n = len(offs)
    rows, js = [], []
    for i in range(n):
        g = first + i
        if g % every == 0:
            col = 0
        elif g % every == 1:
            col = 1 + (g // every) % L
            js.append(col - 1)
        else:
            continue
        o[offs[i] + 0] = vals[i, col]
        rows.append(i)
    return o, rows, sorted(set(js))


@pytest.mark.parametrize("negation", [False, True])
def test_values_16_labels(torch, keys, negation):
    """3000 rows x (1 + 16) values (1 + 32 with label negation: F + L_j for all
    j, then F - L_j), equal to the oracle's."""
    from cudasp_amd import Scanner
    from oracle import oracle
    scan, spend, labels = keys
    n = 3000
    x, y, _, _, _ = synth_var(torch, 4242, n)
    W = 1 + (32 if negation else 16)
    with Scanner(scan, spend, labels, max_rows=n) as s:
        if negation:
            s.set_options(1, True)
        t = torch.empty((8, n), dtype=torch.int32, device="cuda")
        v = torch.empty((W, n), dtype=torch.int64, device="cuda")
        s.row_values_device(x, y, t, v)
        s.sync()
    _, ov = oracle.scan_ex(scan, spend, labels, rows_of(x, y), label_negation=negation, threads=16,
                           want_values=True)
    gv = v.cpu().numpy().T
    assert ov.shape == (n, 1, W)
    ov = ov[:, 0, :]
    for c in range(W):  # per label index, so a failure names the entry
        assert (gv[:, c] == ov[:, c]).all(), "value column %d differs" % c
    assert (gv == ov).all()


@pytest.mark.parametrize("negation", [False, True])
def test_flags_16_labels_variable_outputs(torch, keys, negation):
    """3000 rows with 1..15 outputs per row and a planted match every 7th
    row rotating over the base value and every label entry: device and host
    flags equal the oracle's."""
    from cudasp_amd import Scanner
    from oracle import oracle
    scan, spend, labels = keys
    n = 3000
    x, y, outs, offs, lens = synth_var(torch, 90210, n)
    rows = rows_of(x, y)
    W = 1 + (32 if negation else 16)
    _, ov = oracle.scan_ex(scan, spend, labels, rows, label_negation=negation, threads=16, want_values=True)
    ov = ov[:, 0, :]
    o = outs.cpu().numpy()
    of = offs.cpu().numpy().view(np.uint32)
    ln = lens.cpu().numpy().view(np.uint32)
    for i in range(0, n, 7):
        col = (i // 7) % W
        o[of[i] + ln[i] - 1] = ov[i, col]  # the list's last slot
    od = torch.from_numpy(o).cuda()
    want, _ = oracle.scan_ex(scan, spend, labels, rows, o, of, ln, label_negation=negation, threads=16)
    assert int(want.sum()) >= (n + 6) // 7
    with Scanner(scan, spend, labels, max_rows=n) as s:
        if negation:
            s.set_options(1, True)
        flags = torch.zeros(n, dtype=torch.uint8, device="cuda")
        s.scan_device(x, y, od, offs, lens, flags)
        s.sync()
        hf = s.scan_host(rows, o, of, ln)
    assert (flags.cpu().numpy() == want).all()
    assert (hf == want).all()


def test_full_batch_16_labels_all_indices(torch, keys):
    """A full 300000-row batch with 16 labels and 1..15 outputs per row: base
    values planted on rows 0 mod 1000, label values on rows 1 mod 1000 with
    the label index cycling over all 16; the flags equal the oracle's over the
    whole batch and the compacted match rows are exactly the planted rows."""
    from cudasp_amd import Scanner
    from oracle import oracle
    scan, spend, labels = keys
    n = 300000
    first = 7_000_000
    x, y, outs, offs, lens = synth_var(torch, first, n)
    idx = torch.tensor([i for i in range(n) if (first + i) % 1000 in (0, 1)], dtype=torch.int64, device="cuda")
    with Scanner(scan, spend, labels, max_rows=n) as s:
        t = torch.empty((8, len(idx)), dtype=torch.int32, device="cuda")
        v = torch.empty((17, len(idx)), dtype=torch.int64, device="cuda")
        s.row_values_device(x.index_select(1, idx).contiguous(), y.index_select(1, idx).contiguous(), t, v)
        s.sync()
        vals = np.zeros((n, 17), dtype=np.int64)
        vals[idx.cpu().numpy()] = v.cpu().numpy().T
        o, planted, js = plant_rotating(outs.cpu().numpy(), offs.cpu().numpy().view(np.uint32), vals, 16,
                                        first=first)
        assert js == list(range(16))
        od = torch.from_numpy(o).cuda()
        flags = torch.zeros(n, dtype=torch.uint8, device="cuda")
        mrows = torch.zeros(n, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
        s.scan_device(x, y, od, offs, lens, flags, mrows, cnt)
        s.sync()
    gf = flags.cpu().numpy()
    c = int(cnt.item())
    assert sorted(mrows[:c].cpu().tolist()) == planted
    assert sorted(np.nonzero(gf)[0].tolist()) == planted
    want, _ = oracle.scan(scan, spend, labels, rows_of(x, y), o, offs.cpu().numpy().view(np.uint32),
                          lens.cpu().numpy().view(np.uint32), threads=16)
    assert (gf == want).all()
