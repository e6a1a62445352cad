"""GPU: synthetic-table generation and full-batch properties.

* generated tweak rows equal the oracle's (s0 + i) G (sampled indices);
* per-row compare values on a few thousand synthetic rows with labels equal
  the oracle's, bit for bit;
* at the benchmark's batch size (300000 rows): every planted value is found,
  results are deterministic, split-invariant (one batch vs two halves vs the
  host path) and label-order invariant."""
import ctypes
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
SCAN = bytes.fromhex("2c1f0cb94db3946522cc1487256535dd33a1f911946baff817a72880064e690f")
SPEND = bytes.fromhex("36cf8fcd4d4890ab6c1083aeb5b50c260c20acda7839120e3575836f6d85c95ce0d705e31ff9fdcce67a8f3598871c6dfbe6bcde8a51cb7b48b0f95be0ea94de")
LABEL = bytes.fromhex("cd63f9212a2deebde8a71e9ea23f6f958c47c41d2ed74b9617fe6fb554d1524e292fabddbdcbb643eafc328875c46d75a1d697b2b31c42d38aa93f85eab34bc1")


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def s0():
    return (int.from_bytes(hashlib.sha256(b"cudasp-synth-v1").digest(), "big") % N).to_bytes(32, "little")


def synth(torch, first, n):
    from cudasp_amd import _native
    lib = _native.load()
    x = torch.empty((8, n), dtype=torch.int32, device="cuda")
    y = torch.empty((8, n), dtype=torch.int32, device="cuda")
    outs = torch.empty((2 * n,), dtype=torch.int64, device="cuda")
    offs = torch.empty((n,), dtype=torch.int32, device="cuda")
    lens = torch.empty((n,), dtype=torch.int32, device="cuda")
    _native.check(lib.cudasp_synth_tweak_columns(0, s0(), first, n, x.data_ptr(), y.data_ptr(), None))
    _native.check(lib.cudasp_synth_outputs(0xC0DA5EED, first, n, 2, outs.data_ptr(), offs.data_ptr(),
                                           lens.data_ptr(), None))
    torch.cuda.synchronize()
    return x, y, outs, offs, lens


def rows_of(x, y):
    xs = x.cpu().numpy().view(np.uint32)
    ys = y.cpu().numpy().view(np.uint32)
    return np.ascontiguousarray(np.concatenate([xs.T, ys.T], axis=1).astype("<u4")).view(np.uint8).reshape(-1, 64)


def test_synth_tweaks_match_oracle(torch):
    from oracle import oracle
    first = 10**9
    x, y, _, _, _ = synth(torch, first, 4096)
    rows = rows_of(x, y)
    for i in (0, 1, 2, 1000, 4095):
        assert rows[i].tobytes() == oracle.synth_tweak(s0(), first + i)


def test_values_match_oracle_with_labels(torch):
    from cudasp_amd import Scanner
    from oracle import oracle
    n = 3000
    x, y, outs, offs, lens = synth(torch, 777, n)
    labels = [LABEL, SPEND]
    with Scanner(SCAN, SPEND, labels, max_rows=n) as s:
        t = torch.empty((8, n), dtype=torch.int32, device="cuda")
        v = torch.empty((3, n), dtype=torch.int64, device="cuda")
        s.row_values_device(x, y, t, v)
        s.sync()
    _, ov = oracle.scan(SCAN, SPEND, labels, rows_of(x, y), threads=16, want_values=True)
    assert (v.cpu().numpy().T == ov).all()


@pytest.mark.parametrize("rows_a,rows_b", [("1", "2"), ("2", "6"), ("4", "6"), ("4", "2"), (None, None)])
def test_rows_per_thread_variants(torch, monkeypatch, rows_a, rows_b):
    """Stage A at 1, 2 or 4 rows per thread and stage B at 2 or 6 (4 / 6 by
    default; launches too small to fill the GPU take fewer, rows_a_for /
    rows_b_for in scan_kernels.hip; forced here with CUDASP_ROWS_A_FORCE /
    CUDASP_ROWS_B_FORCE): 3001 synthetic rows (not a multiple of 2, 4 or 6)
    with two labels, values and flags equal to the oracle's."""
    from cudasp_amd import Scanner
    from oracle import oracle
    for var, val in (("CUDASP_ROWS_A_FORCE", rows_a), ("CUDASP_ROWS_B_FORCE", rows_b)):
        if val:
            monkeypatch.setenv(var, val)
        else:
            monkeypatch.delenv(var, raising=False)
    n = 3001
    labels = [LABEL, SPEND]
    x, y, outs, offs, lens = synth(torch, 555, n)
    rows = rows_of(x, y)
    _, ov = oracle.scan(SCAN, SPEND, labels, rows, threads=16, want_values=True)
    # plant every 7th row's second-label value as its first output
    o = outs.cpu().numpy().reshape(n, 2)
    o[::7, 0] = ov[::7, 2]
    outs.copy_(torch.from_numpy(o.reshape(-1)))
    with Scanner(SCAN, SPEND, labels, max_rows=n) as s:
        t = torch.empty((8, n), dtype=torch.int32, device="cuda")
        v = torch.empty((3, n), dtype=torch.int64, device="cuda")
        s.row_values_device(x, y, t, v)
        flags = torch.zeros(n, dtype=torch.uint8, device="cuda")
        s.scan_device(x, y, outs, offs, lens, flags)
        s.sync()
    assert (v.cpu().numpy().T == ov).all()
    want, _ = oracle.scan(SCAN, SPEND, labels, rows, o.reshape(-1), offs.cpu().numpy().view(np.uint32),
                          lens.cpu().numpy().view(np.uint32), threads=16)
    assert int(want.sum()) >= n // 7
    assert (flags.cpu().numpy() == want).all()


def test_rows_per_thread_large_launch(torch, monkeypatch):
    """200k rows at 1, 2 and 4 rows per thread give identical t: the 1- and
    2-row launches need more scratch slots than the scanner holds, so their
    grids are capped and the grid-stride loop takes the remaining rows.  Stage
    B at 6 and 2 rows per thread gives identical values."""
    from cudasp_amd import Scanner
    n = 200000
    x, y, _, _, _ = synth(torch, 31337, n)
    ts = []
    for r in ("4", "2", "1"):
        monkeypatch.setenv("CUDASP_ROWS_A_FORCE", r)
        with Scanner(SCAN, SPEND, [], max_rows=n) as s:
            t = torch.zeros((8, n), dtype=torch.int32, device="cuda")
            s.stage_shared_secret(x, y, n, t_out=t)
            s.sync()
        ts.append(t.cpu())
    assert torch.equal(ts[0], ts[1]) and torch.equal(ts[0], ts[2])
    # stage B at 6 and 2 rows per thread on the same t: identical values
    vs = []
    for r in ("6", "2"):
        monkeypatch.setenv("CUDASP_ROWS_B_FORCE", r)
        with Scanner(SCAN, SPEND, [LABEL], max_rows=n) as s:
            t = torch.zeros((8, n), dtype=torch.int32, device="cuda")
            v = torch.zeros((2, n), dtype=torch.int64, device="cuda")
            s.row_values_device(x, y, t, v)
            s.sync()
        vs.append(v.cpu())
    assert torch.equal(vs[0], vs[1])


def _plant(torch, x, y, outs, labels, every=1000):
    from cudasp_amd import Scanner
    n = x.shape[1]
    idx = torch.arange(0, n, every, device="cuda")
    with Scanner(SCAN, SPEND, labels, max_rows=len(idx)) as s:
        t = torch.empty((8, len(idx)), dtype=torch.int32, device="cuda")
        v = torch.empty((1 + len(labels), len(idx)), dtype=torch.int64, device="cuda")
        s.row_values_device(x.index_select(1, idx).contiguous(), y.index_select(1, idx).contiguous(), t, v)
        s.sync()
    outs.index_copy_(0, idx * 2, v[-1])  # plant the last label's (or base) value
    return idx


def test_full_batch_properties(torch):
    from cudasp_amd import Scanner
    n = 300000
    x, y, outs, offs, lens = synth(torch, 0, n)
    labels = [LABEL, SPEND]
    planted = _plant(torch, x, y, outs, labels)
    flags = torch.zeros(n, dtype=torch.uint8, device="cuda")
    rows = torch.zeros(n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    with Scanner(SCAN, SPEND, labels, max_rows=n) as s:
        s.scan_device(x, y, outs, offs, lens, flags, rows, cnt)
        s.sync()
        f1 = flags.cpu().numpy().copy()
        c = int(cnt.item())
        assert set(np.nonzero(f1)[0].tolist()) == set(planted.cpu().tolist())
        assert sorted(rows[:c].cpu().tolist()) == planted.cpu().tolist()
        # deterministic
        flags.zero_()
        s.scan_device(x, y, outs, offs, lens, flags)
        s.sync()
        assert (flags.cpu().numpy() == f1).all()
        # split invariance: two halves as separate batches
        h = n // 2
        parts = []
        for a, b in ((0, h), (h, n)):
            xs, ys = x[:, a:b].contiguous(), y[:, a:b].contiguous()
            o = outs[2 * a:2 * b].contiguous()
            of = (offs[a:b] - 2 * a).contiguous()
            fl = torch.zeros(b - a, dtype=torch.uint8, device="cuda")
            s.scan_device(xs, ys, o, of, lens[a:b].contiguous(), fl)
            s.sync()
            parts.append(fl.cpu().numpy())
        assert (np.concatenate(parts) == f1).all()
        # host path on the same rows
        hf = s.scan_host(rows_of(x, y), outs.cpu().numpy(), offs.cpu().numpy().view(np.uint32),
                         lens.cpu().numpy().view(np.uint32))
        assert (hf == f1).all()
    # label order does not change the flags
    with Scanner(SCAN, SPEND, labels[::-1], max_rows=n) as s2:
        flags.zero_()
        s2.scan_device(x, y, outs, offs, lens, flags)
        s2.sync()
        assert (flags.cpu().numpy() == f1).all()


def test_max_batch_size(torch):
    """The reference's largest batch_size (10,000,000 rows, bind limit
    src/cudasp_extension.cu:483-486) in one launch: the stage-A scratch is capped
    below 4 GiB, so the grid is capped and threads take several row groups.
    Every planted value is found, exactly, and the flags equal those of the
    same rows scanned as 300000-row batches."""
    from cudasp_amd import Scanner
    n = 10_000_000
    x, y, outs, offs, lens = synth(torch, 5_000_000, n)
    planted = _plant(torch, x, y, outs, [], every=10007)
    flags = torch.zeros(n, dtype=torch.uint8, device="cuda")
    rows = torch.zeros(n, dtype=torch.int32, device="cuda")
    cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
    with Scanner(SCAN, SPEND, [], max_rows=n) as s:
        s.scan_device(x, y, outs, offs, lens, flags, rows, cnt)
        s.sync()
        c = int(cnt.item())
        assert c == len(planted)
        assert sorted(rows[:c].cpu().tolist()) == planted.cpu().tolist()
        f1 = flags.cpu().numpy()
    step = 300000
    parts = []
    with Scanner(SCAN, SPEND, [], max_rows=step) as s:
        for a in range(0, n, step):
            b = min(n, a + step)
            fl = torch.zeros(b - a, dtype=torch.uint8, device="cuda")
            s.scan_device(x[:, a:b].contiguous(), y[:, a:b].contiguous(), outs[2 * a:2 * b].contiguous(),
                          (offs[a:b] - 2 * a).contiguous(), lens[a:b].contiguous(), fl)
            parts.append(fl)
        s.sync()
    assert (torch.cat(parts).cpu().numpy() == f1).all()


def test_layout_probe_runs(torch):
    """The measurement-only layout probe (cudasp_layout_probe) touches every
    row: it writes a 0/1 flag for each, including a partial last row group."""
    from cudasp_amd import _native
    n = 300001
    x, y, outs, offs, lens = synth(torch, 0, n)
    flags = torch.full((n,), 7, dtype=torch.uint8, device="cuda")
    lib = _native.load()
    _native.check(lib.cudasp_layout_probe(x.data_ptr(), y.data_ptr(), n, outs.data_ptr(), offs.data_ptr(),
                                          lens.data_ptr(), flags.data_ptr(), None))
    torch.cuda.synchronize()
    assert int((flags > 1).sum().item()) == 0
