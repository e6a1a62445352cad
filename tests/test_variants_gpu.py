"""GPU: the protocol variants (cudasp_scan_options: output indices k > 0,
label negation, full-x compare) through the HIP
kernels, bit-exact against the C oracle's variant entry points (which
tests/test_variants_cpu.py checks against the pure-Python statement in
tests/variants.py).  The reference implements none of the variants, so their
parity is unpinned against it; with the default options the path is the
reference's (the other GPU tests)."""
import itertools

import numpy as np
import pytest

import golden_io
import variants as V
from oracle import oracle

pytestmark = pytest.mark.gpu

COMBOS = list(itertools.product((1, 3), (False, True), (False, True)))


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _case(nrows=64, nlabels=2):
    rr = golden_io.load("random_rows.json")
    rows = rr["rows"][:nrows]
    return (bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]),
            [bytes.fromhex(l) for l in rr["label_keys"]][:nlabels], rows)


def _outputs(scan, spend, labels, rows, K, neg, full_x):
    """Per row: a decoy plus one planted candidate chosen round-robin over all
    (k, candidate) pairs of the variant, so that every kind of hit occurs;
    every 5th row gets decoys only."""
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    _, v = oracle.scan_ex(scan, spend, labels, tw, output_count=K, label_negation=neg, want_values=True)
    W = v.shape[2]
    lists = []
    for i, r in enumerate(rows):
        q = i % (K * W)
        k, c = divmod(q, W)
        if i % 5 == 4 or (c and v[i, k, c] == V.LABEL_INFINITY):
            lists.append([("decoy", i)])
        else:
            lists.append([("decoy", i), ("hit", k, c)])
    if full_x:
        out = []
        for i, (r, lst) in enumerate(zip(rows, lists)):
            _, _, x = oracle.row_ex(scan, spend, labels, bytes.fromhex(r["tweak"]), K, neg)
            out.append([bytes([i % 256]) * 32 if e[0] == "decoy" else x[e[1]][e[2]] for e in lst])
        offs = np.cumsum([0] + [len(o) for o in out[:-1]]).astype(np.uint32)
        lens = np.array([len(o) for o in out], dtype=np.uint32)
        flat = np.frombuffer(b"".join(b"".join(o) for o in out), dtype=np.uint8).reshape(-1, 32)
        return flat, offs, lens
    vals = [[(0x5EED0000 + i) if e[0] == "decoy" else int(v[i, e[1], e[2]]) for e in lst]
            for i, lst in enumerate(lists)]
    return golden_io.csr(vals)


@pytest.mark.parametrize("K,neg,full_x", COMBOS)
def test_values_and_t(torch_cuda, K, neg, full_x):
    torch = torch_cuda
    from cudasp_amd import Scanner
    scan, spend, labels, rows = _case()
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    n = len(rows)
    x, y = golden_io.tweak_columns(tw)
    with Scanner(scan, spend, labels, max_rows=n) as s:
        s.set_options(K, neg, full_x)
        W = s.value_rows
        dx = torch.from_numpy(x.view(np.int32)).cuda()
        dy = torch.from_numpy(y.view(np.int32)).cuda()
        dt = torch.zeros((8, K * n), dtype=torch.int32, device="cuda")
        dv = torch.zeros((W, K * n), dtype=torch.int64, device="cuda")
        s.row_values_device(dx, dy, dt, dv)
        s.sync()
        got = dv.cpu().numpy().reshape(W, K, n).transpose(2, 1, 0)
        t = dt.cpu().numpy().view(np.uint32).reshape(8, K, n)
    _, want = oracle.scan_ex(scan, spend, labels, tw, output_count=K, label_negation=neg, want_values=True)
    assert (got == want).all()
    for i in (0, 1, n - 1):
        digests, _, _ = oracle.row_ex(scan, spend, labels, bytes.fromhex(rows[i]["tweak"]), K, neg)
        for k in range(K):
            tv = sum(int(t[j, k, i]) << (32 * j) for j in range(8))
            assert tv == int.from_bytes(digests[k], "big")


@pytest.mark.parametrize("K,neg,full_x", COMBOS)
def test_flags_host_and_device(torch_cuda, K, neg, full_x):
    torch = torch_cuda
    from cudasp_amd import Scanner
    scan, spend, labels, rows = _case()
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    n = len(rows)
    outs, offs, lens = _outputs(scan, spend, labels, rows, K, neg, full_x)
    want, _ = oracle.scan_ex(scan, spend, labels, tw, outs, offs, lens, output_count=K, label_negation=neg,
                             full_x=full_x)
    assert 0 < int(want.sum()) < n
    with Scanner(scan, spend, labels, max_rows=n) as s:
        s.set_options(K, neg, full_x)
        assert (s.scan_host(tw, outs, offs, lens) == want).all()
        x, y = golden_io.tweak_columns(tw)
        dx = torch.from_numpy(x.view(np.int32)).cuda()
        dy = torch.from_numpy(y.view(np.int32)).cuda()
        do = torch.from_numpy(np.ascontiguousarray(outs).view(np.int64).copy()).cuda()
        doff = torch.from_numpy(offs.view(np.int32)).cuda()
        dlen = torch.from_numpy(lens.view(np.int32)).cuda()
        flags = torch.zeros(n, dtype=torch.uint8, device="cuda")
        rows_out = torch.zeros(n, dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
        s.scan_device(dx, dy, do, doff, dlen, flags, rows_out, cnt)
        s.sync()
        assert (flags.cpu().numpy() == want).all()
        c = int(cnt.item())
        assert sorted(rows_out[:c].cpu().tolist()) == list(np.flatnonzero(want))
        # the two stage launches with K output indices
        flags.zero_()
        s.stage_shared_secret(dx, dy, n)
        s.stage_match(do, doff, dlen, n, flags)
        s.sync()
        assert (flags.cpu().numpy() == want).all()


def test_options_validation_and_reset(torch_cuda):
    from cudasp_amd import Scanner, _native
    scan, spend, labels, rows = _case(8)
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    outs, offs, lens = golden_io.csr([r["outputs"] for r in rows])
    with Scanner(scan, spend, labels, max_rows=8) as s:
        base = s.scan_host(tw, outs, offs, lens)
        for bad in (0, _native.CUDASP_MAX_OUTPUT_COUNT + 1):
            with pytest.raises(_native.CudaspError):
                s.set_options(bad)
        s.set_options(4, True, False)
        s.set_keys(scan, spend, labels)  # keys rebound under the options
        s.set_options()
        assert (s.scan_host(tw, outs, offs, lens) == base).all()


def test_synthetic_batch_against_oracle(torch_cuda):
    """Compare values of 3000 synthetic rows, K = 2, 2 labels with negation."""
    torch = torch_cuda
    import bench
    from cudasp_amd import Scanner, _native
    n = 3000
    dev = torch.device("cuda", 0)
    tx = torch.empty((8, n), dtype=torch.int32, device=dev)
    ty = torch.empty((8, n), dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()
    lib = _native.load()
    _native.check(lib.cudasp_synth_tweak_columns(0, bench.synth_s0(), 777, n, tx.data_ptr(), ty.data_ptr(),
                                                 _native.stream_arg(st)))
    torch.cuda.synchronize()
    x = tx.cpu().numpy().view(np.uint32)
    y = ty.cpu().numpy().view(np.uint32)
    tw = np.ascontiguousarray(np.concatenate([x.T, y.T], axis=1).astype("<u4")).view(np.uint8).reshape(n, 64)
    labels = bench.label_keys(2)
    _, vals = oracle.scan_ex(bench.SCAN_KEY, bench.SPEND_KEY, labels, tw, output_count=2, label_negation=True,
                             want_values=True, threads=16)
    with Scanner(bench.SCAN_KEY, bench.SPEND_KEY, labels, max_rows=n) as s:
        s.set_options(2, True, False)
        dt = torch.zeros((8, 2 * n), dtype=torch.int32, device=dev)
        dv = torch.zeros((s.value_rows, 2 * n), dtype=torch.int64, device=dev)
        s.row_values_device(tx, ty, dt, dv)
        s.sync()
        got = dv.cpu().numpy().reshape(s.value_rows, 2, n).transpose(2, 1, 0)
    assert (got == vals).all()


def _tf_rows(rows, outs, offs, lens, full_x):
    out = []
    for i, r in enumerate(rows):
        o = [bytes(outs[k]) if full_x else int(outs[k]) for k in range(offs[i], offs[i] + lens[i])]
        out.append((i.to_bytes(32, "big"), 1000 + i, bytes.fromhex(r["tweak"]), o))
    return out


@pytest.mark.parametrize("K,neg,full_x", [(2, True, False), (2, True, True), (3, False, True)])
def test_table_function_variants(torch_cuda, K, neg, full_x):
    """The named parameters through the C++ table-function host (row chunks
    and Arrow columns), against the oracle's flags."""
    import pyarrow as pa
    from cudasp_amd import cudasp_scan, cudasp_scan_arrow
    scan, spend, labels, rows = _case()
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    outs, offs, lens = _outputs(scan, spend, labels, rows, K, neg, full_x)
    want, _ = oracle.scan_ex(scan, spend, labels, tw, outs, offs, lens, output_count=K, label_negation=neg,
                             full_x=full_x)
    expect = sorted(1000 + i for i in np.flatnonzero(want))
    trows = _tf_rows(rows, outs, offs, lens, full_x)
    got = cudasp_scan(trows, scan, spend, labels, batch_size=20, threads=2, chunk_rows=16, output_count=K,
                      label_negation=neg, full_x=full_x)
    assert sorted(h for _, h, _ in got) == expect
    # without the parameters: the reference semantics (a subset of the hits)
    if not full_x:
        base = cudasp_scan(trows, scan, spend, labels, batch_size=20)
        ref, _ = oracle.scan(scan, spend, labels, tw, outs, offs, lens)
        assert sorted(h for _, h, _ in base) == sorted(1000 + i for i in np.flatnonzero(ref))
    vt = pa.binary(32) if full_x else pa.int64()
    for child_type in ([vt, pa.binary()] if full_x else [vt]):
        table = pa.table({
            "txid": pa.array([r[0] for r in trows], pa.binary()),
            "height": pa.array([r[1] for r in trows], pa.int32()),
            "tweak_key": pa.array([r[2] for r in trows], pa.binary(64)),
            "outputs": pa.array([r[3] for r in trows], pa.list_(child_type)),
        })
        res = cudasp_scan_arrow(table, scan, spend, labels, batch_size=20, threads=2, piece_rows=24,
                                output_count=K, label_negation=neg, full_x=full_x)
        assert sorted(res.column("height").to_pylist()) == expect


def test_table_function_full_x_rejects_short_keys(torch_cuda):
    from cudasp_amd import cudasp_scan, _native
    scan, spend, labels, rows = _case(4)
    trows = [(b"t", 1, bytes.fromhex(r["tweak"]), [b"\x01" * 31]) for r in rows]
    with pytest.raises(_native.CudaspError) as e:
        cudasp_scan(trows, scan, spend, labels, full_x=True)
    assert "full_x outputs must be 32-byte x-only keys, got 31 bytes" in str(e.value)
