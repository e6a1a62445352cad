"""GPU parity: the HIP kernels against the committed golden fixtures (which
were produced by the reference's own oracle, tests/golden/make_golden.py) --
bit-exact t, compare values and match flags."""
import ctypes

import numpy as np
import pytest

import golden_io

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _values(torch, scanner, tweaks):
    x, y = golden_io.tweak_columns(tweaks)
    n = tweaks.shape[0]
    dx = torch.from_numpy(x.view(np.int32)).cuda()
    dy = torch.from_numpy(y.view(np.int32)).cuda()
    dt = torch.zeros((8, n), dtype=torch.int32, device="cuda")
    dv = torch.zeros((1 + scanner.label_count, n), dtype=torch.int64, device="cuda")
    scanner.row_values_device(dx, dy, dt, dv)
    scanner.sync()
    t = dt.cpu().numpy().view(np.uint32)
    tv = [sum(int(t[j, i]) << (32 * j) for j in range(8)) for i in range(n)]
    return tv, dv.cpu().numpy()


def test_stage_kats(torch_cuda):
    from cudasp_amd import Scanner
    for k in golden_io.load("stage_kats.json"):
        labels = [bytes.fromhex(l) for l in k["label_keys"]]
        with Scanner(bytes.fromhex(k["scan_key"]), bytes.fromhex(k["spend_key"]), labels, max_rows=16) as s:
            tw = golden_io.tweak_array([k["tweak"]])
            tv, vals = _values(torch_cuda, s, tw)
            assert tv[0] == int(k["t"], 16), k["height"]
            assert int(vals[0, 0]) == k["v"], k["height"]
            assert [int(v) for v in vals[1:, 0]] == k["label_values"], k["height"]


def test_random_rows_values_and_flags(torch_cuda):
    from cudasp_amd import Scanner
    rr = golden_io.load("random_rows.json")
    rows = rr["rows"]
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    outs, offs, lens = golden_io.csr([r["outputs"] for r in rows])
    spend = bytes.fromhex(rr["spend_key"])
    scan = bytes.fromhex(rr["scan_key"])
    labels = [bytes.fromhex(l) for l in rr["label_keys"]]
    for nl, key in ((len(labels), "match_all_labels"), (1, "match_first_label"), (0, "match_no_labels")):
        with Scanner(scan, spend, labels[:nl], max_rows=len(rows)) as s:
            tv, vals = _values(torch_cuda, s, tw)
            assert [int(v) for v in vals[0]] == [r["v"] for r in rows]
            for j in range(nl):
                assert [int(v) for v in vals[1 + j]] == [r["label_values"][j] for r in rows]
            assert tv == [int(r["t"], 16) for r in rows]
            flags = s.scan_host(tw, outs, offs, lens)
            assert [bool(f) for f in flags] == [r[key] for r in rows], key


def test_device_path_compaction(torch_cuda):
    torch = torch_cuda
    from cudasp_amd import Scanner
    rr = golden_io.load("random_rows.json")
    rows = rr["rows"]
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    outs, offs, lens = golden_io.csr([r["outputs"] for r in rows])
    x, y = golden_io.tweak_columns(tw)
    n = len(rows)
    labels = [bytes.fromhex(l) for l in rr["label_keys"]]
    with Scanner(bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]), labels, max_rows=n) as s:
        dx = torch.from_numpy(x.view(np.int32)).cuda()
        dy = torch.from_numpy(y.view(np.int32)).cuda()
        do = torch.from_numpy(outs).cuda()
        dof = torch.from_numpy(offs.view(np.int32)).cuda()
        dl = torch.from_numpy(lens.view(np.int32)).cuda()
        flags = torch.zeros(n, dtype=torch.uint8, device="cuda")
        rows_out = torch.zeros(n, dtype=torch.int32, device="cuda")
        count = torch.zeros(1, dtype=torch.int32, device="cuda")
        s.scan_device(dx, dy, do, dof, dl, flags, rows_out, count)
        s.sync()
        f = flags.cpu().numpy()
        c = int(count.cpu()[0])
        got = sorted(rows_out.cpu().numpy()[:c].tolist())
        assert [bool(v) for v in f] == [r["match_all_labels"] for r in rows]
        assert got == [i for i, r in enumerate(rows) if r["match_all_labels"]]


def test_legacy_three_phase_abi(torch_cuda):
    """The reference host's call sequence (src/cudasp_extension.cu:308-400)."""
    from cudasp_amd import _native
    lib = _native.load()
    rr = golden_io.load("random_rows.json")
    rows = rr["rows"]
    n = len(rows)
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    outs, offs, lens = golden_io.csr([r["outputs"] for r in rows])
    x, y = golden_io.tweak_columns(tw)
    w = lambda b: np.frombuffer(b, dtype="<u4").copy()
    scan = w(bytes.fromhex(rr["scan_key"]))
    spend = w(bytes.fromhex(rr["spend_key"]))
    labs = [w(bytes.fromhex(l)) for l in rr["label_keys"]]
    lx = np.concatenate([l[:8] for l in labs]); ly = np.concatenate([l[8:] for l in labs])
    sx, sy = spend[:8].copy(), spend[8:].copy()
    px = ctypes.c_void_p(); py = ctypes.c_void_p(); pf = ctypes.c_void_p()
    st = lib.LaunchBatchScan(ctypes.byref(px), ctypes.byref(py), scan.ctypes.data, sx.ctypes.data,
                             sy.ctypes.data, lx.ctypes.data, ly.ctypes.data, len(labs),
                             outs.ctypes.data, offs.ctypes.data, lens.ctypes.data, ctypes.byref(pf), n, outs.size)
    assert st, _native.load().cudasp_last_error()
    ctypes.memmove(px.value, x.ctypes.data, x.nbytes)
    ctypes.memmove(py.value, y.ctypes.data, y.nbytes)
    rc = lib.RunBatchScanKernels(st, px, py, scan.ctypes.data, None, None, None, None, len(labs), pf, n)
    assert rc == 0
    flags = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(pf.value)).copy()
    for p in (px, py, pf):
        lib.FreeBatchScanManaged(p)
    lib.FreeBatchScanState(st)
    assert [bool(v) for v in flags] == [r["match_all_labels"] for r in rows]


def test_default_stream_ordering(torch_cuda):
    """Launches without an explicit stream run on torch's current stream, also
    when that is the default stream (handle 0, passed as CUDASP_STREAM_DEFAULT):
    inputs written by a delayed copy on the default stream are the ones read.
    (Before the fix the kernels ran on the scanner's own stream and raced the
    copy; the bench's planting lost that race when another process shared the GPU.)"""
    torch = torch_cuda
    from cudasp_amd import Scanner
    rr = golden_io.load("random_rows.json")
    rows = rr["rows"][:64]
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    x, y = golden_io.tweak_columns(tw)
    n = len(rows)
    with torch.cuda.stream(torch.cuda.default_stream()):
        assert torch.cuda.current_stream().cuda_stream == 0
        with Scanner(bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]), [], max_rows=n) as s:
            src_x = torch.from_numpy(x.view(np.int32)).cuda()
            src_y = torch.from_numpy(y.view(np.int32)).cuda()
            torch.cuda.synchronize()
            dx = torch.zeros_like(src_x)
            dy = torch.zeros_like(src_y)
            dt = torch.zeros((8, n), dtype=torch.int32, device="cuda")
            dv = torch.zeros((1, n), dtype=torch.int64, device="cuda")
            torch.cuda.synchronize()
            torch.cuda._sleep(50_000_000)  # hold the default stream back
            dx.copy_(src_x)
            dy.copy_(src_y)
            s.row_values_device(dx, dy, dt, dv)
            s.sync()
            assert [int(v) for v in dv.cpu().numpy()[0]] == [r["v"] for r in rows]


def test_exceptional_label_sums_shared_inversion(torch_cuda):
    """Label sums that hit the exceptional cases -- F == L_j (doubling) and
    F == -L_j (infinity, INT64_MIN) -- inside the batched inversion that all
    rows of a thread share (match_labels_rows), next to ordinary labels and
    rows; values bit-exact against the oracle, which follows the reference's
    Python oracle there (scripts/compute_bip352_expected.py:42-46)."""
    import variants as V
    from cudasp_amd import Scanner
    from oracle import oracle
    rr = golden_io.load("random_rows.json")
    rows = rr["rows"][:13]
    scan, spend = bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"])
    F = [V.row(scan, spend, [], bytes.fromhex(r["tweak"]))[0][0][0] for r in rows[:3]]
    labels = [V.point_blob(F[0]), bytes.fromhex(rr["label_keys"][0]), V.point_blob(V.neg(F[1])),
              V.point_blob(F[2])]
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    with Scanner(scan, spend, labels, max_rows=len(rows)) as s:
        _, vals = _values(torch_cuda, s, tw)
    _, want = oracle.scan(scan, spend, labels, tw, want_values=True)
    assert (vals.T == want).all()
    assert want[1, 3] == oracle.LABEL_INFINITY
