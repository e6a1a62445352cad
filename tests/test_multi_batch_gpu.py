"""GPU: cudasp_scan_device_batches (several resident batches, one persistent
kernel for both stages) gives exactly the per-batch results of
cudasp_scan_device: flags, match counts and match-row sets per batch, for
ragged batch sizes (empty, 1 row, partial wave-rows, full 300k batches), with
0, 2 and 16 labels, variable outputs per row, every guided-scheduling regime
(6, 2 or 1 rows per thread throughout), and the per-batch fallback of the
protocol variants; and its flags equal the C oracle's."""
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


def labels16():
    import bench
    return bench.label_keys(16)


def make_batch(torch, first, n, kmax=0):
    """Synthetic batch: tweak columns, outputs CSR (2 per row, or 1..kmax)."""
    from cudasp_amd import _native
    lib = _native.load()
    m = max(n, 1)
    x = torch.empty((8, m), dtype=torch.int32, device="cuda")
    y = torch.empty((8, m), dtype=torch.int32, device="cuda")
    offs = torch.zeros((m,), dtype=torch.int32, device="cuda")
    lens = torch.zeros((m,), dtype=torch.int32, device="cuda")
    cap = kmax if kmax else 2
    outs = torch.zeros((m * cap,), dtype=torch.int64, device="cuda")
    if n:
        _native.check(lib.cudasp_synth_tweak_columns(0, s0(), first, n, x.data_ptr(), y.data_ptr(), None))
        if kmax:
            _native.check(lib.cudasp_synth_output_lengths(0xC0DA5EED, first, n, kmax, lens.data_ptr(), None))
            torch.cuda.synchronize()
            ln = lens[:n].to(torch.int64)
            offs[:n] = (torch.cumsum(ln, 0) - ln).to(torch.int32)
            _native.check(lib.cudasp_synth_output_values(0xC0DA5EED, first, n, offs.data_ptr(), lens.data_ptr(),
                                                         outs.data_ptr(), None))
        else:
            _native.check(lib.cudasp_synth_outputs(0xC0DA5EED, first, n, 2, outs.data_ptr(), offs.data_ptr(),
                                                   lens.data_ptr(), None))
    torch.cuda.synchronize()
    return dict(tweak_x=x[:, :n].contiguous() if n else x, tweak_y=y[:, :n].contiguous() if n else y,
                outputs=outs, offsets=offs, lengths=lens, n=n)


def plant(torch, batches, labels, every=97):
    """Plant base / label values (from the per-row values path) as each
    planted row's first output; returns the planted row lists."""
    from cudasp_amd import Scanner
    L = len(labels)
    for bi, b in enumerate(batches):
        n = b["n"]
        if n == 0:
            continue
        idx = list(range(bi % every, n, every))
        if not idx:
            continue
        it = torch.tensor(idx, dtype=torch.int64, device="cuda")
        with Scanner(SCAN, SPEND, labels, max_rows=len(idx)) as s:
            t = torch.empty((8, len(idx)), dtype=torch.int32, device="cuda")
            v = torch.empty((1 + L, len(idx)), dtype=torch.int64, device="cuda")
            s.row_values_device(b["tweak_x"].index_select(1, it).contiguous(),
                                b["tweak_y"].index_select(1, it).contiguous(), t, v)
            s.sync()
        col = torch.tensor([(i // every) % (1 + L) for i in idx], dtype=torch.int64, device="cuda")
        vals = v[col, torch.arange(len(idx), device="cuda")]
        pos = b["offsets"][:n].index_select(0, it).to(torch.int64)
        b["outputs"].index_copy_(0, pos, vals)
    torch.cuda.synchronize()


def run_per_batch(torch, batches, labels, **opts):
    from cudasp_amd import Scanner
    cap = max(1, max(b["n"] for b in batches))
    res = []
    with Scanner(SCAN, SPEND, labels, max_rows=cap) as s:
        if opts:
            s.set_options(**opts)
        for b in batches:
            n = b["n"]
            fl = torch.zeros(max(n, 1), dtype=torch.uint8, device="cuda")
            rows = torch.zeros(max(n, 1), dtype=torch.int32, device="cuda")
            cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
            if n:
                s.scan_device(b["tweak_x"], b["tweak_y"], b["outputs"], b["offsets"], b["lengths"], fl[:n], rows, cnt)
            res.append((fl, rows, cnt))
        s.sync()
    return [(fl[:b["n"]].cpu().numpy(), sorted(rows[:int(cnt.item())].cpu().tolist()), int(cnt.item()))
            for (fl, rows, cnt), b in zip(res, batches)]


def run_multi(torch, batches, labels, max_rows=300000, **opts):
    from cudasp_amd import Scanner
    outs = []
    descs = []
    for b in batches:
        n = b["n"]
        fl = torch.full((max(n, 1),), 7, dtype=torch.uint8, device="cuda")
        rows = torch.zeros(max(n, 1), dtype=torch.int32, device="cuda")
        cnt = torch.zeros(1, dtype=torch.int32, device="cuda")
        outs.append((fl, rows, cnt))
        descs.append(dict(tweak_x=b["tweak_x"], tweak_y=b["tweak_y"], outputs=b["outputs"], offsets=b["offsets"],
                          lengths=b["lengths"], flags=fl[:n], match_rows=rows, match_count=cnt))
    with Scanner(SCAN, SPEND, labels, max_rows=max_rows) as s:
        if opts:
            s.set_options(**opts)
        s.scan_device_batches(descs)
        s.sync()
    return [(fl[:b["n"]].cpu().numpy(), sorted(rows[:int(cnt.item())].cpu().tolist()), int(cnt.item()))
            for (fl, rows, cnt), b in zip(outs, batches)]


def same(a, b):
    assert len(a) == len(b)
    for i, ((fa, ra, ca), (fb, rb, cb)) in enumerate(zip(a, b)):
        assert (fa == fb).all(), "batch %d flags" % i
        assert ca == cb and ra == rb, "batch %d matches" % i


SIZES = [3001, 64, 1, 0, 129, 70000, 65, 2047]


@pytest.mark.parametrize("nlabels", [0, 2])
def test_multi_equals_per_batch(torch, nlabels):
    labels = [LABEL, SPEND][:nlabels]
    batches = [make_batch(torch, 1000 + 100000 * i, n) for i, n in enumerate(SIZES)]
    plant(torch, batches, labels)
    want = run_per_batch(torch, batches, labels)
    assert sum(c for _, _, c in want) > 0
    same(run_multi(torch, batches, labels), want)


def test_multi_matches_oracle(torch):
    """Flags of the persistent path against the C oracle on a ragged set."""
    from oracle import oracle
    labels = [LABEL]
    batches = [make_batch(torch, 7 + 50000 * i, n) for i, n in enumerate([700, 1, 64, 300])]
    plant(torch, batches, labels, every=13)
    got = run_multi(torch, batches, labels)
    for b, (fl, rows, cnt) in zip(batches, got):
        n = b["n"]
        xs = b["tweak_x"].cpu().numpy().view(np.uint32)
        ys = b["tweak_y"].cpu().numpy().view(np.uint32)
        tw = np.ascontiguousarray(np.concatenate([xs.T, ys.T], axis=1).astype("<u4")).view(np.uint8).reshape(n, 64)
        want, _ = oracle.scan(SCAN, SPEND, labels, tw, b["outputs"].cpu().numpy(),
                              b["offsets"][:n].cpu().numpy().view(np.uint32),
                              b["lengths"][:n].cpu().numpy().view(np.uint32), threads=16)
        assert (fl == want).all()
        assert cnt == int(want.sum()) and rows == sorted(np.nonzero(want)[0].tolist())


def test_multi_16_labels_variable_outputs(torch):
    """Config-5 shape: 16 labels, 1..15 outputs per row, planted values over
    every label index."""
    labels = labels16()
    batches = [make_batch(torch, 3 + 40000 * i, n, kmax=15) for i, n in enumerate([5000, 333, 4096])]
    plant(torch, batches, labels, every=7)
    want = run_per_batch(torch, batches, labels)
    assert sum(c for _, _, c in want) > 1000
    same(run_multi(torch, batches, labels), want)


@pytest.mark.parametrize("g1,g2,rows", [("0", "0", None), ("100000", "100000", None), ("0", "0", "2"),
                                         ("100", "0", None), ("150", "400", None)])
def test_multi_guided_regimes(torch, monkeypatch, g1, g2, rows):
    """Every chunk size regime of the guided schedule (CUDASP_MULTI_G1/G2,
    hundredths of the grid's waves; CUDASP_MULTI_ROWS): all 6 (MULTI_RMAX),
    all 1, all 2 rows per thread, the default rule (every size from 6 down to
    1) and a leading 6-row phase, give the per-batch results."""
    monkeypatch.setenv("CUDASP_MULTI_G1", g1)
    monkeypatch.setenv("CUDASP_MULTI_G2", g2)
    if rows:
        monkeypatch.setenv("CUDASP_MULTI_ROWS", rows)
    labels = [LABEL]
    batches = [make_batch(torch, 555 + 20000 * i, n) for i, n in enumerate([9000, 17, 4000])]
    plant(torch, batches, labels)
    same(run_multi(torch, batches, labels), run_per_batch(torch, batches, labels))


def test_multi_full_batches(torch):
    """Five full 300k-row batches (a rank's resident share), 0 labels:
    planted matches found exactly, results equal to the per-batch path."""
    batches = [make_batch(torch, 300000 * i, 300000) for i in range(5)]
    plant(torch, batches, [], every=1000)
    want = run_per_batch(torch, batches, [])
    got = run_multi(torch, batches, [])
    same(got, want)
    assert [c for _, _, c in got] == [300, 300, 300, 300, 300]


def test_multi_variants_fall_back(torch):
    """Protocol variants take the per-batch path inside the same call: the
    results equal cudasp_scan_device's with the same options."""
    labels = [LABEL]
    batches = [make_batch(torch, 11 + 9000 * i, n) for i, n in enumerate([2000, 70])]
    plant(torch, batches, labels)
    opts = dict(output_count=2, label_negation=True)
    same(run_multi(torch, batches, labels, max_rows=2000, **opts), run_per_batch(torch, batches, labels, **opts))


def test_fused_single_batch_equals_two_kernels(torch, monkeypatch):
    """cudasp_scan_device runs both stages in one k_scan_multi launch by
    default; CUDASP_FUSED_SINGLE=0 selects the two stage kernels.  Same flags
    and match sets on ragged batches with labels."""
    labels = [LABEL, SPEND]
    batches = [make_batch(torch, 77 + 30000 * i, n) for i, n in enumerate([3001, 1, 300, 20000])]
    plant(torch, batches, labels)
    fused = run_per_batch(torch, batches, labels)
    monkeypatch.setenv("CUDASP_FUSED_SINGLE", "0")
    same(run_per_batch(torch, batches, labels), fused)
    assert sum(c for _, _, c in fused) > 0


def test_multi_100_labels(torch, monkeypatch):
    """100 label keys (6 x 100 prefix products per thread in the label
    scratch): the multi-batch path equals the two stage kernels, and planted
    values of label indices 0..99 are found."""
    import bench
    labels = bench.label_keys(100)
    batches = [make_batch(torch, 900 + 5000 * i, n) for i, n in enumerate([1500, 700])]
    plant(torch, batches, labels, every=3)
    got = run_multi(torch, batches, labels)
    monkeypatch.setenv("CUDASP_FUSED_SINGLE", "0")
    same(got, run_per_batch(torch, batches, labels))
    assert sum(c for _, _, c in got) == len(range(0, 1500, 3)) + len(range(1, 700, 3))


@pytest.mark.parametrize("g1,g2", [("0", "0"), ("100", "0"), ("100000", "100000")])
def test_multi_pipelined_equals_unpipelined(torch, monkeypatch, g1, g2):
    """The default schedule finishes a piece's stage B one iteration later,
    with its Z inversion merged into the next piece's stage-A inversion
    (CUDASP_MULTI_PIPE=0: two inversions per piece).  Same flags and match
    sets as that schedule and as the two stage kernels, in every chunk-size
    regime, with labels."""
    monkeypatch.setenv("CUDASP_MULTI_G1", g1)
    monkeypatch.setenv("CUDASP_MULTI_G2", g2)
    labels = [LABEL, SPEND]
    batches = [make_batch(torch, 4242 + 25000 * i, n) for i, n in enumerate([5000, 1, 65, 12000, 640])]
    plant(torch, batches, labels)
    piped = run_multi(torch, batches, labels)
    assert sum(c for _, _, c in piped) > 0
    monkeypatch.setenv("CUDASP_MULTI_PIPE", "0")
    same(run_multi(torch, batches, labels), piped)
    monkeypatch.setenv("CUDASP_FUSED_SINGLE", "0")
    same(run_per_batch(torch, batches, labels), piped)


def test_many_small_batches(torch, monkeypatch):
    """600 ragged batches (0..200 rows) cut from one table: more descriptors
    than the scanner's first staging area holds (it grows), then a second
    call on the same scanner with the batches in reverse order (the staging
    ring).  Flags and match-row sets equal the two stage kernels' over the
    whole table."""
    from cudasp_amd import Scanner
    rng = np.random.default_rng(600)
    sizes = [int(x) for x in rng.integers(0, 201, 600)]
    sizes[:3] = [0, 1, 64]
    total = sum(sizes)
    labels = [LABEL]
    big = make_batch(torch, 123457, total)
    plant(torch, [big], labels, every=11)
    monkeypatch.setenv("CUDASP_FUSED_SINGLE", "0")
    want = run_per_batch(torch, [big], labels)[0][0]
    monkeypatch.delenv("CUDASP_FUSED_SINGLE")
    cuts = np.concatenate([[0], np.cumsum(sizes)])
    subs = []
    for i, n in enumerate(sizes):
        a = int(cuts[i])
        subs.append(dict(tweak_x=big["tweak_x"][:, a:a + n].contiguous(), tweak_y=big["tweak_y"][:, a:a + n].contiguous(),
                         outputs=big["outputs"], offsets=big["offsets"][a:a + max(n, 1)],
                         lengths=big["lengths"][a:a + max(n, 1)], n=n, first=a))

    def descs(order):
        out = []
        for i in order:
            b = subs[i]
            n = b["n"]
            b["res"] = (torch.full((max(n, 1),), 7, dtype=torch.uint8, device="cuda"),
                        torch.zeros(max(n, 1), dtype=torch.int32, device="cuda"),
                        torch.zeros(1, dtype=torch.int32, device="cuda"))
            fl, rows, cnt = b["res"]
            out.append(dict(tweak_x=b["tweak_x"], tweak_y=b["tweak_y"], outputs=b["outputs"], offsets=b["offsets"],
                            lengths=b["lengths"], flags=fl[:n], match_rows=rows, match_count=cnt))
        return out

    with Scanner(SCAN, SPEND, labels, max_rows=1000) as s:
        for order in (range(600), range(599, -1, -1)):
            s.scan_device_batches(descs(order))
            s.sync()
            found = 0
            for b in subs:
                n, a = b["n"], b["first"]
                fl, rows, cnt = b["res"]
                got = fl[:n].cpu().numpy()
                assert (got == want[a:a + n]).all(), "batch at row %d" % a
                c = int(cnt.item())
                assert sorted(rows[:c].cpu().tolist()) == np.nonzero(want[a:a + n])[0].tolist()
                found += c
            assert found == int(want.sum()) > 0


@pytest.mark.parametrize("pipe", ["1", "0"])
@pytest.mark.parametrize("g1,g2", [("100000", "100000"), ("100", "0")])
def test_multi_exceptional_label_sums(torch, monkeypatch, pipe, g1, g2):
    """k_scan_multi -- the kernel of every default batch -- with label keys
    that make a row's label sum exceptional inside a thread's piece: rows 5,
    69 and 133 sit in one lane of consecutive wave-rows (one thread's piece in
    the all-6-row regime), with L_0 = F(row 5) (the sum doubles), L_2 =
    -F(row 69) (the sum is the point at infinity) and L_3 = F(row 133), next
    to an ordinary label and ordinary rows.  Row 5 carries the doubled sum's
    value and must match; row 69 carries INT64_MIN and 0 and must not (a label
    at infinity never matches).  Pipelined and two-inversion schedules
    (CUDASP_MULTI_PIPE), all-6-row and adaptive pieces, and the two stage
    kernels as control: flags equal the oracle's, which follows the
    reference's Python oracle there (scripts/compute_bip352_expected.py:42-46)."""
    import variants as V
    from oracle import oracle
    monkeypatch.setenv("CUDASP_MULTI_PIPE", pipe)
    monkeypatch.setenv("CUDASP_MULTI_G1", g1)
    monkeypatch.setenv("CUDASP_MULTI_G2", g2)
    n = 64 * 6 * 2 + 17
    b = make_batch(torch, 31337, n)
    xs = b["tweak_x"].cpu().numpy().view(np.uint32)
    ys = b["tweak_y"].cpu().numpy().view(np.uint32)
    tw = np.ascontiguousarray(np.concatenate([xs.T, ys.T], axis=1).astype("<u4")).view(np.uint8).reshape(n, 64)
    ra, rb, rc = 5, 5 + 64, 5 + 128
    F = [V.row(SCAN, SPEND, [], bytes(tw[i]))[0][0][0] for i in (ra, rb, rc)]
    labels = [V.point_blob(F[0]), LABEL, V.point_blob(V.neg(F[1])), V.point_blob(F[2])]
    _, vals = oracle.scan(SCAN, SPEND, labels, tw, want_values=True)
    assert vals[rb, 3] == oracle.LABEL_INFINITY
    outs = b["outputs"].cpu().numpy()
    offs = b["offsets"][:n].cpu().numpy().view(np.uint32)
    lens = b["lengths"][:n].cpu().numpy().view(np.uint32)
    assert (lens == 2).all()
    for i in range(n):
        if i in (ra, rb, rc):
            continue
        if i % 11 == 0:
            outs[offs[i]] = vals[i, 0]       # base
        elif i % 9 == 0:
            outs[offs[i] + 1] = vals[i, 2]   # the ordinary label
    outs[offs[ra]] = vals[ra, 1]             # F + L_0 = 2F
    outs[offs[rb]] = oracle.LABEL_INFINITY   # F + L_2 = infinity: never a match
    outs[offs[rb] + 1] = 0
    outs[offs[rc] + 1] = vals[rc, 4]         # F + L_3 = 2F as well
    b["outputs"] = torch.from_numpy(outs).cuda()
    want, _ = oracle.scan(SCAN, SPEND, labels, tw, outs, offs, lens, threads=16)
    assert want[ra] == 1 and want[rb] == 0 and want[rc] == 1
    got = run_multi(torch, [b], labels)[0]
    assert (got[0] == want).all()
    assert got[1] == np.nonzero(want)[0].tolist()
    same([got], run_per_batch(torch, [b], labels))  # the fused single-batch launch
    monkeypatch.setenv("CUDASP_FUSED_SINGLE", "0")
    same([got], run_per_batch(torch, [b], labels))  # the two stage kernels
