"""CPU: the kernel math of duckdb-cudasp-extension_amd/csrc/*.hpp, compiled for
the host with every field-magnitude precondition checked (tests/native), against
Python integers, the golden fixtures and the C oracle.  This is how the HIP
arithmetic is verified in the GPU-less build container; the GPU parity tests
(-m gpu) then check the device build of the same code."""
import ctypes
import os
import random
import subprocess

import numpy as np
import pytest

import golden_io
from oracle import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
P = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
GX = 0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798
GY = 0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8
LAMBDA = 0x5363ad4cc05c30e0a5261c028812645a122e22ea20816678df02967c1b23bd72


@pytest.fixture(scope="module", params=["libcudasp_emu.so", "libcudasp_emu29.so"], ids=["10x26", "9x29"])
def emu(request):
    """The kernel math host-compiled once per field layout (tests/native)."""
    path = os.path.join(HERE, "native", request.param)
    subprocess.check_call(["make", "-s", "-C", os.path.join(HERE, "native")])  # rebuilds when csrc changed
    lib = ctypes.CDLL(path)
    V = ctypes.c_void_p
    lib.emu_row_values.argtypes = [V, V, V, ctypes.c_uint32, V, ctypes.c_uint32, V, V, V, V, V, V]
    lib.emu_fb_entry.argtypes = [ctypes.c_uint32, ctypes.c_uint32, V]
    lib.emu_fb_layout.argtypes = [V, V, V]
    lib.emu_pend_invert.argtypes = [ctypes.c_char_p, ctypes.c_int, V]
    lib.emu_wnaf.argtypes = [V, ctypes.c_int, V, ctypes.c_int]
    lib.emu_fe_raw_op.argtypes = [ctypes.c_int, V, V, V, V, V]
    return lib


def _add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    if a[0] == b[0]:
        if (a[1] + b[1]) % P == 0:
            return None
        lam = 3 * a[0] * a[0] * pow(2 * a[1], -1, P) % P
    else:
        lam = (b[1] - a[1]) * pow(b[0] - a[0], -1, P) % P
    x = (lam * lam - a[0] - b[0]) % P
    return (x, (lam * (a[0] - x) - a[1]) % P)


def _mul(k, p=(GX, GY)):
    r = None
    while k:
        if k & 1:
            r = _add(r, p)
        p = _add(p, p)
        k >>= 1
    return r


def _le(pt):
    return pt[0].to_bytes(32, "little") + pt[1].to_bytes(32, "little")


def test_field_ops(emu):
    rng = random.Random(11)
    out = ctypes.create_string_buffer(32)
    edge = [0, 1, P - 1, P, P + 1, 2**256 - 1, 2**255, 2**32 + 977]
    vals = edge + [rng.getrandbits(256) for _ in range(600)]
    for a in vals:
        b = rng.choice(vals)
        emu.emu_fe_mul(a.to_bytes(32, "little"), b.to_bytes(32, "little"), out)
        assert int.from_bytes(out.raw, "little") == a * b % P
        emu.emu_fe_sqr(a.to_bytes(32, "little"), out)
        assert int.from_bytes(out.raw, "little") == a * a % P
        emu.emu_fe_normalize(a.to_bytes(32, "little"), out)
        assert int.from_bytes(out.raw, "little") == a % P
    inv_vals = vals[:40] + [P - 2, 2, 3, 2**255, 2**256 - 2**32 - 978, P + 5] + [rng.randrange(1, P) for _ in range(3000)]
    for a in inv_vals:
        if a % P == 0:
            continue
        emu.emu_fe_inv(a.to_bytes(32, "little"), out)  # safegcd (the kernels' inversion)
        assert int.from_bytes(out.raw, "little") == pow(a, -1, P), hex(a)
    for a in inv_vals[:60]:
        if a % P == 0:
            continue
        emu.emu_fe_inv_fermat(a.to_bytes(32, "little"), out)
        assert int.from_bytes(out.raw, "little") == pow(a, -1, P)


def test_field_magnitude_edges(emu):
    """The host build of the field ops at the edges of the magnitude rules
    (same cases as tests/test_gpu_field.py), preconditions checked."""
    import test_gpu_field as g
    n = emu.emu_fe_limbs()
    lay = (dict(limbs=9, bits=29, top=24, mul_max=7, sqr_max=2, limb_max=7, slack=(1 << 16, 1 << 11)) if n == 9 else
           dict(limbs=10, bits=26, top=22, mul_max=400, sqr_max=20, limb_max=31, slack=(1 << 23, 1 << 13)))
    out = np.zeros(n, dtype=np.uint32)

    def run(op, a, b, c, e):
        for i in range(a.shape[0]):
            args = [np.ascontiguousarray(x[i]) for x in (a, b, c, e)]
            assert emu.emu_fe_raw_op(op, *[x.ctypes.data for x in args], out.ctypes.data) == 0
            assert (out.astype(np.uint64) <= g.limb_bounds(lay, 1)).all(), op
            va, vb, vc, ve = (g.value(lay, x) for x in args)
            want = g.FUSED[op](va, vb, vc, ve) if op >= 2 else (va * vb if op == 0 else va * va)
            assert g.value(lay, out) % P == want % P, (op, i)

    rng = np.random.default_rng(5)
    for ma, mb in g.mag_pairs(lay):
        a, b = g.operands(lay, rng, ma, 16), g.operands(lay, rng, mb, 16)
        run(0, a, b, a, a)
    for m in range(1, lay["sqr_max"] + 1):
        a = g.operands(lay, rng, m, 16)
        run(1, a, a, a, a)
    if n == 9:
        for op, ma, mb, mc, me in g.fused_cases(lay):
            run(op, *(g.operands(lay, rng, m, 8) for m in (ma, mb, mc, me)))


def test_glv_split(emu):
    rng = random.Random(5)
    k1b, k2b = ctypes.create_string_buffer(32), ctypes.create_string_buffer(32)
    n1, n2 = ctypes.c_int(), ctypes.c_int()
    for k in [1, 2, N - 1, N // 2, LAMBDA] + [rng.randrange(1, N) for _ in range(300)]:
        emu.emu_glv_split(k.to_bytes(32, "little"), k1b, ctypes.byref(n1), k2b, ctypes.byref(n2))
        k1 = int.from_bytes(k1b.raw, "little") * (-1 if n1.value else 1)
        k2 = int.from_bytes(k2b.raw, "little") * (-1 if n2.value else 1)
        assert (k1 + k2 * LAMBDA - k) % N == 0
        assert abs(k1) < 2**129 and abs(k2) < 2**129


def test_wnaf(emu):
    rng = random.Random(9)
    d = (ctypes.c_int8 * 300)()
    for k in [0, 1, 15, 16, 31, 2**129 - 1] + [rng.getrandbits(130) for _ in range(200)]:
        ln = emu.emu_wnaf(k.to_bytes(32, "little"), 5, d, 300)
        digits = list(d)
        assert sum(x << i for i, x in enumerate(digits)) == k
        nz = [i for i, x in enumerate(digits) if x]
        assert all(digits[i] % 2 and -16 < digits[i] < 16 for i in nz)
        assert all(b - a >= 5 for a, b in zip(nz, nz[1:]))
        assert ln == (nz[-1] + 1 if nz else 0)


def test_scan_digits(emu):
    """The ladder digits (scalar_host.hpp scan_digits): any lattice point
    searched must still represent d = k1 + k2 lambda (mod n) as two width-5
    NAFs, and the chosen one costs no more than the Babai split (search 0)."""
    rng = random.Random(21)
    M = 136
    naf = (ctypes.c_int8 * (2 * M))()
    ln = ctypes.c_uint32()
    emu.emu_scan_digits.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    sc = golden_io.load("sql_cases.json")
    keys = [int.from_bytes(bytes.fromhex(sc["queries"][0]["scan_key"]), "little"), 1, 2, N - 1, LAMBDA]
    keys += [rng.randrange(1, N) for _ in range(60)]
    saved = 0
    for d in keys:
        costs = []
        for search in (0, 8):
            assert emu.emu_scan_digits(d.to_bytes(32, "little"), search, naf, M, ctypes.byref(ln)) == 0
            dg = list(naf)
            k1 = sum(x << i for i, x in enumerate(dg[:M]))
            k2 = sum(x << i for i, x in enumerate(dg[M:]))
            assert (k1 + k2 * LAMBDA - d) % N == 0
            for half in (dg[:M], dg[M:]):
                nz = [i for i, x in enumerate(half) if x]
                assert all(half[i] % 2 and -16 < half[i] < 16 for i in nz)
                assert all(b - a >= 5 for a, b in zip(nz, nz[1:]))
            top = max([i + 1 for i, x in enumerate(dg[:M]) if x] + [i + 1 for i, x in enumerate(dg[M:]) if x])
            assert ln.value == top
            weight = sum(1 for x in dg if x)
            costs.append((ln.value - 1) * 903 + (weight - 1) * 1600)
        assert costs[1] <= costs[0]
        saved += costs[0] - costs[1]
    assert saved > 0


def fb_layout(emu):
    bits, windows, entries = ctypes.c_int(), ctypes.c_int(), ctypes.c_uint32()
    emu.emu_fb_layout(ctypes.byref(bits), ctypes.byref(windows), ctypes.byref(entries))
    return bits.value, windows.value, entries.value


def test_fixed_base_layout(emu):
    bits, windows, entries = fb_layout(emu)
    assert entries == 1 << (bits - 1) and windows * bits >= 256 > (windows - 1) * bits


def test_fixed_base_entries(emu):
    rng = random.Random(13)
    bits, windows, entries = fb_layout(emu)
    out = (ctypes.c_uint32 * 16)()
    cases = [(0, 0), (0, entries - 1), (windows - 1, 0), (windows - 1, entries - 1)]
    cases += [(rng.randrange(windows), rng.randrange(entries)) for _ in range(6)]
    for w, j in cases:
        emu.emu_fb_entry(w, j, out)
        x = sum(out[i] << (32 * i) for i in range(8))
        y = sum(out[8 + i] << (32 * i) for i in range(8))
        assert (x, y) == _mul((2 * j + 1) << (bits * w))


def test_fixed_base_mul_recoding(emu):
    """fixed_base_mul's constant-free recoding: t mod n (t >= n is possible,
    the hash is not reduced), the odd representative n - t for even t (the
    point negated), signed digits with a positive top digit."""
    rng = random.Random(17)
    ts = [1, 2, 3, N - 1, N - 2, N + 1, N + 2, N + 12345, (1 << 256) - 1, (1 << 256) - 2, 1 << 255,
          (1 << 255) + 1, 2 * N - (1 << 256) + 7]
    ts += [rng.getrandbits(256) for _ in range(24)]
    out = (ctypes.c_uint32 * 16)()
    for t in ts:
        tw = (ctypes.c_uint32 * 8)(*[(t >> (32 * i)) & 0xFFFFFFFF for i in range(8)])
        assert emu.emu_fixed_base_mul(tw, out) == 0
        x = sum(out[i] << (32 * i) for i in range(8))
        y = sum(out[8 + i] << (32 * i) for i in range(8))
        assert (x, y) == _mul(t % N), hex(t)


def _w16(pt):
    return (ctypes.c_uint32 * 16)(*[(pt[0] >> (32 * i)) & 0xFFFFFFFF for i in range(8)],
                                  *[(pt[1] >> (32 * i)) & 0xFFFFFFFF for i in range(8)])


def _pt(out):
    return (sum(out[i] << (32 * i) for i in range(8)), sum(out[8 + i] << (32 * i) for i in range(8)))


def test_spend_key_folded_into_top_window(emu):
    """The spend key folded into the fixed-base table's top window
    (ScanConsts::fb_top, round 5): fb_fold_entry gives P + B and P - B; with
    it fixed_base_mul returns t G + B directly -- for odd t and for even t
    (whose lanes read the - B half and negate at the end), t >= n, and the
    scalar extremes -- equal to the separate chord addition of the
    reference; x(P) = x(B) is refused (the scanner then adds B on its own);
    the on-curve check accepts B and rejects (x, y + 1)."""
    rng = random.Random(352)
    ts = [1, 2, 3, N - 1, N - 2, N + 1, (1 << 256) - 1, (1 << 256) - 2, 1 << 255]
    ts += [rng.getrandbits(256) for _ in range(24)]
    out = (ctypes.c_uint32 * 16)()
    for i, t in enumerate(ts):
        B = _mul(rng.randrange(1, N))
        assert emu.emu_on_curve(_w16(B)) == 1
        tw = (ctypes.c_uint32 * 8)(*[(t >> (32 * q)) & 0xFFFFFFFF for q in range(8)])
        assert emu.emu_fixed_base_mul_folded(tw, _w16(B), out) == 0
        assert _pt(out) == _add(_mul(t % N), B), hex(t)
    B = _mul(12345)
    assert emu.emu_on_curve(_w16((B[0], (B[1] + 1) % P))) == 0
    P0 = _mul(777)
    pos, neg = (ctypes.c_uint32 * 16)(), (ctypes.c_uint32 * 16)()
    assert emu.emu_fb_fold_entry(_w16(P0), _w16(B), pos, neg) == 1
    assert _pt(pos) == _add(P0, B) and _pt(neg) == _add(P0, (B[0], P - B[1]))
    assert emu.emu_fb_fold_entry(_w16(P0), _w16(P0), pos, neg) == 0  # x(P) = x(B): doubling / infinity


def _values(emu, scan, spend, labels, tweaks, outs=None, offs=None, lens=None):
    n = len(tweaks) // 64
    L = len(labels)
    vals = (ctypes.c_int64 * (n * (1 + L)))()
    t = (ctypes.c_uint32 * (8 * n))()
    flags = (ctypes.c_uint8 * n)()
    p = lambda a: None if a is None else a.ctypes.data
    rc = emu.emu_row_values(scan, spend, b"".join(labels) if labels else None, L, tweaks, n, vals, t,
                            p(outs) if outs is not None and outs.size else None, p(offs), p(lens),
                            flags if outs is not None else None)
    assert rc == 0
    v = np.frombuffer(vals, dtype=np.int64).reshape(n, 1 + L)
    tt = np.frombuffer(t, dtype=np.uint32).reshape(n, 8)
    return v, tt, np.frombuffer(flags, dtype=np.uint8)


def test_stage_kats(emu):
    for k in golden_io.load("stage_kats.json"):
        labels = [bytes.fromhex(l) for l in k["label_keys"]]
        v, t, _ = _values(emu, bytes.fromhex(k["scan_key"]), bytes.fromhex(k["spend_key"]), labels,
                          bytes.fromhex(k["tweak"]))
        assert sum(int(t[0, j]) << (32 * j) for j in range(8)) == int(k["t"], 16)
        assert list(v[0]) == [k["v"]] + k["label_values"]


def test_random_rows_and_flags(emu):
    rr = golden_io.load("random_rows.json")
    rows = rr["rows"]
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    outs, offs, lens = golden_io.csr([r["outputs"] for r in rows])
    labels = [bytes.fromhex(l) for l in rr["label_keys"]]
    v, t, f = _values(emu, bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"]), labels, tw.tobytes(),
                      outs, offs, lens)
    assert list(v[:, 0]) == [r["v"] for r in rows]
    assert [list(x) for x in v[:, 1:]] == [r["label_values"] for r in rows]
    assert [bool(x) for x in f] == [r["match_all_labels"] for r in rows]


def test_against_oracle_random_keys(emu):
    """Random scan keys (including ones whose GLV halves are negative) and 2 labels."""
    rng = random.Random(21)
    for _ in range(3):
        scan = rng.randrange(1, N).to_bytes(32, "little")
        spend = _le(_mul(rng.randrange(1, N)))
        labels = [_le(_mul(rng.randrange(1, N))) for _ in range(2)]
        tw = b"".join(_le(_mul(rng.randrange(1, N))) for _ in range(6))
        v, _, _ = _values(emu, scan, spend, labels, tw)
        _, ov = oracle.scan(scan, spend, labels, np.frombuffer(tw, dtype=np.uint8).reshape(-1, 64), want_values=True)
        assert (v == ov).all()


def test_lds_y_split_equals_scratch_table(emu):
    """The kernels keep the y of odd multiples 1T..9T in LDS (LdsY<5>) and the
    rest in scratch: the same stage A with that split (a host array standing
    in for the LDS, another lane's slots interleaved) gives the t of the
    all-scratch table, and never touches those entries' scratch words."""
    emu.emu_shared_secret_lds_y.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_void_p]
    rng = random.Random(52)
    k = golden_io.load("stage_kats.json")[0]
    keys = [bytes.fromhex(k["scan_key"])] + [rng.randrange(1, N).to_bytes(32, "little") for _ in range(2)]
    spend = _le(_mul(7))
    for scan in keys:
        tw = b"".join(_le(_mul(rng.randrange(1, N))) for _ in range(4))
        _, t_ref, _ = _values(emu, scan, spend, [], tw)
        for stride in (1, 64):
            t = (ctypes.c_uint32 * (8 * 4))()
            assert emu.emu_shared_secret_lds_y(scan, tw, 4, stride, t) == 0
            assert (np.frombuffer(t, dtype=np.uint32).reshape(4, 8) == t_ref).all()


def test_exceptional_labels(emu):
    """Label == F doubles, label == -F is infinity (reference Python oracle
    semantics, scripts/compute_bip352_expected.py:42-46)."""
    k = [k for k in golden_io.load("stage_kats.json") if k["height"] == 200][0]
    F = (int(k["F_x"], 16), int(k["F_y"], 16))
    labels = [_le(F), _le((F[0], (-F[1]) % P))]
    v, _, _ = _values(emu, bytes.fromhex(k["scan_key"]), bytes.fromhex(k["spend_key"]), labels,
                      bytes.fromhex(k["tweak"]))
    two_f = _add(F, F)
    up = lambda x: (x >> 192) - (1 << 64) if (x >> 192) >= 1 << 63 else (x >> 192)
    assert v[0, 1] == up(two_f[0])
    assert v[0, 2] == oracle.LABEL_INFINITY
    _, ov = oracle.scan(bytes.fromhex(k["scan_key"]), bytes.fromhex(k["spend_key"]), labels,
                        golden_io.tweak_array([k["tweak"]]), want_values=True)
    assert list(ov[0]) == list(v[0])


def test_shared_inversion(emu):
    """pend_invert: several rows' Z inverted with one field inversion; a zero Z
    gets 0 (like fe_inv) without spoiling the other rows."""
    rng = random.Random(29)
    cases = [[rng.randrange(1, P) for _ in range(4)], [rng.randrange(1, P)], [0, rng.randrange(1, P), 5],
             [rng.randrange(1, P), 0], [0, 0, 0, 0], [P - 1, 1, 2, 3]]
    for zs in cases:
        buf = b"".join(z.to_bytes(32, "little") for z in zs)
        out = (ctypes.c_uint8 * (32 * len(zs)))()
        emu.emu_pend_invert(buf, len(zs), out)
        got = [int.from_bytes(bytes(out[32 * j:32 * j + 32]), "little") for j in range(len(zs))]
        assert got == [pow(z, P - 2, P) if z % P else 0 for z in zs], zs


def _grouped(emu, scan, spend, labels, tw, R, outs=None, offs=None, lens=None):
    n = len(tw) // 64
    L = len(labels)
    emu.emu_row_values_grouped.restype = ctypes.c_int
    P_ = ctypes.c_void_p
    emu.emu_row_values_grouped.argtypes = [P_, P_, P_, ctypes.c_uint32, P_, ctypes.c_uint32, ctypes.c_int, P_, P_, P_,
                                           P_, P_]
    lab = b"".join(labels) if labels else None
    vals = (ctypes.c_int64 * (n * (1 + L)))()
    assert emu.emu_row_values_grouped(scan, spend, lab, L, tw, n, R, vals, None, None, None, None) == 0
    v = np.frombuffer(vals, dtype=np.int64).reshape(1 + L, n).T
    f = None
    if outs is not None:
        fl = (ctypes.c_uint8 * n)()
        p = lambda a: a.ctypes.data
        assert emu.emu_row_values_grouped(scan, spend, lab, L, tw, n, R, None, p(outs) if outs.size else None,
                                          p(offs), p(lens), fl) == 0
        f = np.frombuffer(fl, dtype=np.uint8)
    return v, f


def test_grouped_stage_b_shared_label_inversion(emu):
    """The kernel's grouped stage B (k_match, ROWS_B rows per thread): one Z
    inversion and one label inversion shared by all rows of the group
    (match_labels_rows), with the magnitude checks on.  Values equal the
    per-row path and the oracle, including exceptional label sums inside the
    shared batch and partial groups; flags equal the fixtures'."""
    rr = golden_io.load("random_rows.json")
    rows = rr["rows"][:14]
    scan, spend = bytes.fromhex(rr["scan_key"]), bytes.fromhex(rr["spend_key"])
    tw = golden_io.tweak_array([r["tweak"] for r in rows])
    labels = [bytes.fromhex(l) for l in rr["label_keys"]]
    outs, offs, lens = golden_io.csr([r["outputs"] for r in rows])
    per_row, _, _ = _values(emu, scan, spend, labels, tw.tobytes())
    for R in (1, 4, 6, 8):
        v, f = _grouped(emu, scan, spend, labels, tw.tobytes(), R, outs, offs, lens)
        assert (v == per_row).all(), R
        assert [bool(x) for x in f] == [r["match_all_labels"] for r in rows], R
    # exceptional sums: L == F of row 0 (doubling), L == -F of row 1 (infinity)
    import variants as Vv
    F = [Vv.row(scan, spend, [], bytes.fromhex(r["tweak"]))[0][0][0] for r in rows[:2]]
    ex = [Vv.point_blob(F[0]), labels[0], Vv.point_blob(Vv.neg(F[1]))]
    v, _ = _grouped(emu, scan, spend, ex, tw.tobytes(), 6)
    _, ov = oracle.scan(scan, spend, ex, tw, want_values=True)
    assert (v == ov).all()
    assert ov[1, 3] == oracle.LABEL_INFINITY
