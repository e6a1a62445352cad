"""GPU: the kernels' field multiply / square (secp256k1_fe.hpp /
secp256k1_fe29.hpp; on gfx950 the generated asm blocks) against Python
integers, over the whole input range the group formulas rely on: every operand
magnitude pair the build's layout allows (cudasp_field_layout: 10 x 26 limbs
take mag(a) * mag(b) <= 400, 9 x 29 limbs <= 7), random limbs and every limb at
its maximum.  The 9 x 29 layout's fused forms (a b + c e, a b + c^2, a b + c,
a^2 + c, 3 a^2) are swept over every split of the shared budget.  The result must be
congruent mod p and of magnitude 1."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 2**256 - 2**32 - 977


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


@pytest.fixture(scope="module")
def layout(torch):
    from cudasp_amd import _native
    v = [ctypes.c_int() for _ in range(5)]
    _native.check(_native.load().cudasp_field_layout(*[ctypes.byref(x) for x in v]))
    limbs, bits, mul_max, sqr_max, limb_max = (x.value for x in v)
    top = 256 - bits * (limbs - 1)
    slack = (1 << 23, 1 << 13) if bits == 26 else (1 << 16, 1 << 11)
    return dict(limbs=limbs, bits=bits, top=top, mul_max=mul_max, sqr_max=sqr_max, limb_max=limb_max, slack=slack)


def limb_bounds(lay, m):
    b = np.full(lay["limbs"], m * (1 << lay["bits"]) + lay["slack"][0], dtype=np.uint64)
    b[-1] = m * (1 << lay["top"]) + lay["slack"][1]
    return b


def operands(lay, rng, m, count):
    hi = limb_bounds(lay, m)
    a = (rng.random((count, lay["limbs"])) * (hi + 1)).astype(np.uint64)
    a[0] = hi           # every limb at its maximum
    a[1] = 0
    a[2] = hi
    a[2, -1] = 0
    return np.minimum(a, hi).astype(np.uint32)


def value(lay, limbs):
    return sum(int(v) << (lay["bits"] * k) for k, v in enumerate(limbs))


def run(torch, op, a, b, c=None, e=None):
    from cudasp_amd import _native
    lib = _native.load()
    if c is not None:
        b = np.concatenate([b, c, e if e is not None else c])
    da = torch.from_numpy(a.view(np.int32).copy()).cuda()
    db = torch.from_numpy(b.view(np.int32).copy()).cuda()
    out = torch.zeros_like(da)
    _native.check(lib.cudasp_debug_field_ops(op, da.data_ptr(), db.data_ptr(), out.data_ptr(), a.shape[0]))
    return out.cpu().numpy().view(np.uint32)


FUSED = {2: lambda a, b, c, e: a * b + c * e, 3: lambda a, b, c, e: a * b + c * c,
         4: lambda a, b, c, e: a * b + c, 5: lambda a, b, c, e: a * a + c, 6: lambda a, b, c, e: 3 * a * a}


def fused_cases(lay):
    """(op, mag a, mag b, mag c, mag e) at the edge of the shared budget."""
    top, lim = lay["mul_max"], lay["limb_max"]
    cases = []
    for s in range(1, top):
        for ma in range(1, s + 1):
            if s % ma:
                continue
            mb = s // ma
            rest = top - s
            for mc in range(1, rest + 1):
                if rest % mc == 0:
                    cases.append((2, ma, mb, mc, rest // mc))
            for mc in range(1, lay["sqr_max"] + 1):
                if mc * mc <= rest:
                    cases.append((3, ma, mb, mc, 1))
    for ma in range(1, lim + 1):
        mb = min(lim, top // ma)
        cases.append((4, ma, mb, lim, 1))
    for ma in range(1, lay["sqr_max"] + 1):
        cases.append((5, ma, 1, lim, 1))
    cases.append((6, 1, 1, 1, 1))
    return cases


def check(lay, a, b, r, sqr):
    assert (r.astype(np.uint64) <= limb_bounds(lay, 1)).all(), "result not of magnitude 1"
    for i in range(a.shape[0]):
        va = value(lay, a[i])
        vb = va if sqr else value(lay, b[i])
        assert value(lay, r[i]) % P == (va * vb) % P, (i, a[i], b[i], r[i])


def mag_pairs(lay):
    top, lim = lay["mul_max"], lay["limb_max"]
    pairs = {(1, 1), (1, lim), (lim, 1)}
    for ma in range(1, lim + 1):
        mb = min(lim, top // ma)
        pairs.add((ma, mb))
    return sorted(pairs)


def test_mul_magnitudes(torch, layout):
    for ma, mb in mag_pairs(layout):
        rng = np.random.default_rng(1000 * ma + mb)
        a = operands(layout, rng, ma, 1024)
        b = operands(layout, rng, mb, 1024)
        check(layout, a, b, run(torch, 0, a, b), sqr=False)


def test_sqr_magnitudes(torch, layout):
    for m in range(1, layout["sqr_max"] + 1):
        rng = np.random.default_rng(7 + m)
        a = operands(layout, rng, m, 1024)
        check(layout, a, a, run(torch, 1, a, a), sqr=True)


def test_mul_reduced_edge_values(torch, layout):
    """Values around p and 2^256 in normal form."""
    vals = [0, 1, 2, P - 1, P - 2, P, P + 1, 2**256 - 1, 2**255, 2**32 + 977, 2**26 - 1, 2**52]
    bits, n = layout["bits"], layout["limbs"]
    rows = [[(v >> (bits * k)) & (2**bits - 1) if k < n - 1 else v >> (bits * (n - 1)) for k in range(n)] for v in vals]
    a = np.array([x for x in rows for _ in rows], dtype=np.uint32)
    b = np.array([y for _ in rows for y in rows], dtype=np.uint32)
    check(layout, a, b, run(torch, 0, a, b), sqr=False)
    check(layout, a, a, run(torch, 1, a, a), sqr=True)


def test_fused_magnitudes(torch, layout):
    if layout["limbs"] != 9:
        pytest.skip("fused forms exist in the 9 x 29 layout only")
    for op, ma, mb, mc, me in fused_cases(layout):
        rng = np.random.default_rng(10007 * op + 1000 * ma + 100 * mb + 10 * mc + me)
        a, b = operands(layout, rng, ma, 512), operands(layout, rng, mb, 512)
        c, e = operands(layout, rng, mc, 512), operands(layout, rng, me, 512)
        r = run(torch, op, a, b, c, e)
        assert (r.astype(np.uint64) <= limb_bounds(layout, 1)).all(), ("magnitude", op, ma, mb, mc, me)
        f = FUSED[op]
        for i in range(a.shape[0]):
            want = f(value(layout, a[i]), value(layout, b[i]), value(layout, c[i]), value(layout, e[i])) % P
            assert value(layout, r[i]) % P == want, (op, ma, mb, mc, me, i)


def test_inverse(torch, layout):
    """fe_inv (safegcd divsteps; on gfx950 partly asm) against pow(a, -1, p):
    random values of every magnitude the kernels pass in, 0, 1, p - 1, p,
    small and 2^k values, and values congruent to them."""
    rng = np.random.default_rng(4242)
    lay = layout
    vals = [0, 1, 2, 3, P - 1, P - 2, P, P + 1, 2 * P - 1, 2**255, 2**256 - 1, (P + 1) // 2, 977, 2**32 + 977]
    vals += [2**k for k in range(0, 256, 17)]
    rows = []
    for v in vals:
        limbs, x = [], v
        for k in range(lay["limbs"]):
            w = lay["bits"] if k < lay["limbs"] - 1 else 32
            limbs.append(x & ((1 << w) - 1))
            x >>= w
        assert x == 0
        rows.append(limbs)
    a = np.concatenate([np.array(rows, dtype=np.uint64).astype(np.uint32),
                        operands(lay, rng, 1, 4000), operands(lay, rng, 2, 4000)])
    r = run(torch, 7, a, np.zeros_like(a))
    for i in range(a.shape[0]):
        x = value(lay, a[i]) % P
        got = value(lay, r[i])
        assert got < P, i
        assert got == (pow(x, -1, P) if x else 0), (i, hex(x))
