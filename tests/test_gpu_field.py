"""GPU: the kernels' field multiply / square (secp256k1_fe.hpp; on gfx950 the
generated asm blocks of secp256k1_fe_asm.inc) against Python integers, over the
whole input range the group formulas rely on: operand magnitudes with
mag(a) * mag(b) <= 400 (each <= 31), random limbs and every limb at its maximum.
The result must be congruent mod p and of magnitude 1."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

P = 2**256 - 2**32 - 977
MAG_PAIRS = [(1, 1), (2, 1), (8, 8), (7, 17), (17, 7), (15, 15), (20, 20), (31, 12), (12, 31), (16, 25), (1, 31),
             (31, 1), (3, 35 // 3)]


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def limb_bounds(m):
    b = np.full(10, m * (1 << 26) + (1 << 23), dtype=np.uint64)
    b[9] = m * (1 << 22) + (1 << 13)
    return b


def operands(rng, m, count):
    hi = limb_bounds(m)
    a = (rng.random((count, 10)) * (hi + 1)).astype(np.uint64)
    a[0] = hi           # every limb at its maximum
    a[1] = 0
    a[2] = hi
    a[2, 9] = 0
    return np.minimum(a, hi).astype(np.uint32)


def value(limbs):
    return sum(int(v) << (26 * k) for k, v in enumerate(limbs))


def run(torch, op, a, b):
    from cudasp_amd import _native
    lib = _native.load()
    da = torch.from_numpy(a.view(np.int32).copy()).cuda()
    db = torch.from_numpy(b.view(np.int32).copy()).cuda()
    out = torch.zeros_like(da)
    _native.check(lib.cudasp_debug_field_ops(op, da.data_ptr(), db.data_ptr(), out.data_ptr(), a.shape[0]))
    return out.cpu().numpy().view(np.uint32)


def check(a, b, r, sqr):
    bound = limb_bounds(1)
    assert (r.astype(np.uint64) <= bound).all(), "result not of magnitude 1"
    for i in range(a.shape[0]):
        va = value(a[i])
        vb = va if sqr else value(b[i])
        assert value(r[i]) % P == (va * vb) % P, (i, a[i], b[i], r[i])


@pytest.mark.parametrize("ma,mb", MAG_PAIRS)
def test_mul_magnitudes(torch, ma, mb):
    rng = np.random.default_rng(1000 * ma + mb)
    a = operands(rng, ma, 2048)
    b = operands(rng, mb, 2048)
    check(a, b, run(torch, 0, a, b), sqr=False)


@pytest.mark.parametrize("m", [1, 2, 8, 17, 20])
def test_sqr_magnitudes(torch, m):
    rng = np.random.default_rng(7 + m)
    a = operands(rng, m, 2048)
    check(a, a, run(torch, 1, a, a), sqr=True)


def test_mul_reduced_edge_values(torch):
    """Values around p and 2^256 in normal form."""
    vals = [0, 1, 2, P - 1, P - 2, P, P + 1, 2**256 - 1, 2**255, 2**32 + 977, 2**26 - 1, 2**52]
    rows = [[(v >> (26 * k)) & (2**26 - 1) if k < 9 else v >> 234 for k in range(10)] for v in vals]
    a = np.array([x for x in rows for _ in rows], dtype=np.uint32)
    b = np.array([y for _ in rows for y in rows], dtype=np.uint32)
    check(a, b, run(torch, 0, a, b), sqr=False)
    check(a, a, run(torch, 1, a, a), sqr=True)
