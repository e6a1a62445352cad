"""Pure-Python statement of the protocol variants (cudasp_scan_options,
include/cudasp_abi.h) for small test cases.

TEST INFRASTRUCTURE ONLY.  The reference implements none of the variants (it
hashes output index 0, adds labels without negation and compares the upper
64 bits of x: src/cudasp_gpu.cu:278-282, :133-172, :29-41), so their parity is
*unpinned* against it; these functions restate BIP-352's definitions
(t_k = hash_BIP0352/SharedSecret(ser_P(S) || ser_32(k)), P_k = B + t_k G) in
the reference's own pipeline shape (scripts/compute_bip352_expected.py:109-164)
so the C oracle and the GPU kernels can be checked against an independent
implementation.
"""
import hashlib

P = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F
N = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
G = (0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
     0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8)
TAG = hashlib.sha256(b"BIP0352/SharedSecret").digest()
LABEL_INFINITY = -(1 << 63)


def add(p, q):
    if p is None:
        return q
    if q is None:
        return p
    if p[0] == q[0]:
        if (p[1] + q[1]) % P == 0:
            return None
        lam = 3 * p[0] * p[0] * pow(2 * p[1], P - 2, P) % P
    else:
        lam = (q[1] - p[1]) * pow(q[0] - p[0], P - 2, P) % P
    x = (lam * lam - p[0] - q[0]) % P
    return (x, (lam * (p[0] - x) - p[1]) % P)


def mul(k, p):
    r = None
    while k:
        if k & 1:
            r = add(r, p)
        p = add(p, p)
        k >>= 1
    return r


def neg(p):
    return (p[0], (-p[1]) % P)


def point_le(blob):
    return (int.from_bytes(blob[:32], "little"), int.from_bytes(blob[32:64], "little"))


def point_blob(p):
    return p[0].to_bytes(32, "little") + p[1].to_bytes(32, "little")


def upper64(x):
    v = x >> 192
    return v - (1 << 64) if v >= 1 << 63 else v


def row(scan_le, spend_le, labels_le, tweak_le, output_count=1, label_negation=False):
    """-> per output index k: list of candidate points [F, F + L_0, ...,
    (F - L_0, ...)] (None at infinity), and the digests t_k."""
    d = int.from_bytes(scan_le, "little")
    S = mul(d, point_le(tweak_le))
    B = point_le(spend_le)
    labs = [point_le(l) for l in labels_le]
    if label_negation:
        labs = labs + [neg(l) for l in labs]
    out, digests = [], []
    for k in range(output_count):
        ser = bytes([2 | (S[1] & 1)]) + S[0].to_bytes(32, "big") + k.to_bytes(4, "big")
        h = hashlib.sha256(TAG + TAG + ser).digest()
        digests.append(h)
        F = add(mul(int.from_bytes(h, "big"), G), B)
        out.append([F] + [add(F, l) for l in labs])
    return out, digests


def values(cands):
    return [[LABEL_INFINITY if p is None else upper64(p[0]) for p in ks] for ks in cands]


def x_bytes(p):
    return p[0].to_bytes(32, "big")
