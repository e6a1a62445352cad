"""Generate csrc/secp256k1_fe_asm.inc: fe_mul / fe_sqr as single inline-asm
blocks for gfx950 (CUDASP_FE_VARIANT 3).

Why one block per operation: clang reassociates the carry-free column sums
(it sums each column's products from zero and adds the carry afterwards with an
extra 64-bit add + register-pair moves), and per-instruction asm makes the
hazard recognizer pad every statement with s_nop.  One block holds the exact
schedule: every column is ONE v_mad_u64_u32 chain that starts from the
previous column's carry.

Layout (same arithmetic as variant 1, secp256k1_fe.hpp):
  * high columns c_10..c_18 -> pairs H0..H8 (fixed VGPRs), chains interleaved;
  * top = hi(H8) * (R1<<6)       (weight 2^260 again);
  * low column k: acc = carry + lo(H_k) R0 + lo(H_k-1) R1 + hi(H_k-1) (R0<<6)
                        + hi(H_k-2) (R1<<6) + sum a_i b_(k-i);
    r_k = acc & (2^26-1), acc >>= 26 (k < 9); r_9 = acc & (2^22-1), u = acc >> 22;
  * u * 2^256 = u * (F0 + F1 2^26) folded into r0..r2 through u's 32-bit halves.
Temporaries live in fixed VGPRs v[BASE .. BASE+25] (clobbered), the sdst of
every v_mad_u64_u32 is vcc (clobbered, never read).

    python tools/gen_fe_asm.py     (rewrites the .inc; commit both)
"""
import os

BASE = 96
M26 = "0x3ffffff"
M22 = "0x3fffff"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "duckdb-cudasp-extension_amd", "csrc",
                   "secp256k1_fe_asm.inc")
OUT29 = os.path.join(os.path.dirname(OUT), "secp256k1_fe29_asm.inc")


def pair(i):
    return "v[%d:%d]" % (BASE + i, BASE + i + 1)


def lo(i):
    return "v%d" % (BASE + i)


def hi(i):
    return "v%d" % (BASE + i + 1)


H = [2 * m for m in range(9)]  # H_m pair offset
ACC, Z, Y, W = 18, 20, 22, 24  # accumulator, r0 pair, r1 pair, top
NTMP = 26


def product_terms(k, sqr):
    """(x, y) operand names of column k's products."""
    t = []
    for i in range(10):
        j = k - i
        if j < 0 or j >= 10:
            continue
        if sqr:
            if j > i:
                t.append(("%[d" + str(i) + "]", "%[a" + str(j) + "]"))
            elif j == i:
                t.append(("%[a" + str(i) + "]", "%[a" + str(i) + "]"))
        else:
            t.append(("%[a" + str(i) + "]", "%[b" + str(j) + "]"))
    return t


def gen(sqr):
    ins = []

    def mad(dst, x, y, acc):
        ins.append("v_mad_u64_u32 %s, vcc, %s, %s, %s" % (dst, x, y, acc))

    # high columns, interleaved round-robin across the 9 chains
    cols = [product_terms(10 + m, sqr) for m in range(9)]
    depth = max(len(c) for c in cols)
    for d in range(depth):
        for m in range(9):
            if d < len(cols[m]):
                x, y = cols[m][d]
                mad(pair(H[m]), x, y, "0" if d == 0 else pair(H[m]))
    mad(pair(W), hi(H[8]), "%[r1s]", "0")  # top, weight 2^260
    # low columns: one chain each, seeded with the previous carry
    for k in range(10):
        terms = []
        if k < 9:
            terms.append((lo(H[k]), "%[r0]"))
        if k == 0:
            terms.append((lo(W), "%[r0]"))
        if 1 <= k <= 9:
            terms += [(lo(H[k - 1]), "%[r1]"), (hi(H[k - 1]), "%[r0s]")]
        if k == 1:
            terms += [(lo(W), "%[r1]"), (hi(W), "%[r0s]")]
        if 2 <= k <= 9:
            terms.append((hi(H[k - 2]), "%[r1s]"))
        if k == 2:
            terms.append((hi(W), "%[r1s]"))
        terms += product_terms(k, sqr)
        for n, (x, y) in enumerate(terms):
            mad(pair(ACC), x, y, "0" if (k == 0 and n == 0) else pair(ACC))
        if k == 0:
            ins.append("v_and_b32 %s, %s, %s" % (lo(Z), M26, lo(ACC)))
            ins.append("v_mov_b32 %s, 0" % hi(Z))
        elif k == 1:
            ins.append("v_and_b32 %s, %s, %s" % (lo(Y), M26, lo(ACC)))
            ins.append("v_mov_b32 %s, 0" % hi(Y))
        elif k < 9:
            ins.append("v_and_b32 %%[o%d], %s, %s" % (k, M26, lo(ACC)))
        else:
            ins.append("v_and_b32 %%[o9], %s, %s" % (M22, lo(ACC)))
        ins.append("v_lshrrev_b64 %s, %d, %s" % (pair(ACC), 26 if k < 9 else 22, pair(ACC)))
    # u = ACC (< 2^42): u * 2^256 = u*F0 + u*F1 * 2^26
    ulo, uhi = lo(ACC), hi(ACC)
    mad(pair(Z), ulo, "%[f0]", pair(Z))                                  # r0 + ulo F0 (< 2^52)
    ins.append("v_and_b32 %%[o0], %s, %s" % (M26, lo(Z)))
    ins.append("v_alignbit_b32 %s, %s, %s, 26" % (lo(W), hi(Z), lo(Z)))  # carry (< 2^26)
    ins.append("v_add_u32 %s, %s, %s" % (lo(Y), lo(Y), lo(W)))
    mad(pair(Y), ulo, "64", pair(Y))                                     # + ulo F1 (F1 = 64)
    mad(pair(Y), uhi, "%[f0s]", pair(Y))                                 # + uhi (F0<<6)
    ins.append("v_and_b32 %%[o1], %s, %s" % (M26, lo(Y)))
    ins.append("v_alignbit_b32 %s, %s, %s, 26" % (lo(W), hi(Y), lo(Y)))  # carry (< 2^23)
    ins.append("v_lshl_add_u32 %s, %s, 12, %s" % (lo(W), uhi, lo(W)))   # + uhi (F1<<6) = uhi << 12
    ins.append("v_add_u32 %%[o2], %%[o2], %s" % lo(W))
    return ins


class Layout:
    """Limb layout: n limbs of `bits` bits, the top one `top` bits (n*bits ..
    256); 2^(n*bits) = r0 + r1*2^bits and 2^256 = f0 + f1*2^bits (mod p)."""

    def __init__(self, n, bits, top, r0, r1, f0, f1, top_has_hi):
        self.n, self.bits, self.top, self.r0, self.r1, self.f0, self.f1 = n, bits, top, r0, r1, f0, f1
        self.s = 32 - bits              # hi * 2^32 = (hi << s) * 2^bits
        self.top_has_hi = top_has_hi    # the wrapped term hi(H_(n-2)) * (r1 << s) may exceed 32 bits
        self.mask = "0x%x" % ((1 << bits) - 1)
        self.tmask = "0x%x" % ((1 << top) - 1)


L26 = Layout(10, 26, 22, 0x3D10, 0x400, 0x3D1, 0x40, True)
L29 = Layout(9, 29, 24, 0x7A20, 0x100, 0x3D1, 0x8, False)


def product_terms_l(lay, k, sqr):
    t = []
    for i in range(lay.n):
        j = k - i
        if j < 0 or j >= lay.n:
            continue
        if sqr:
            if j > i:
                t.append(("%[d" + str(i) + "]", "%[a" + str(j) + "]"))
            elif j == i:
                t.append(("%[a" + str(i) + "]", "%[a" + str(i) + "]"))
        else:
            t.append(("%[a" + str(i) + "]", "%[b" + str(j) + "]"))
    return t


def gen_layout(lay, sqr):
    """gen() for any Layout (serial schedule)."""
    return gen_layout_terms(lay, lambda k: product_terms_l(lay, k, sqr))


def spec_terms(lay, k, spec):
    """Column k's terms of a sum of products: spec = [("mul", x, y) |
    ("sqr", x, d) | ("sqr3", x, q)] with operand prefixes: d = the doubled
    limbs of x; for 3 x^2, q = 6 x for the cross products and q + "h" = 3 x
    for the squares.  (Prefixes must not collide with the constants' names
    r0, r1, r0s, r1s, f0, f0s or the outputs o0...)"""
    t = []
    for kind, x, y in spec:
        for i in range(lay.n):
            j = k - i
            if j < 0 or j >= lay.n:
                continue
            if kind == "mul":
                t.append(("%%[%s%d]" % (x, i), "%%[%s%d]" % (y, j)))
            elif j > i:
                t.append(("%%[%s%d]" % (y, i), "%%[%s%d]" % (x, j)))
            elif j == i:
                diag = x if kind == "sqr" else y + "h"
                t.append(("%%[%s%d]" % (diag, i), "%%[%s%d]" % (x, i)))
    return t


def gen_layout_terms(lay, col_terms, addend=None):
    """Serial schedule of one reduced sum of products: col_terms(k) gives
    product column k's (x, y) operand pairs; addend (an operand prefix) is a
    field element added into the low columns (one mad by 1 per limb)."""
    n = lay.n
    ins = []
    H = [2 * m for m in range(n - 1)]
    ACC, Z, Y, W = 2 * (n - 1), 2 * (n - 1) + 2, 2 * (n - 1) + 4, 2 * (n - 1) + 6

    def mad(dst, x, y, acc):
        ins.append("v_mad_u64_u32 %s, vcc, %s, %s, %s" % (dst, x, y, acc))

    cols = [col_terms(n + m) for m in range(n - 1)]
    depth = max(len(c) for c in cols)
    for d in range(depth):
        for m in range(n - 1):
            if d < len(cols[m]):
                x, y = cols[m][d]
                mad(pair(H[m]), x, y, "0" if d == 0 else pair(H[m]))
    mad(pair(W), hi(H[n - 2]), "%[r1s]", "0")  # wraps to weight 2^(n bits)
    for k in range(n):
        terms = []
        if k < n - 1:
            terms.append((lo(H[k]), "%[r0]"))
        if k == 0:
            terms.append((lo(W), "%[r0]"))
        if 1 <= k <= n - 1:
            terms += [(lo(H[k - 1]), "%[r1]"), (hi(H[k - 1]), "%[r0s]")]
        if k == 1:
            terms.append((lo(W), "%[r1]"))
            if lay.top_has_hi:
                terms.append((hi(W), "%[r0s]"))
        if 2 <= k <= n - 1 and k - 2 <= n - 3:
            terms.append((hi(H[k - 2]), "%[r1s]"))
        if k == 2 and lay.top_has_hi:
            terms.append((hi(W), "%[r1s]"))
        terms += col_terms(k)
        if addend is not None:
            terms.append(("%%[%s%d]" % (addend, k), "1"))
        for m_, (x, y) in enumerate(terms):
            mad(pair(ACC), x, y, "0" if (k == 0 and m_ == 0) else pair(ACC))
        if k == 0:
            ins += ["v_and_b32 %s, %s, %s" % (lo(Z), lay.mask, lo(ACC)), "v_mov_b32 %s, 0" % hi(Z)]
        elif k == 1:
            ins += ["v_and_b32 %s, %s, %s" % (lo(Y), lay.mask, lo(ACC)), "v_mov_b32 %s, 0" % hi(Y)]
        elif k < n - 1:
            ins.append("v_and_b32 %%[o%d], %s, %s" % (k, lay.mask, lo(ACC)))
        else:
            ins.append("v_and_b32 %%[o%d], %s, %s" % (k, lay.tmask, lo(ACC)))
        ins.append("v_lshrrev_b64 %s, %d, %s" % (pair(ACC), lay.bits if k < n - 1 else lay.top, pair(ACC)))
    ulo, uhi = lo(ACC), hi(ACC)
    t = lo(W)
    f1s_shift = (lay.f1 << lay.s).bit_length() - 1
    assert (lay.f1 << lay.s) == 1 << f1s_shift
    ins += [("v_mad_u64_u32 %s, vcc, %s, %%[f0], %s" % (pair(Z), ulo, pair(Z))),
            "v_and_b32 %%[o0], %s, %s" % (lay.mask, lo(Z)),
            "v_alignbit_b32 %s, %s, %s, %d" % (t, hi(Z), lo(Z), lay.bits),
            "v_add_u32 %s, %s, %s" % (lo(Y), lo(Y), t),
            "v_mad_u64_u32 %s, vcc, %s, %d, %s" % (pair(Y), ulo, lay.f1, pair(Y)),
            "v_mad_u64_u32 %s, vcc, %s, %%[f0s], %s" % (pair(Y), uhi, pair(Y)),
            "v_and_b32 %%[o1], %s, %s" % (lay.mask, lo(Y)),
            "v_alignbit_b32 %s, %s, %s, %d" % (t, hi(Y), lo(Y), lay.bits),
            "v_lshl_add_u32 %s, %s, %d, %s" % (t, uhi, f1s_shift, t),
            "v_add_u32 %%[o2], %%[o2], %s" % t]
    return ins, 2 * (n - 1) + 8


def emit_layout(lay, name, sqr):
    ins, ntmp = gen_layout(lay, sqr)
    n = lay.n
    body = "\n".join('      "%s\\n"' % s for s in ins)
    outs = ", ".join('[o%d] "=&v"(r.n[%d])' % (k, k) for k in range(n))
    if sqr:
        inl = ['[a%d] "v"(a.n[%d])' % (i, i) for i in range(n)] + ['[d%d] "v"(d[%d])' % (i, i) for i in range(n - 1)]
    else:
        inl = ['[a%d] "v"(a.n[%d])' % (i, i) for i in range(n)] + ['[b%d] "v"(b.n[%d])' % (i, i) for i in range(n)]
    inl += ['[r0] "s"(c_r0)', '[r1] "s"(c_r1)', '[r0s] "s"(c_r0s)', '[r1s] "s"(c_r1s)', '[f0] "s"(c_f0)',
            '[f0s] "s"(c_f0s)']
    clob = ", ".join(['"vcc"'] + ['"v%d"' % (BASE + i) for i in range(ntmp)])
    sig = "fe& r, const fe& a" if sqr else "fe& r, const fe& a, const fe& b"
    pre = ""
    if sqr:
        pre = "  uint32_t d[%d];\n#pragma unroll\n  for (int i = 0; i < %d; i++) d[i] = a.n[i] << 1;\n" % (n - 1, n - 1)
    return ("__device__ __forceinline__ void %s(%s) {\n%s"
            "  const uint32_t c_r0 = opaque_const(R0), c_r1 = opaque_const(R1);\n"
            "  const uint32_t c_r0s = opaque_const(R0 << %d), c_r1s = opaque_const(R1 << %d);\n"
            "  const uint32_t c_f0 = opaque_const(F0), c_f0s = opaque_const(F0 << %d);\n"
            "  asm(\n%s\n      : %s\n      : %s\n      : %s);\n}\n"
            % (name, sig, pre, lay.s, lay.s, lay.s, body, outs, ",\n        ".join(inl), clob)), len(ins), ntmp


def emit_fused(lay, name, spec, addend=None):
    """One asm block for a reduced sum of products (+ an addend): spec as in
    spec_terms with single-letter operand names that are also the C
    parameter names; a "sqr" entry's doubled limbs are formed outside the
    block."""
    n = lay.n
    ins, ntmp = gen_layout_terms(lay, lambda k: spec_terms(lay, k, spec), addend)
    body = "\n".join('      "%s\\n"' % s for s in ins)
    outs = ", ".join('[o%d] "=&v"(r.n[%d])' % (k, k) for k in range(n))
    params, inl, pre = [], [], ""
    for kind, x, y in spec:
        for v in (x,) if kind in ("sqr", "sqr3") else (x, y):
            if v not in params:
                params.append(v)
        if kind == "sqr":
            pre += "  uint32_t %s[%d];\n#pragma unroll\n  for (int i = 0; i < %d; i++) %s[i] = %s.n[i] << 1;\n" % (
                y, n - 1, n - 1, y, x)
            inl += ['[%s%d] "v"(%s[%d])' % (y, i, y, i) for i in range(n - 1)]
        if kind == "sqr3":
            pre += ("  uint32_t %sh[%d], %s[%d];\n#pragma unroll\n  for (int i = 0; i < %d; i++) %sh[i] = %s.n[i] * 3;\n"
                    "#pragma unroll\n  for (int i = 0; i < %d; i++) %s[i] = %sh[i] << 1;\n"
                    % (y, n, y, n - 1, n, y, x, n - 1, y, y))
            inl += ['[%s%d] "v"(%s[%d])' % (y, i, y, i) for i in range(n - 1)]
            inl += ['[%sh%d] "v"(%sh[%d])' % (y, i, y, i) for i in range(n)]
    if addend is not None:
        params.append(addend)
    inl = ['[%s%d] "v"(%s.n[%d])' % (v, i, v, i) for v in params for i in range(n)] + inl
    inl += ['[r0] "s"(c_r0)', '[r1] "s"(c_r1)', '[r0s] "s"(c_r0s)', '[r1s] "s"(c_r1s)', '[f0] "s"(c_f0)',
            '[f0s] "s"(c_f0s)']
    clob = ", ".join(['"vcc"'] + ['"v%d"' % (BASE + i) for i in range(ntmp)])
    sig = "fe& r, " + ", ".join("const fe& %s" % v for v in params)
    return ("__device__ __forceinline__ void %s(%s) {\n%s"
            "  const uint32_t c_r0 = opaque_const(R0), c_r1 = opaque_const(R1);\n"
            "  const uint32_t c_r0s = opaque_const(R0 << %d), c_r1s = opaque_const(R1 << %d);\n"
            "  const uint32_t c_f0 = opaque_const(F0), c_f0s = opaque_const(F0 << %d);\n"
            "  asm(\n%s\n      : %s\n      : %s\n      : %s);\n}\n"
            % (name, sig, pre, lay.s, lay.s, lay.s, body, outs, ",\n        ".join(inl), clob)), len(ins)


# Fused 9 x 29 operations (secp256k1_fe29.hpp): name, products, addend.
FUSED29 = [
    ("fe_mul2_asm", [("mul", "a", "b"), ("mul", "c", "e")], None),   # a b + c e
    ("fe_mulsqr_asm", [("mul", "a", "b"), ("sqr", "c", "g")], None),  # a b + c^2
    ("fe_mul_add_asm", [("mul", "a", "b")], "c"),                     # a b + c
    ("fe_sqr_add_asm", [("sqr", "a", "d")], "c"),                     # a^2 + c
    ("fe_sqr3_asm", [("sqr3", "a", "q")], None),                      # 3 a^2
]


def interleave(a, b):
    """Alternate two independent instruction streams (2-way ILP)."""
    out = []
    for i in range(max(len(a), len(b))):
        if i < len(a):
            out.append(a[i])
        if i < len(b):
            out.append(b[i])
    return out


# Register offsets of the pipelined schedule (gen_pipelined).
PH = [0, 2, 4, 6]               # rotating slots for H_0..H_7 (H_k in PH[k % 4])
PH8, PW, PACC, PACC2, PZ, PY = 8, 10, 12, 14, 16, 18
PNTMP = 20


def gen_pipelined(sqr):
    """Same arithmetic as gen(), scheduled for 2-way ILP with 20 temporaries:
    high column H_(k+1) is computed while low column k's chain runs (a low
    column k needs H_k, H_(k-1), H_(k-2) only, so four rotating H slots
    suffice); low columns 7..9, which have no H left to overlap with, split
    their products over two accumulators merged by one 64-bit add."""
    def mad(dst, x, y, acc):
        return "v_mad_u64_u32 %s, vcc, %s, %s, %s" % (dst, x, y, acc)

    def hslot(k):
        return PH8 if k == 8 else PH[k % 4]

    def hchain(m):
        terms = product_terms(10 + m, sqr)
        return [mad(pair(hslot(m)), x, y, "0" if d == 0 else pair(hslot(m))) for d, (x, y) in enumerate(terms)]

    ins = []
    # H8 (column 18) and top = hi(H8) (R1<<6) beside H0's chain
    a = hchain(8) + [mad(pair(PW), hi(PH8), "%[r1s]", "0")]
    ins += interleave(hchain(0), a)
    for k in range(10):
        fold = []
        if k < 9:
            fold.append((lo(hslot(k)), "%[r0]"))
        if k == 0:
            fold.append((lo(PW), "%[r0]"))
        if 1 <= k <= 9:
            fold += [(lo(hslot(k - 1)), "%[r1]"), (hi(hslot(k - 1)), "%[r0s]")]
        if k == 1:
            fold += [(lo(PW), "%[r1]"), (hi(PW), "%[r0s]")]
        if 2 <= k <= 9:
            fold.append((hi(hslot(k - 2)), "%[r1s]"))
        if k == 2:
            fold.append((hi(PW), "%[r1s]"))
        prods = product_terms(k, sqr)
        merge = []
        if k + 1 <= 7:
            terms_a, b = fold + prods, hchain(k + 1)
        else:
            # no H left to overlap: split this column over ACC and ACC2
            total = len(fold) + len(prods)
            nb = min(len(prods), total // 2)
            terms_a, terms_b = fold + prods[:len(prods) - nb], prods[len(prods) - nb:]
            b = [mad(pair(PACC2), x, y, "0" if d == 0 else pair(PACC2)) for d, (x, y) in enumerate(terms_b)]
            if b:
                merge = ["v_lshl_add_u64 %s, %s, 0, %s" % (pair(PACC), pair(PACC2), pair(PACC))]
        a = [mad(pair(PACC), x, y, "0" if (k == 0 and n == 0) else pair(PACC)) for n, (x, y) in enumerate(terms_a)]
        ins += interleave(a, b) + merge
        if k == 0:
            ins += ["v_and_b32 %s, %s, %s" % (lo(PZ), M26, lo(PACC)), "v_mov_b32 %s, 0" % hi(PZ)]
        elif k == 1:
            ins += ["v_and_b32 %s, %s, %s" % (lo(PY), M26, lo(PACC)), "v_mov_b32 %s, 0" % hi(PY)]
        elif k < 9:
            ins.append("v_and_b32 %%[o%d], %s, %s" % (k, M26, lo(PACC)))
        else:
            ins.append("v_and_b32 %%[o9], %s, %s" % (M22, lo(PACC)))
        ins.append("v_lshrrev_b64 %s, %d, %s" % (pair(PACC), 26 if k < 9 else 22, pair(PACC)))
    ulo, uhi = lo(PACC), hi(PACC)
    t = lo(PW)
    ins += [mad(pair(PZ), ulo, "%[f0]", pair(PZ)),
            "v_and_b32 %%[o0], %s, %s" % (M26, lo(PZ)),
            "v_alignbit_b32 %s, %s, %s, 26" % (t, hi(PZ), lo(PZ)),
            "v_add_u32 %s, %s, %s" % (lo(PY), lo(PY), t),
            mad(pair(PY), ulo, "64", pair(PY)),
            mad(pair(PY), uhi, "%[f0s]", pair(PY)),
            "v_and_b32 %%[o1], %s, %s" % (M26, lo(PY)),
            "v_alignbit_b32 %s, %s, %s, 26" % (t, hi(PY), lo(PY)),
            "v_lshl_add_u32 %s, %s, 12, %s" % (t, uhi, t),
            "v_add_u32 %%[o2], %%[o2], %s" % t]
    return ins


def emit(name, sqr, pipelined=False):
    ins = gen_pipelined(sqr) if pipelined else gen(sqr)
    ntmp = PNTMP if pipelined else NTMP
    body = "\n".join('      "%s\\n"' % s for s in ins)
    outs = ", ".join('[o%d] "=&v"(r.n[%d])' % (k, k) for k in range(10))
    if sqr:
        inl = ['[a%d] "v"(a.n[%d])' % (i, i) for i in range(10)] + ['[d%d] "v"(d[%d])' % (i, i) for i in range(9)]
    else:
        inl = ['[a%d] "v"(a.n[%d])' % (i, i) for i in range(10)] + ['[b%d] "v"(b.n[%d])' % (i, i) for i in range(10)]
    inl += ['[r0] "s"(c_r0)', '[r1] "s"(c_r1)', '[r0s] "s"(c_r0s)', '[r1s] "s"(c_r1s)', '[f0] "s"(c_f0)',
            '[f0s] "s"(c_f0s)']
    clob = ", ".join(['"vcc"'] + ['"v%d"' % (BASE + i) for i in range(ntmp)])
    sig = "fe& r, const fe& a" if sqr else "fe& r, const fe& a, const fe& b"
    pre = ""
    if sqr:
        pre = "  uint32_t d[9];\n#pragma unroll\n  for (int i = 0; i < 9; i++) d[i] = a.n[i] << 1;\n"
    return ("__device__ __forceinline__ void %s(%s) {\n%s"
            "  const uint32_t c_r0 = opaque_const(R0), c_r1 = opaque_const(R1);\n"
            "  const uint32_t c_r0s = opaque_const(R0 << 6), c_r1s = opaque_const(R1 << 6);\n"
            "  const uint32_t c_f0 = opaque_const(F0), c_f0s = opaque_const(F0 << 6);\n"
            "  asm(\n%s\n      : %s\n      : %s\n      : %s);\n}\n"
            % (name, sig, pre, body, outs, ",\n        ".join(inl), clob)), len(ins)


def main():
    mul, nm = emit("fe_mul_asm", False)
    sqr, ns = emit("fe_sqr_asm", True)
    pmul, pnm = emit("fe_mul_asm_p", False, True)
    psqr, pns = emit("fe_sqr_asm_p", True, True)
    # the layout-generic generator must reproduce the 10x26 serial blocks exactly
    assert emit_layout(L26, "fe_mul_asm", False)[0] == mul and emit_layout(L26, "fe_sqr_asm", True)[0] == sqr
    text = ("// GENERATED by tools/gen_fe_asm.py -- do not edit; regenerate and commit both.\n"
            "// Serial schedule (variant 3): fe_mul %d instructions, fe_sqr %d, temporaries v%d..v%d.\n"
            "// Pipelined schedule (variant 4): fe_mul %d, fe_sqr %d, temporaries v%d..v%d.\n"
            "// (fe_sqr: +9 doublings outside the block.)  vcc is clobbered by both.\n\n"
            % (nm, ns, BASE, BASE + NTMP - 1, pnm, pns, BASE, BASE + PNTMP - 1)) + mul + "\n" + sqr + "\n" + pmul + "\n" + psqr
    with open(OUT, "w") as f:
        f.write(text)
    print("wrote %s: serial mul %d / sqr %d, pipelined mul %d / sqr %d instructions" % (OUT, nm, ns, pnm, pns))
    m29, n29m, t29 = emit_layout(L29, "fe_mul_asm", False)
    s29, n29s, _ = emit_layout(L29, "fe_sqr_asm", True)
    fused = [emit_fused(L29, name, spec, add) for name, spec, add in FUSED29]
    text = ("// GENERATED by tools/gen_fe_asm.py -- do not edit; regenerate and commit both.\n"
            "// 9 x 29-bit limbs: fe_mul %d instructions, fe_sqr %d (+8 doublings outside the block),\n"
            "// fused: %s;\n"
            "// temporaries v%d..v%d and vcc (clobbered).\n\n"
            % (n29m, n29s, ", ".join("%s %d" % (f[0], c) for f, (_, c) in zip(FUSED29, fused)), BASE,
               BASE + t29 - 1)) + m29 + "\n" + s29 + "".join("\n" + t for t, _ in fused)
    with open(OUT29, "w") as f:
        f.write(text)
    print("wrote %s: mul %d / sqr %d instructions" % (OUT29, n29m, n29s))


if __name__ == "__main__":
    main()
