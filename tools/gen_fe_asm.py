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
    text = ("// GENERATED by tools/gen_fe_asm.py -- do not edit; regenerate and commit both.\n"
            "// Serial schedule (variant 3): fe_mul %d instructions, fe_sqr %d, temporaries v%d..v%d.\n"
            "// Pipelined schedule (variant 4): fe_mul %d, fe_sqr %d, temporaries v%d..v%d.\n"
            "// (fe_sqr: +9 doublings outside the block.)  vcc is clobbered by both.\n\n"
            % (nm, ns, BASE, BASE + NTMP - 1, pnm, pns, BASE, BASE + PNTMP - 1)) + mul + "\n" + sqr + "\n" + pmul + "\n" + psqr
    with open(OUT, "w") as f:
        f.write(text)
    print("wrote %s: serial mul %d / sqr %d, pipelined mul %d / sqr %d instructions" % (OUT, nm, ns, pnm, pns))


if __name__ == "__main__":
    main()
