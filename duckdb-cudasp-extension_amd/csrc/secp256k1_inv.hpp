// Constant-time modular inversion mod p by Bernstein-Yang "safegcd"
// divsteps (half-delta variant, 20 x 30 = 600 >= 590 divsteps, enough for any
// 256-bit input), on signed 30-bit limbs.  Replaces the Fermat chain
// (255 squarings + 15 multiplications, ~48k VALU instructions) at about a
// third of the cost; uniform control flow, so no divergence across a wave.
//
// State: f = p, g = x, d = 0, e = 1 with f = d x, g = e x (mod p).  Each
// round runs 30 divsteps on the low 30 bits of f and g to get the transition
// matrix T (entries bounded by 2^30), then [f g] <- T [f g] / 2^30 exactly and
// [d e] <- T [d e] / 2^30 mod p.  At the end g = 0, f = +-1, 1/x = d f.
// The half-delta divstep is tracked as zeta = -(delta + 1/2) (starts at -1,
// delta > 0 iff zeta < 0):
//   delta > 0 and g odd:  zeta <- -zeta - 2,  (f, g) <- (g, (g - f)/2)
//   g odd:                zeta <- zeta - 1,   g <- (g + f)/2
//   otherwise:            zeta <- zeta - 1,   g <- g/2
#pragma once
#include "secp256k1_fe.hpp"

namespace cudasp {

struct s30 {
  int32_t v[9];
};

constexpr int32_t S30_MASK = 0x3FFFFFFF;
// p in signed 30-bit limbs: p = -977 - 4*2^30 + 65536*2^240.
constexpr int32_t P30_0 = -977;
constexpr int32_t P30_1 = -4;
constexpr int32_t P30_8 = 65536;
constexpr uint32_t P_INV30 = 0x2DDACACFu;  // p^-1 mod 2^30

// a + b + c as one v_add3_u32.  In plain C the compiler rewrites
// x + (m & 1) for a 0 / -1 mask m into x - m and then needs a separate sub.
CUDASP_HD uint32_t add3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
#else
  return a + b + c;
#endif
}

// 30 divsteps on the low bits; returns the new zeta and the matrix (scaled by
// 2^30).  Per step: g += odd ? (swap ? -f : f) : 0 is written as
// g + ((f ^ swap) & odd) + (swap & 1) -- one 3-input bit operation and one
// 3-input add on gfx950 (v_bitop3_b32, v_add3_u32) instead of xor, sub, and,
// add -- and the zeta update (zeta ^ swap) - 1 is one v_xad_u32.
CUDASP_HD int32_t divsteps_30(int32_t zeta, uint32_t f, uint32_t g, int32_t& tu, int32_t& tv, int32_t& tq,
                              int32_t& tr) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  uint32_t z = (uint32_t)zeta;
#pragma unroll
  for (int i = 0; i < 30; i++) {
    const uint32_t m_pos = (uint32_t)((int32_t)z >> 31);  // all ones iff delta > 0
    const uint32_t m_odd = 0u - (g & 1u);
    const uint32_t m_swap = m_odd & m_pos;
    const uint32_t n_swap = m_swap & 1u;  // -m_swap
    g = add3(g, (f ^ m_swap) & m_odd, n_swap);
    q = add3(q, (u ^ m_swap) & m_odd, n_swap);
    r = add3(r, (v ^ m_swap) & m_odd, n_swap);
    z = (z ^ m_swap) - 1u;
    f += g & m_swap;  // swap: f <- old g (= new g + f)
    u = (u + (q & m_swap)) << 1;
    v = (v + (r & m_swap)) << 1;
    g >>= 1;
  }
  tu = (int32_t)u;
  tv = (int32_t)v;
  tq = (int32_t)q;
  tr = (int32_t)r;
  return (int32_t)z;
}

// c + a * b (signed 32 x 32 -> 64) as one v_mad_i64_i32.  Compiled C builds
// these sums from unsigned 64-bit multiplies with sign corrections (about 3x
// the instructions).
CUDASP_HD int64_t mad_i64(int32_t a, int32_t b, int64_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  int64_t r;
  uint64_t carry;  // unused carry-out; its own SGPR pair, no vcc hazards
  asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(carry) : "v"(a), "v"(b), "v"(c));
  return r;
#else
  return c + (int64_t)a * b;
#endif
}

// cf += u a + v b and cg += q a + r b: the four mads of one limb of a matrix
// update in one asm block (separate asm statements each get an s_nop).
CUDASP_HD void mad_2x2(int64_t& cf, int64_t& cg, int32_t u, int32_t v, int32_t q, int32_t r, int32_t a, int32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t carry;
  asm("v_mad_i64_i32 %0, %2, %3, %7, %0\n\t"
      "v_mad_i64_i32 %1, %2, %5, %7, %1\n\t"
      "v_mad_i64_i32 %0, %2, %4, %8, %0\n\t"
      "v_mad_i64_i32 %1, %2, %6, %8, %1"
      : "+v"(cf), "+v"(cg), "=s"(carry)
      : "v"(u), "v"(v), "v"(q), "v"(r), "v"(a), "v"(b));
#else
  cf += (int64_t)u * a + (int64_t)v * b;
  cg += (int64_t)q * a + (int64_t)r * b;
#endif
}

// cd += P md and ce += P me (P a constant limb of p) in one asm block.
CUDASP_HD void mad_p2(int64_t& cd, int64_t& ce, int32_t P, int32_t md, int32_t me) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t carry;
  asm("v_mad_i64_i32 %0, %2, %3, %4, %0\n\t"
      "v_mad_i64_i32 %1, %2, %3, %5, %1"
      : "+v"(cd), "+v"(ce), "=s"(carry)
      : "v"(P), "v"(md), "v"(me));
#else
  cd += (int64_t)P * md;
  ce += (int64_t)P * me;
#endif
}

// [f g] <- T [f g] / 2^30 (exact).
CUDASP_HD void s30_update_fg(s30& f, s30& g, int32_t u, int32_t v, int32_t q, int32_t r) {
  int64_t cf = 0, cg = 0;
  mad_2x2(cf, cg, u, v, q, r, f.v[0], g.v[0]);
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    mad_2x2(cf, cg, u, v, q, r, f.v[i], g.v[i]);
    f.v[i - 1] = (int32_t)cf & S30_MASK;
    g.v[i - 1] = (int32_t)cg & S30_MASK;
    cf >>= 30;
    cg >>= 30;
  }
  f.v[8] = (int32_t)cf;
  g.v[8] = (int32_t)cg;
}

// [d e] <- T [d e] / 2^30 mod p, keeping -2p < d, e < p.
CUDASP_HD void s30_update_de(s30& d, s30& e, int32_t u, int32_t v, int32_t q, int32_t r) {
  const int32_t sd = d.v[8] >> 31, se = e.v[8] >> 31;
  // Work with d + p (if d < 0) and e + p (if e < 0) so the result stays in range.
  int32_t md = (u & sd) + (v & se);
  int32_t me = (q & sd) + (r & se);
  int64_t cd = 0, ce = 0;
  mad_2x2(cd, ce, u, v, q, r, d.v[0], e.v[0]);
  // Pick md, me so that the low 30 bits cancel.
  md -= (int32_t)((P_INV30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)S30_MASK);
  me -= (int32_t)((P_INV30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)S30_MASK);
  mad_p2(cd, ce, P30_0, md, me);
  cd >>= 30;
  ce >>= 30;
  // limb 1 (p has -4 there)
  mad_2x2(cd, ce, u, v, q, r, d.v[1], e.v[1]);
  mad_p2(cd, ce, P30_1, md, me);
  d.v[0] = (int32_t)cd & S30_MASK;
  e.v[0] = (int32_t)ce & S30_MASK;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 2; i < 8; i++) {
    mad_2x2(cd, ce, u, v, q, r, d.v[i], e.v[i]);
    d.v[i - 1] = (int32_t)cd & S30_MASK;
    e.v[i - 1] = (int32_t)ce & S30_MASK;
    cd >>= 30;
    ce >>= 30;
  }
  mad_2x2(cd, ce, u, v, q, r, d.v[8], e.v[8]);
  mad_p2(cd, ce, P30_8, md, me);
  d.v[7] = (int32_t)cd & S30_MASK;
  e.v[7] = (int32_t)ce & S30_MASK;
  cd >>= 30;
  ce >>= 30;
  d.v[8] = (int32_t)cd;
  e.v[8] = (int32_t)ce;
}

// 8 LE u32 words (< 2^256) -> signed30.
CUDASP_HD void s30_from_words(s30& r, const uint32_t w[8]) {
  r.v[0] = (int32_t)(w[0] & 0x3FFFFFFFu);
  r.v[1] = (int32_t)(((w[0] >> 30) | (w[1] << 2)) & 0x3FFFFFFFu);
  r.v[2] = (int32_t)(((w[1] >> 28) | (w[2] << 4)) & 0x3FFFFFFFu);
  r.v[3] = (int32_t)(((w[2] >> 26) | (w[3] << 6)) & 0x3FFFFFFFu);
  r.v[4] = (int32_t)(((w[3] >> 24) | (w[4] << 8)) & 0x3FFFFFFFu);
  r.v[5] = (int32_t)(((w[4] >> 22) | (w[5] << 10)) & 0x3FFFFFFFu);
  r.v[6] = (int32_t)(((w[5] >> 20) | (w[6] << 12)) & 0x3FFFFFFFu);
  r.v[7] = (int32_t)(((w[6] >> 18) | (w[7] << 14)) & 0x3FFFFFFFu);
  r.v[8] = (int32_t)(w[7] >> 16);
}

// r = a^-1 mod p (a != 0 mod p; a = 0 gives 0).  Input any weak fe; output
// fully normalized.
CUDASP_HD void fe_inv_safegcd(fe& r, const fe& a_in) {
  fe a = a_in;
  fe_normalize(a);
  uint32_t w[8];
  fe_to_u32x8(w, a);
  s30 f, g, d, e;
  f.v[0] = P30_0;
  f.v[1] = P30_1;
#pragma unroll
  for (int i = 2; i < 8; i++) f.v[i] = 0;
  f.v[8] = P30_8;
  s30_from_words(g, w);
#pragma unroll
  for (int i = 0; i < 9; i++) {
    d.v[i] = 0;
    e.v[i] = 0;
  }
  e.v[0] = 1;
  int32_t zeta = -1;  // delta = 1/2
#pragma unroll 1
  for (int it = 0; it < 20; it++) {
    int32_t u, v, q, rr;
    zeta = divsteps_30(zeta, (uint32_t)f.v[0], (uint32_t)g.v[0], u, v, q, rr);
    s30_update_de(d, e, u, v, q, rr);
    s30_update_fg(f, g, u, v, q, rr);
  }
  // f = +-1: 1/a = d * f.  d is in (-2p, p); negate if f < 0, then add 2p so
  // the value is in (0, 4p) and carry into 30-bit limbs.
  const int32_t sf = f.v[8] >> 31;  // -1 if f < 0
  int64_t c = 0;
  int32_t t[9];
#pragma unroll
  for (int i = 0; i < 9; i++) {
    int32_t di = (d.v[i] ^ sf) - sf;
    int32_t pi = i == 0 ? P30_0 : (i == 1 ? P30_1 : (i == 8 ? P30_8 : 0));
    c += (int64_t)di + 2 * (int64_t)pi;
    t[i] = (int32_t)c & S30_MASK;
    c >>= 30;
  }
  // Value = sum t[i] 2^(30 i) + c * 2^270, in (0, 4p): c == 0 and t[8] < 2^18.
  uint32_t lo[8];
  lo[0] = (uint32_t)t[0] | ((uint32_t)t[1] << 30);
  lo[1] = ((uint32_t)t[1] >> 2) | ((uint32_t)t[2] << 28);
  lo[2] = ((uint32_t)t[2] >> 4) | ((uint32_t)t[3] << 26);
  lo[3] = ((uint32_t)t[3] >> 6) | ((uint32_t)t[4] << 24);
  lo[4] = ((uint32_t)t[4] >> 8) | ((uint32_t)t[5] << 22);
  lo[5] = ((uint32_t)t[5] >> 10) | ((uint32_t)t[6] << 20);
  lo[6] = ((uint32_t)t[6] >> 12) | ((uint32_t)t[7] << 18);
  lo[7] = ((uint32_t)t[7] >> 14) | ((uint32_t)t[8] << 16);
  uint32_t hi = (uint32_t)t[8] >> 16;  // bits 256.. (< 4)
  fe_from_u32x8(r, lo);
  // + hi * 2^256 = hi * (F0 + F1 * 2^26)
  r.n[0] += hi * F0;
  r.n[1] += hi * F1;
  fe_normalize(r);
}

}  // namespace cudasp
