// secp256k1 base-field arithmetic for gfx950, 9 x 29-bit limbs
// (CUDASP_FE_LIMBS=9; included by secp256k1_fe.hpp).
//
// Same scheme as the 10 x 26 layout (carry-free 64-bit v_mad_u64_u32 column
// chains, lazy additions, fold through each high column's 32-bit halves) with
// 81 instead of 100 limb products per multiplication (45 instead of 55 per
// square): 118 / 82 mads per mul / sqr against 143 / 98.  The price is
// headroom: a product column holds up to eight full 58-bit products, so
// operands must stay small (mag(a) * mag(b) <= 7) and the group formulas
// normalize more often (secp256k1_group29.hpp).
//
// Limbs 0..7 hold 29 bits, limb 8 the top 24 (bits 232..255).
// Magnitude m: limbs 0..7 <= m * 2^29 + 2^16, limb 8 <= m * 2^24 + 2^11.
//   mul/sqr: mag(a) * mag(b) <= 7 (sqr: mag(a) <= 2); output magnitude 1.
//            The widest column (7: eight products of full 29-bit limbs) stays
//            below 8 * 7.01 * 2^58 + 2^52 < 2^64 (mag product 8 overflows).
//   add: result <= 7 (32-bit limbs).
//   fe_sub<K>(r, a, b), fe_negate<K>: mag(b) <= K; add (K + 1) p, so the
//            result has magnitude mag(a) + K + 1 (<= 7).
#pragma once

namespace cudasp {

constexpr int FE_LIMBS = 9;
constexpr int FE_BITS = 29;

struct fe {
  uint32_t n[9];
};

constexpr uint32_t M29 = 0x1FFFFFFFu;
constexpr uint32_t M24 = 0xFFFFFFu;
// 2^261 mod p = 0x7A20 + 0x100 * 2^29
constexpr uint32_t R0 = 0x7A20u;
constexpr uint32_t R1 = 0x100u;
// 2^256 mod p = 0x3D1 + 0x8 * 2^29
constexpr uint32_t F0 = 0x3D1u;
constexpr uint32_t F1 = 0x8u;
constexpr uint32_t MUL_MAG_MAX = 7;
constexpr uint32_t SQR_MAG_MAX = 2;
constexpr uint32_t LIMB_MAG_MAX = 7;
// p in 9 x 29: 0x1FFFFC2F, 0x1FFFFFF7, 0x1FFFFFFF x 6, 0xFFFFFF
constexpr uint32_t P0 = 0x1FFFFC2Fu, P1 = 0x1FFFFFF7u;

#ifdef CUDASP_FE_CHECK
void fe_check_fail(const char* what, int limb, uint32_t v);
CUDASP_HD void fe_check_mag(const fe& a, uint32_t m, const char* what) {
  for (int i = 0; i < 8; i++)
    if ((uint64_t)a.n[i] > (uint64_t)m * (1ull << 29) + (1ull << 16)) fe_check_fail(what, i, a.n[i]);
  if ((uint64_t)a.n[8] > (uint64_t)m * (1ull << 24) + (1ull << 11)) fe_check_fail(what, 8, a.n[8]);
}
CUDASP_HD uint32_t fe_mag_of(const fe& a) {
  uint64_t m = 1;
  for (int i = 0; i < 8; i++)
    if (a.n[i] > (1u << 16)) {
      uint64_t need = ((uint64_t)a.n[i] - (1u << 16) + (1u << 29) - 1) >> 29;
      if (need > m) m = need;
    }
  if (a.n[8] > (1u << 11)) {
    uint64_t need = ((uint64_t)a.n[8] - (1u << 11) + (1u << 24) - 1) >> 24;
    if (need > m) m = need;
  }
  return (uint32_t)m;
}
CUDASP_HD void fe_check_mul(const fe& a, const fe& b, const char* what) {
  uint32_t ma = fe_mag_of(a), mb = fe_mag_of(b);
  if (ma > LIMB_MAG_MAX) fe_check_fail(what, -1, ma);
  if (mb > LIMB_MAG_MAX) fe_check_fail(what, -2, mb);
  if (ma * mb > MUL_MAG_MAX) fe_check_fail(what, -3, ma * mb);
}
CUDASP_HD void fe_check_mul2(const fe& a, const fe& b, const fe& c, const fe& e, const char* what) {
  uint32_t ma = fe_mag_of(a), mb = fe_mag_of(b), mc = fe_mag_of(c), me = fe_mag_of(e);
  if (ma > LIMB_MAG_MAX || mb > LIMB_MAG_MAX || mc > LIMB_MAG_MAX || me > LIMB_MAG_MAX) fe_check_fail(what, -1, ma);
  if (ma * mb + mc * me > MUL_MAG_MAX) fe_check_fail(what, -3, ma * mb + mc * me);
}
CUDASP_HD void fe_check_sqr(const fe& a, const char* what) {
  uint32_t ma = fe_mag_of(a);
  if (ma > SQR_MAG_MAX) fe_check_fail(what, -4, ma);
}
CUDASP_HD void fe_check_sum(const fe& a, const char* what) {
  uint32_t ma = fe_mag_of(a);
  if (ma > LIMB_MAG_MAX) fe_check_fail(what, -5, ma);
}
#define FE_CHECK(a, m, what) fe_check_mag(a, m, what)
#define FE_CHECK_MUL(a, b, what) fe_check_mul(a, b, what)
#define FE_CHECK_MUL2(a, b, c, e, what) fe_check_mul2(a, b, c, e, what)
#define FE_CHECK_SQR(a, what) fe_check_sqr(a, what)
#define FE_CHECK_SUM(a, what) fe_check_sum(a, what)
#else
#define FE_CHECK(a, m, what) ((void)0)
#define FE_CHECK_MUL(a, b, what) ((void)0)
#define FE_CHECK_MUL2(a, b, c, e, what) ((void)0)
#define FE_CHECK_SQR(a, what) ((void)0)
#define FE_CHECK_SUM(a, what) ((void)0)
#endif

CUDASP_HD void fe_from_u32x8(fe& r, const uint32_t w[8]) {
  r.n[0] = w[0] & M29;
  r.n[1] = ((w[0] >> 29) | (w[1] << 3)) & M29;
  r.n[2] = ((w[1] >> 26) | (w[2] << 6)) & M29;
  r.n[3] = ((w[2] >> 23) | (w[3] << 9)) & M29;
  r.n[4] = ((w[3] >> 20) | (w[4] << 12)) & M29;
  r.n[5] = ((w[4] >> 17) | (w[5] << 15)) & M29;
  r.n[6] = ((w[5] >> 14) | (w[6] << 18)) & M29;
  r.n[7] = ((w[6] >> 11) | (w[7] << 21)) & M29;
  r.n[8] = w[7] >> 8;
}

// Fully normalized 9 x 29 -> 8 little-endian u32 words.
CUDASP_HD void fe_to_u32x8(uint32_t w[8], const fe& a) {
  w[0] = a.n[0] | (a.n[1] << 29);
  w[1] = (a.n[1] >> 3) | (a.n[2] << 26);
  w[2] = (a.n[2] >> 6) | (a.n[3] << 23);
  w[3] = (a.n[3] >> 9) | (a.n[4] << 20);
  w[4] = (a.n[4] >> 12) | (a.n[5] << 17);
  w[5] = (a.n[5] >> 15) | (a.n[6] << 14);
  w[6] = (a.n[6] >> 18) | (a.n[7] << 11);
  w[7] = (a.n[7] >> 21) | (a.n[8] << 8);
}

CUDASP_HD void fe_add(fe& r, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < 9; i++) r.n[i] = a.n[i] + b.n[i];
  FE_CHECK_SUM(r, "add");
}

// r = 2 (a + b): one v_add_lshl_u32 per limb.
CUDASP_HD void fe_add_x2(fe& r, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < 9; i++) r.n[i] = (a.n[i] + b.n[i]) << 1;
  FE_CHECK_SUM(r, "add_x2");
}

CUDASP_HD void fe_add_to(fe& r, const fe& a) {
#pragma unroll
  for (int i = 0; i < 9; i++) r.n[i] += a.n[i];
  FE_CHECK_SUM(r, "add_to");
}

CUDASP_HD void fe_mul_int(fe& r, const fe& a, uint32_t k) {
#pragma unroll
  for (int i = 0; i < 9; i++) r.n[i] = a.n[i] * k;
  FE_CHECK_SUM(r, "mul_int");
}

// r = (K + 1) p - a with mag(a) <= K; mag(r) <= K + 1.
template <uint32_t K>
CUDASP_HD void fe_negate(fe& r, const fe& a) {
  static_assert(K + 1 <= LIMB_MAG_MAX, "fe_negate magnitude");
  FE_CHECK(a, K, "negate");
  r.n[0] = P0 * (K + 1) - a.n[0];
  r.n[1] = P1 * (K + 1) - a.n[1];
#pragma unroll
  for (int i = 2; i < 8; i++) r.n[i] = M29 * (K + 1) - a.n[i];
  r.n[8] = M24 * (K + 1) - a.n[8];
}

// r = a - b with mag(b) <= K: r = a + ((K + 1) p - b); mag(r) <= mag(a) + K + 1.
template <uint32_t K>
CUDASP_HD void fe_sub(fe& r, const fe& a, const fe& b) {
  FE_CHECK(b, K, "sub");
  r.n[0] = a.n[0] + (P0 * (K + 1) - b.n[0]);
  r.n[1] = a.n[1] + (P1 * (K + 1) - b.n[1]);
#pragma unroll
  for (int i = 2; i < 8; i++) r.n[i] = a.n[i] + (M29 * (K + 1) - b.n[i]);
  r.n[8] = a.n[8] + (M24 * (K + 1) - b.n[8]);
  FE_CHECK_SUM(r, "sub");
}

#ifndef CUDASP_NORM_PAR
#define CUDASP_NORM_PAR 0
#endif

// Carry-propagate and fold the bits above 2^256 once (inputs of magnitude
// <= 7).  Output magnitude 1.  Serial form: limbs 0..7 < 2^29.  Parallel form
// (CUDASP_NORM_PAR): every limb keeps its low bits plus the carry of the limb
// below (<= 7, or 7 * 0x3D1 into limb 0), so the result is within magnitude
// 1's slack (limbs <= 2^29 + 2^13) and the nine carries are independent.
CUDASP_HD void fe_normalize_weak(fe& r) {
  FE_CHECK_SUM(r, "normalize_weak");
#if CUDASP_NORM_PAR
  {
    uint32_t c[9];
#pragma unroll
    for (int i = 0; i < 8; i++) c[i] = r.n[i] >> 29;
    c[8] = r.n[8] >> 24;
    r.n[0] = (r.n[0] & M29) + c[8] * F0;
    r.n[1] = (r.n[1] & M29) + c[0] + (c[8] << 3);
#pragma unroll
    for (int i = 2; i < 8; i++) r.n[i] = (r.n[i] & M29) + c[i - 1];
    r.n[8] = (r.n[8] & M24) + c[7];
    return;
  }
#endif
  uint32_t t[9];
#pragma unroll
  for (int i = 0; i < 9; i++) t[i] = r.n[i];
  uint32_t x = t[8] >> 24;
  t[8] &= M24;
  t[0] += x * F0;
  t[1] += x << 3;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    t[i + 1] += t[i] >> 29;
    t[i] &= M29;
  }
#pragma unroll
  for (int i = 0; i < 9; i++) r.n[i] = t[i];
}

// Serial carry propagation (limbs 0..7 < 2^29 afterwards).
CUDASP_HD void fe_normalize_weak_serial(fe& r) {
  uint32_t t[9];
#pragma unroll
  for (int i = 0; i < 9; i++) t[i] = r.n[i];
  uint32_t x = t[8] >> 24;
  t[8] &= M24;
  t[0] += x * F0;
  t[1] += x << 3;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    t[i + 1] += t[i] >> 29;
    t[i] &= M29;
  }
#pragma unroll
  for (int i = 0; i < 9; i++) r.n[i] = t[i];
}

// Full normalization to the canonical representative in [0, p).
CUDASP_HD void fe_normalize(fe& r) {
  FE_CHECK_SUM(r, "normalize");
  fe_normalize_weak_serial(r);
  fe_normalize_weak_serial(r);
  // r >= p  <=>  r + 0x1000003D1 >= 2^256.
  uint32_t t[9];
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    uint32_t add = i == 0 ? F0 : (i == 1 ? F1 : 0);
    t[i] = r.n[i] + add + c;
    c = i < 8 ? t[i] >> 29 : 0;
  }
  if ((t[8] >> 24) != 0) {
#pragma unroll
    for (int i = 0; i < 8; i++) r.n[i] = t[i] & M29;
    r.n[8] = t[8] & M24;
  }
}

// r = a / 2 mod p (a of magnitude m <= 5; result <= (m + 2) / 2, i.e. 3 for
// m <= 4): a (made even by adding p when odd) shifted right by one bit.
CUDASP_HD void fe_half(fe& r, const fe& a) {
  const uint32_t odd = 0u - (a.n[0] & 1u);
  uint32_t t[9];
  t[0] = a.n[0] + (P0 & odd);
  t[1] = a.n[1] + (P1 & odd);
#pragma unroll
  for (int i = 2; i < 8; i++) t[i] = a.n[i] + (M29 & odd);
  t[8] = a.n[8] + (M24 & odd);
  // (t_i + (t_(i+1) mod 2) 2^29) / 2 = (t_i >> 1) + (t_(i+1) mod 2) 2^28 (2^29 is
  // even): and, shift, shift-add (v_lshl_add_u32) per limb.
#pragma unroll
  for (int i = 0; i < 8; i++) {
#if defined(__HIP_DEVICE_COMPILE__)
    // 3 instructions (the compiler turns (x & 1) << 28 into a shift and a
    // mask and does not form the shift-add: 4)
    uint32_t b, h;
    asm("v_and_b32 %0, 1, %2\n"
        "v_lshrrev_b32 %1, 1, %3\n"
        "v_lshl_add_u32 %1, %0, 28, %1"
        : "=&v"(b), "=&v"(h)
        : "v"(t[i + 1]), "v"(t[i]));
    r.n[i] = h;
#else
    r.n[i] = (t[i] >> 1) + ((t[i + 1] & 1u) << 28);
#endif
  }
  r.n[8] = t[8] >> 1;
}

// ---------------------------------------------------------------- mul / sqr
// Same column/fold structure as the 10 x 26 variant 1 (secp256k1_fe.hpp);
// on the device the generated asm blocks of secp256k1_fe29_asm.inc.
CUDASP_HD void fe29_reduce_columns(fe& r, const uint64_t c[17]) {
  uint64_t t[10];
#pragma unroll
  for (int k = 0; k < 9; k++) t[k] = c[k];
  t[9] = 0;
#pragma unroll
  for (int m = 0; m < 8; m++) {  // column 9 + m, weight 2^(261 + 29 m)
    uint32_t lo = (uint32_t)c[9 + m], hi = (uint32_t)(c[9 + m] >> 32);
    t[m] += (uint64_t)lo * R0;
    t[m + 1] += (uint64_t)lo * R1 + (uint64_t)hi * (R0 << 3);
    t[m + 2] += (uint64_t)hi * (R1 << 3);
  }
  {  // t[9] (weight 2^261 again) < 2^32 for the magnitudes allowed
    uint32_t lo = (uint32_t)t[9], hi = (uint32_t)(t[9] >> 32);
    t[0] += (uint64_t)lo * R0;
    t[1] += (uint64_t)lo * R1 + (uint64_t)hi * (R0 << 3);
    t[2] += (uint64_t)hi * (R1 << 3);
  }
  uint32_t o[9];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    o[k] = (uint32_t)t[k] & M29;
    t[k + 1] += t[k] >> 29;
  }
  o[8] = (uint32_t)t[8] & M24;
  uint64_t u = t[8] >> 24;
  uint32_t ulo = (uint32_t)u, uhi = (uint32_t)(u >> 32);
  uint64_t s0 = (uint64_t)o[0] + (uint64_t)ulo * F0;
  uint64_t s1 = (uint64_t)o[1] + (uint64_t)ulo * F1 + (uint64_t)uhi * (F0 << 3) + (s0 >> 29);
  uint64_t s2 = (uint64_t)o[2] + (uint64_t)uhi * (F1 << 3) + (s1 >> 29);
  r.n[0] = (uint32_t)s0 & M29;
  r.n[1] = (uint32_t)s1 & M29;
  r.n[2] = (uint32_t)s2;
#pragma unroll
  for (int k = 3; k < 9; k++) r.n[k] = o[k];
}

// Product columns, accumulated into c[0..16].
CUDASP_HD void fe29_mul_columns(uint64_t c[17], const fe& a, const fe& b) {
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = 0; i < 9; i++) {
      int j = k - i;
      if (j >= 0 && j < 9) c[k] += (uint64_t)a.n[i] * b.n[j];
    }
  }
}

CUDASP_HD void fe29_sqr_columns(uint64_t c[17], const fe& a) {
  uint32_t a2[9];
#pragma unroll
  for (int i = 0; i < 9; i++) a2[i] = a.n[i] * 2;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = 0; i < 9; i++) {
      int j = k - i;
      if (j > i && j < 9) c[k] += (uint64_t)a2[i] * a.n[j];
      else if (j == i) c[k] += (uint64_t)a.n[i] * a.n[i];
    }
  }
}

CUDASP_HD void fe29_add_columns(uint64_t c[17], const fe& a) {
#pragma unroll
  for (int k = 0; k < 9; k++) c[k] += a.n[k];
}

CUDASP_HD void fe_mul_c(fe& r, const fe& a, const fe& b) {
  uint64_t c[17] = {};
  fe29_mul_columns(c, a, b);
  fe29_reduce_columns(r, c);
}

CUDASP_HD void fe_sqr_c(fe& r, const fe& a) {
  uint64_t c[17] = {};
  fe29_sqr_columns(c, a);
  fe29_reduce_columns(r, c);
}

#if defined(__HIP_DEVICE_COMPILE__)
#include "secp256k1_fe29_asm.inc"
#endif

CUDASP_HD void fe_mul(fe& r, const fe& a, const fe& b) {
  FE_CHECK_MUL(a, b, "mul");
#if defined(__HIP_DEVICE_COMPILE__)
  fe_mul_asm(r, a, b);
#else
  fe_mul_c(r, a, b);
#endif
}

CUDASP_HD void fe_sqr(fe& r, const fe& a) {
  FE_CHECK_SQR(a, "sqr");
#if defined(__HIP_DEVICE_COMPILE__)
  fe_sqr_asm(r, a);
#else
  fe_sqr_c(r, a);
#endif
}

// ------------------------------------------------------------ fused forms
// One reduction for a sum of products (+ an addend): the columns of every
// term are summed before the fold, so the reduction (37 of a mul's 118 mads)
// and the carry chain are paid once, and the result has magnitude 1 without
// a separate normalization.  The column budget is shared: the operands'
// magnitude products sum to <= 7 (an addend of magnitude <= 7 adds < 2^32 to
// a low column, well inside the slack).

// r = a b + c e
CUDASP_HD void fe_mul2(fe& r, const fe& a, const fe& b, const fe& c, const fe& e) {
  FE_CHECK_MUL2(a, b, c, e, "mul2");
#if defined(__HIP_DEVICE_COMPILE__)
  fe_mul2_asm(r, a, b, c, e);
#else
  uint64_t col[17] = {};
  fe29_mul_columns(col, a, b);
  fe29_mul_columns(col, c, e);
  fe29_reduce_columns(r, col);
#endif
}

// r = a b + c^2
CUDASP_HD void fe_mulsqr(fe& r, const fe& a, const fe& b, const fe& c) {
  FE_CHECK_MUL2(a, b, c, c, "mulsqr");
#if defined(__HIP_DEVICE_COMPILE__)
  fe_mulsqr_asm(r, a, b, c);
#else
  uint64_t col[17] = {};
  fe29_mul_columns(col, a, b);
  fe29_sqr_columns(col, c);
  fe29_reduce_columns(r, col);
#endif
}

// r = 3 a^2 (mag(a) <= 1: the columns of 3 a^2 fit like a product of
// magnitude 3); the squares' operand is 3 a, the cross products' 6 a.
CUDASP_HD void fe_sqr3(fe& r, const fe& a) {
  FE_CHECK_MUL2(a, a, a, a, "sqr3");  // 2 m^2 <= 7 <=> m = 1 (3 m^2 <= 7)
#if defined(__HIP_DEVICE_COMPILE__)
  fe_sqr3_asm(r, a);
#else
  uint64_t col[17] = {};
  fe29_sqr_columns(col, a);
#pragma unroll
  for (int k = 0; k < 17; k++) col[k] *= 3;
  fe29_reduce_columns(r, col);
#endif
}

// r = a b + c
CUDASP_HD void fe_mul_add(fe& r, const fe& a, const fe& b, const fe& c) {
  FE_CHECK_MUL(a, b, "mul_add");
  FE_CHECK_SUM(c, "mul_add addend");
#if defined(__HIP_DEVICE_COMPILE__)
  fe_mul_add_asm(r, a, b, c);
#else
  uint64_t col[17] = {};
  fe29_mul_columns(col, a, b);
  fe29_add_columns(col, c);
  fe29_reduce_columns(r, col);
#endif
}

// r = a^2 + c
CUDASP_HD void fe_sqr_add(fe& r, const fe& a, const fe& c) {
  FE_CHECK_SQR(a, "sqr_add");
  FE_CHECK_SUM(c, "sqr_add addend");
#if defined(__HIP_DEVICE_COMPILE__)
  fe_sqr_add_asm(r, a, c);
#else
  uint64_t col[17] = {};
  fe29_sqr_columns(col, a);
  fe29_add_columns(col, c);
  fe29_reduce_columns(r, col);
#endif
}

}  // namespace cudasp
