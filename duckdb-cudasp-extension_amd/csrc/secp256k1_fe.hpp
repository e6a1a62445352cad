// secp256k1 base-field arithmetic for gfx950, 10 x 26-bit limbs.
//
// Why 10x26 and not 8x32 Montgomery (the reference's gECC layout, see
// /root/reference/src/cudasp_gpu.cu:18 "u32 ... MONTFLAG::SOS"): on gfx950
// v_mad_u64_u32 issues at the full VOP3 rate (tools/microbench, measured
// 60 lane-ops/CU/clk, same as v_add3_u32), while a carry-propagating 8x32
// product needs a v_addc with an SGPR carry-in after every mad (measured 1.4x
// the cost of a mad).  With 26-bit limbs a whole product column accumulates in
// one 64-bit register through a mad chain with no carries at all, additions are
// lazy (no carry chain), and p = 2^256 - 0x1000003D1 folds with two small
// constants.  Values are kept in plain (non-Montgomery) form, so conversions to
// and from the reference's byte layout are shifts only.
//
// Magnitude convention (checked by the host emulation build, see
// CUDASP_FE_CHECK): a value has magnitude m when limbs 0..8 are <= m*2^26 and
// limb 9 <= m*2^22 (plus a 2^23 / 2^13 slack so that the "weak" outputs of
// mul/sqr/normalize_weak, whose limbs may exceed 2^26 by a carry, count as 1).
// mul/sqr accept mag(a) * mag(b) <= MUL_MAG_MAX with each <= 31 and return
// m = 1: the widest product column (column 9: eight full limb products plus
// two with limb 9) stays below 8 * 408 * 2^52 + 2^52 < 2^64.  fe_add adds
// magnitudes; fe_sub<K>(r, a, b) and fe_negate<K> need mag(b) <= K and add 2K.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CUDASP_HD __host__ __device__ __forceinline__

// Limb layout: 9 x 29 bits (secp256k1_fe29.hpp, default: 118 / 82 mads per
// mul / sqr) or 10 x 26 bits (this file: 143 / 98, more headroom).  A/B on
// MI355X: profiles/r01_stage_ab_fe_layouts.txt.
#ifndef CUDASP_FE_LIMBS
#define CUDASP_FE_LIMBS 9
#endif

namespace cudasp {
// Small constants as opaque scalar registers on the device, so that the
// compiler keeps "x * 0x400" as one v_mad_u64_u32 instead of rewriting it as a
// 64-bit shift + add (two VOP3 instructions).
CUDASP_HD uint32_t opaque_const(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("s_mov_b32 %0, %1" : "=s"(r) : "i"(v));
  return r;
#else
  return v;
#endif
}

}  // namespace cudasp

#if CUDASP_FE_LIMBS == 9
#include "secp256k1_fe29.hpp"
#elif CUDASP_FE_LIMBS == 10
namespace cudasp {

constexpr int FE_LIMBS = 10;
constexpr int FE_BITS = 26;

struct fe {
  uint32_t n[10];
};

constexpr uint32_t M26 = 0x3FFFFFFu;
constexpr uint32_t M22 = 0x3FFFFFu;
// 2^260 mod p = 0x3D10 + 0x400 * 2^26
constexpr uint32_t R0 = 0x3D10u;
constexpr uint32_t R1 = 0x400u;
// 2^256 mod p = 0x3D1 + 0x40 * 2^26
constexpr uint32_t F0 = 0x3D1u;
constexpr uint32_t F1 = 0x40u;
constexpr uint32_t MUL_MAG_MAX = 400;
constexpr uint32_t SQR_MAG_MAX = 20;
constexpr uint32_t LIMB_MAG_MAX = 31;

#ifdef CUDASP_FE_CHECK
// Host-emulation builds verify every magnitude precondition.
void fe_check_fail(const char* what, int limb, uint32_t v);
CUDASP_HD void fe_check_mag(const fe& a, uint32_t m, const char* what) {
  for (int i = 0; i < 9; i++)
    if ((uint64_t)a.n[i] > (uint64_t)m * (1ull << 26) + (1ull << 23)) fe_check_fail(what, i, a.n[i]);
  if ((uint64_t)a.n[9] > (uint64_t)m * (1ull << 22) + (1ull << 13)) fe_check_fail(what, 9, a.n[9]);
}
// Smallest magnitude m that a's limbs satisfy.
CUDASP_HD uint32_t fe_mag_of(const fe& a) {
  uint64_t m = 1;
  for (int i = 0; i < 9; i++)
    if (a.n[i] > (1u << 23)) {
      uint64_t need = ((uint64_t)a.n[i] - (1u << 23) + (1u << 26) - 1) >> 26;
      if (need > m) m = need;
    }
  if (a.n[9] > (1u << 13)) {
    uint64_t need = ((uint64_t)a.n[9] - (1u << 13) + (1u << 22) - 1) >> 22;
    if (need > m) m = need;
  }
  return (uint32_t)m;
}
CUDASP_HD void fe_check_mul(const fe& a, const fe& b, const char* what) {
  uint32_t ma = fe_mag_of(a), mb = fe_mag_of(b);
  if (ma > 31) fe_check_fail(what, -1, ma);
  if (mb > 31) fe_check_fail(what, -2, mb);
  if (ma * mb > MUL_MAG_MAX) fe_check_fail(what, -3, ma * mb);
}
#define FE_CHECK(a, m, what) fe_check_mag(a, m, what)
#define FE_CHECK_MUL(a, b, what) fe_check_mul(a, b, what)
#else
#define FE_CHECK(a, m, what) ((void)0)
#define FE_CHECK_MUL(a, b, what) ((void)0)
#endif
#define FE_CHECK_SQR(a, what) FE_CHECK_MUL(a, a, what)
#define FE_CHECK_SUM(a, what) ((void)0)

// 8 little-endian u32 words (the reference's limb layout,
// src/cudasp_extension.cu:59-85) -> 10x26.  Input must be < 2^256.
CUDASP_HD void fe_from_u32x8(fe& r, const uint32_t w[8]) {
  r.n[0] = w[0] & M26;
  r.n[1] = ((w[0] >> 26) | (w[1] << 6)) & M26;
  r.n[2] = ((w[1] >> 20) | (w[2] << 12)) & M26;
  r.n[3] = ((w[2] >> 14) | (w[3] << 18)) & M26;
  r.n[4] = ((w[3] >> 8) | (w[4] << 24)) & M26;
  r.n[5] = (w[4] >> 2) & M26;
  r.n[6] = ((w[4] >> 28) | (w[5] << 4)) & M26;
  r.n[7] = ((w[5] >> 22) | (w[6] << 10)) & M26;
  r.n[8] = ((w[6] >> 16) | (w[7] << 16)) & M26;
  r.n[9] = w[7] >> 10;
}

// Fully normalized 10x26 -> 8 little-endian u32 words.
CUDASP_HD void fe_to_u32x8(uint32_t w[8], const fe& a) {
  w[0] = a.n[0] | (a.n[1] << 26);
  w[1] = (a.n[1] >> 6) | (a.n[2] << 20);
  w[2] = (a.n[2] >> 12) | (a.n[3] << 14);
  w[3] = (a.n[3] >> 18) | (a.n[4] << 8);
  w[4] = (a.n[4] >> 24) | (a.n[5] << 2) | (a.n[6] << 28);
  w[5] = (a.n[6] >> 4) | (a.n[7] << 22);
  w[6] = (a.n[7] >> 10) | (a.n[8] << 16);
  w[7] = (a.n[8] >> 16) | (a.n[9] << 10);
}

CUDASP_HD void fe_add(fe& r, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.n[i] = a.n[i] + b.n[i];
}

CUDASP_HD void fe_add_to(fe& r, const fe& a) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.n[i] += a.n[i];
}

CUDASP_HD void fe_mul_int(fe& r, const fe& a, uint32_t k) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.n[i] = a.n[i] * k;
}

// r = 2K*p - a  with mag(a) <= K; mag(r) <= 2K.
template <uint32_t K>
CUDASP_HD void fe_negate(fe& r, const fe& a) {
  FE_CHECK(a, K, "negate");
  r.n[0] = 0x3FFFC2Fu * 2 * K - a.n[0];
  r.n[1] = 0x3FFFFBFu * 2 * K - a.n[1];
#pragma unroll
  for (int i = 2; i < 9; i++) r.n[i] = 0x3FFFFFFu * 2 * K - a.n[i];
  r.n[9] = 0x3FFFFFu * 2 * K - a.n[9];
}

// r = a - b with mag(b) <= K: r = a + (2K p - b); mag(r) <= mag(a) + 2K.
template <uint32_t K>
CUDASP_HD void fe_sub(fe& r, const fe& a, const fe& b) {
  FE_CHECK(b, K, "sub");
  r.n[0] = a.n[0] + (0x3FFFC2Fu * 2 * K - b.n[0]);
  r.n[1] = a.n[1] + (0x3FFFFBFu * 2 * K - b.n[1]);
#pragma unroll
  for (int i = 2; i < 9; i++) r.n[i] = a.n[i] + (0x3FFFFFFu * 2 * K - b.n[i]);
  r.n[9] = a.n[9] + (0x3FFFFFu * 2 * K - b.n[9]);
}

// Carry-propagate and fold the bits above 2^256 once.  Output magnitude 1
// (value < 2^256 + small, not necessarily < p).
CUDASP_HD void fe_normalize_weak(fe& r) {
  uint32_t t0 = r.n[0], t1 = r.n[1], t2 = r.n[2], t3 = r.n[3], t4 = r.n[4];
  uint32_t t5 = r.n[5], t6 = r.n[6], t7 = r.n[7], t8 = r.n[8], t9 = r.n[9];
  uint32_t x = t9 >> 22;
  t9 &= M22;
  t0 += x * F0;
  t1 += (x << 6) + (t0 >> 26); t0 &= M26;
  t2 += (t1 >> 26); t1 &= M26;
  t3 += (t2 >> 26); t2 &= M26;
  t4 += (t3 >> 26); t3 &= M26;
  t5 += (t4 >> 26); t4 &= M26;
  t6 += (t5 >> 26); t5 &= M26;
  t7 += (t6 >> 26); t6 &= M26;
  t8 += (t7 >> 26); t7 &= M26;
  t9 += (t8 >> 26); t8 &= M26;
  r.n[0] = t0; r.n[1] = t1; r.n[2] = t2; r.n[3] = t3; r.n[4] = t4;
  r.n[5] = t5; r.n[6] = t6; r.n[7] = t7; r.n[8] = t8; r.n[9] = t9;
}

// Full normalization to the canonical representative in [0, p).
CUDASP_HD void fe_normalize(fe& r) {
  fe_normalize_weak(r);
  // Value now < 2^256 + 2^?; a second weak pass makes limb 9 <= 2^22.
  fe_normalize_weak(r);
  // r >= p  <=>  r + 0x1000003D1 >= 2^256.
  uint32_t t0 = r.n[0] + F0;
  uint32_t c = t0 >> 26;
  uint32_t t1 = r.n[1] + F1 + c; c = t1 >> 26;
  uint32_t t2 = r.n[2] + c; c = t2 >> 26;
  uint32_t t3 = r.n[3] + c; c = t3 >> 26;
  uint32_t t4 = r.n[4] + c; c = t4 >> 26;
  uint32_t t5 = r.n[5] + c; c = t5 >> 26;
  uint32_t t6 = r.n[6] + c; c = t6 >> 26;
  uint32_t t7 = r.n[7] + c; c = t7 >> 26;
  uint32_t t8 = r.n[8] + c; c = t8 >> 26;
  uint32_t t9 = r.n[9] + c;
  bool ge = (t9 >> 22) != 0;
  if (ge) {
    r.n[0] = t0 & M26; r.n[1] = t1 & M26; r.n[2] = t2 & M26; r.n[3] = t3 & M26;
    r.n[4] = t4 & M26; r.n[5] = t5 & M26; r.n[6] = t6 & M26; r.n[7] = t7 & M26;
    r.n[8] = t8 & M26; r.n[9] = t9 & M22;
  }
}

// Field multiply/square code shapes (A/B-tested on MI355X, stage A of 300k rows,
// tools/stage_timing.py):
//   0  19 parallel column sums + 26-bit carry chain over the high half, fold,
//      carry chain over the low half                              3.00 ms
//   1  like 0, but each high column folds through its two 32-bit halves
//      (no high-half carry chain)                                 2.85 ms  <- default
//   2  explicit serial mad chains in inline asm: fewest VALU (184/148 per
//      mul/sqr) but the compiler pads every asm result with s_nop  2.94 ms
//   3  variant 1's arithmetic as ONE generated asm block per operation
//      (secp256k1_fe_asm.inc, tools/gen_fe_asm.py): 172 / 127 instructions,
//      every column one mad chain seeded with the previous carry; host
//      builds use variant 1's C code
//   4  as 3, scheduled for 2-way ILP (high column k+1 computed beside low
//      column k; 175 / 130 instructions, 20 fixed temporaries)
#ifndef CUDASP_FE_VARIANT
#define CUDASP_FE_VARIANT 3
#endif
#if CUDASP_FE_VARIANT == 0
// Reduction shared by mul and sqr.  c[0..18] are the product columns
// (each < 2^62).  Folding uses 2^260 = R0 + R1*2^26 (mod p) for the high part
// and 2^256 = F0 + F1*2^26 for the final top bits.
CUDASP_HD void fe_reduce_columns(fe& r, const uint64_t c[19]) {
  // High half (weights 2^260 .. ): split columns 10..18 into 26-bit digits.
  uint32_t x[10];
  uint64_t d = c[10];
  x[0] = (uint32_t)d & M26; d >>= 26; d += c[11];
  x[1] = (uint32_t)d & M26; d >>= 26; d += c[12];
  x[2] = (uint32_t)d & M26; d >>= 26; d += c[13];
  x[3] = (uint32_t)d & M26; d >>= 26; d += c[14];
  x[4] = (uint32_t)d & M26; d >>= 26; d += c[15];
  x[5] = (uint32_t)d & M26; d >>= 26; d += c[16];
  x[6] = (uint32_t)d & M26; d >>= 26; d += c[17];
  x[7] = (uint32_t)d & M26; d >>= 26; d += c[18];
  x[8] = (uint32_t)d & M26; d >>= 26;
  x[9] = (uint32_t)d;  // < 2^25 for inputs of magnitude <= 8
  // x9 sits at weight 2^(260+234); its R1 share lands at weight 2^520 = 2^260 * 2^260.
  uint64_t x9r1 = (uint64_t)x[9] * R1;  // weight 2^260 relative to limb 0
  // Low half plus folded high half, carried into 26-bit limbs.
  uint64_t t = c[0] + (uint64_t)x[0] * R0 + x9r1 * R0;
  uint32_t r0 = (uint32_t)t & M26; t >>= 26;
  t += c[1] + (uint64_t)x[1] * R0 + (uint64_t)x[0] * R1 + x9r1 * R1;
  uint32_t r1 = (uint32_t)t & M26; t >>= 26;
  t += c[2] + (uint64_t)x[2] * R0 + (uint64_t)x[1] * R1;
  uint32_t r2 = (uint32_t)t & M26; t >>= 26;
  t += c[3] + (uint64_t)x[3] * R0 + (uint64_t)x[2] * R1;
  uint32_t r3 = (uint32_t)t & M26; t >>= 26;
  t += c[4] + (uint64_t)x[4] * R0 + (uint64_t)x[3] * R1;
  uint32_t r4 = (uint32_t)t & M26; t >>= 26;
  t += c[5] + (uint64_t)x[5] * R0 + (uint64_t)x[4] * R1;
  uint32_t r5 = (uint32_t)t & M26; t >>= 26;
  t += c[6] + (uint64_t)x[6] * R0 + (uint64_t)x[5] * R1;
  uint32_t r6 = (uint32_t)t & M26; t >>= 26;
  t += c[7] + (uint64_t)x[7] * R0 + (uint64_t)x[6] * R1;
  uint32_t r7 = (uint32_t)t & M26; t >>= 26;
  t += c[8] + (uint64_t)x[8] * R0 + (uint64_t)x[7] * R1;
  uint32_t r8 = (uint32_t)t & M26; t >>= 26;
  t += c[9] + (uint64_t)x[9] * R0 + (uint64_t)x[8] * R1;
  uint32_t r9 = (uint32_t)t & M22;
  uint64_t u = t >> 22;  // bits >= 2^256
  uint64_t s = (uint64_t)r0 + u * F0;
  r0 = (uint32_t)s & M26;
  s = (s >> 26) + r1 + u * F1;
  r1 = (uint32_t)s & M26;
  r2 += (uint32_t)(s >> 26);
  r.n[0] = r0; r.n[1] = r1; r.n[2] = r2; r.n[3] = r3; r.n[4] = r4;
  r.n[5] = r5; r.n[6] = r6; r.n[7] = r7; r.n[8] = r8; r.n[9] = r9;
}

CUDASP_HD void fe_mul(fe& r, const fe& a, const fe& b) {
  FE_CHECK_MUL(a, b, "mul");
  uint64_t c[19];
#pragma unroll
  for (int k = 0; k < 19; k++) {
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      int j = k - i;
      if (j >= 0 && j < 10) s += (uint64_t)a.n[i] * b.n[j];
    }
    c[k] = s;
  }
  fe_reduce_columns(r, c);
}

CUDASP_HD void fe_sqr(fe& r, const fe& a) {
  FE_CHECK_MUL(a, a, "sqr");
  uint32_t a2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) a2[i] = a.n[i] * 2;
  uint64_t c[19];
#pragma unroll
  for (int k = 0; k < 19; k++) {
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      int j = k - i;
      if (j > i && j < 10) s += (uint64_t)a2[i] * a.n[j];
      else if (j == i) s += (uint64_t)a.n[i] * a.n[i];
    }
    c[k] = s;
  }
  fe_reduce_columns(r, c);
}

#elif CUDASP_FE_VARIANT == 1 || CUDASP_FE_VARIANT == 3 || CUDASP_FE_VARIANT == 4
CUDASP_HD void fe_reduce_columns(fe& r, const uint64_t c[19]) {
  const uint32_t r0 = opaque_const(R0), r1 = opaque_const(R1);
  const uint32_t r0s = opaque_const(R0 << 6), r1s = opaque_const(R1 << 6);
  uint64_t t[11];
#pragma unroll
  for (int k = 0; k < 10; k++) t[k] = c[k];
  t[10] = 0;
#pragma unroll
  for (int m = 0; m < 9; m++) {
    uint32_t lo = (uint32_t)c[10 + m], hi = (uint32_t)(c[10 + m] >> 32);
    t[m] += (uint64_t)lo * r0;
    t[m + 1] += (uint64_t)lo * r1 + (uint64_t)hi * r0s;
    t[m + 2] += (uint64_t)hi * r1s;
  }
  {
    uint32_t lo = (uint32_t)t[10], hi = (uint32_t)(t[10] >> 32);
    t[0] += (uint64_t)lo * r0;
    t[1] += (uint64_t)lo * r1 + (uint64_t)hi * r0s;
    t[2] += (uint64_t)hi * r1s;
  }
  uint32_t o[10];
#pragma unroll
  for (int k = 0; k < 9; k++) {
    o[k] = (uint32_t)t[k] & M26;
    t[k + 1] += t[k] >> 26;
  }
  o[9] = (uint32_t)t[9] & M22;
  uint64_t u = t[9] >> 22;
  uint32_t ulo = (uint32_t)u, uhi = (uint32_t)(u >> 32);
  const uint32_t f0 = opaque_const(F0), f1 = opaque_const(F1);
  const uint32_t f0s = opaque_const(F0 << 6), f1s = opaque_const(F1 << 6);
  uint64_t s0 = (uint64_t)o[0] + (uint64_t)ulo * f0;
  uint64_t s1 = (uint64_t)o[1] + (uint64_t)ulo * f1 + (uint64_t)uhi * f0s + (s0 >> 26);
  uint64_t s2 = (uint64_t)o[2] + (uint64_t)uhi * f1s + (s1 >> 26);
  r.n[0] = (uint32_t)s0 & M26;
  r.n[1] = (uint32_t)s1 & M26;
  r.n[2] = (uint32_t)s2;
#pragma unroll
  for (int k = 3; k < 10; k++) r.n[k] = o[k];
}

CUDASP_HD void fe_mul_c(fe& r, const fe& a, const fe& b) {
  uint64_t c[19];
#pragma unroll
  for (int k = 0; k < 19; k++) {
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      int j = k - i;
      if (j >= 0 && j < 10) s += (uint64_t)a.n[i] * b.n[j];
    }
    c[k] = s;
  }
  fe_reduce_columns(r, c);
}

CUDASP_HD void fe_sqr_c(fe& r, const fe& a) {
  uint32_t a2[10];
#pragma unroll
  for (int i = 0; i < 10; i++) a2[i] = a.n[i] * 2;
  uint64_t c[19];
#pragma unroll
  for (int k = 0; k < 19; k++) {
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      int j = k - i;
      if (j > i && j < 10) s += (uint64_t)a2[i] * a.n[j];
      else if (j == i) s += (uint64_t)a.n[i] * a.n[i];
    }
    c[k] = s;
  }
  fe_reduce_columns(r, c);
}

#if CUDASP_FE_VARIANT >= 3 && defined(__HIP_DEVICE_COMPILE__)
#include "secp256k1_fe_asm.inc"
#endif

CUDASP_HD void fe_mul(fe& r, const fe& a, const fe& b) {
  FE_CHECK_MUL(a, b, "mul");
#if CUDASP_FE_VARIANT == 3 && defined(__HIP_DEVICE_COMPILE__)
  fe_mul_asm(r, a, b);
#elif CUDASP_FE_VARIANT == 4 && defined(__HIP_DEVICE_COMPILE__)
  fe_mul_asm_p(r, a, b);
#else
  fe_mul_c(r, a, b);
#endif
}

CUDASP_HD void fe_sqr(fe& r, const fe& a) {
  FE_CHECK_MUL(a, a, "sqr");
#if CUDASP_FE_VARIANT == 3 && defined(__HIP_DEVICE_COMPILE__)
  fe_sqr_asm(r, a);
#elif CUDASP_FE_VARIANT == 4 && defined(__HIP_DEVICE_COMPILE__)
  fe_sqr_asm_p(r, a);
#else
  fe_sqr_c(r, a);
#endif
}

#else
// acc + a*b as one v_mad_u64_u32 (accumulator tied in place).  Written as asm
// so the compiler keeps the carry-free accumulation chains exactly as laid out
// below instead of re-associating them into parallel partial sums that it then
// has to add with extra 64-bit adds and register-pair moves.
CUDASP_HD uint64_t mad64(uint32_t a, uint32_t b, uint64_t acc) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t r, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(a), "v"(b), "0"(acc));
  (void)cc;
  return r;
#else
  return (uint64_t)a * b + acc;
#endif
}

// Same with b in a scalar register (the fold constants).
CUDASP_HD uint64_t mad64s(uint32_t a, uint32_t b_uniform, uint64_t acc) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t r, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(a), "s"(b_uniform), "0"(acc));
  (void)cc;
  return r;
#else
  return (uint64_t)a * b_uniform + acc;
#endif
}

// Product columns: column k = sum_{i+j=k} a_i b_j, each a single mad chain.
// High columns 10..18 are independent chains; the low columns form one carry
// chain (below) that starts each column from the previous column's carry.
//
// Reduction: a high column c_{10+m} (weight 2^(260 + 26m)) is folded through
// its two 32-bit halves, which cost nothing to extract:
//   lo * 2^(260+26m) = lo*R0 @m + lo*R1 @m+1              (2^260 = R0 + R1 2^26)
//   hi * 2^(292+26m) = hi*(R0<<6) @m+1 + hi*(R1<<6) @m+2
// then the low column k is accumulated on top of the carry of column k-1,
// split at 26 bits, and the bits above 2^256 fold with 2^256 = F0 + F1 2^26.
// Bounds (inputs of magnitude <= 8): columns < 2^61.4, folded terms < 2^51.
template <bool SQR>
CUDASP_HD void fe_mul_impl(fe& r, const fe& a, const fe& b) {
  uint32_t a2[10];
  if (SQR) {
#pragma unroll
    for (int i = 0; i < 10; i++) a2[i] = a.n[i] << 1;
  }
  // column term generator
  auto column = [&](int k, uint64_t acc) -> uint64_t {
#pragma unroll
    for (int i = 0; i < 10; i++) {
      int j = k - i;
      if (j < 0 || j >= 10) continue;
      if (SQR) {
        if (j > i) acc = mad64(a2[i], a.n[j], acc);
        else if (j == i) acc = mad64(a.n[i], a.n[i], acc);
      } else {
        acc = mad64(a.n[i], b.n[j], acc);
      }
    }
    return acc;
  };
  uint64_t h[9];
#pragma unroll
  for (int m = 0; m < 9; m++) h[m] = column(10 + m, 0);
  const uint32_t r0 = opaque_const(R0), r1 = opaque_const(R1);
  const uint32_t r0s = opaque_const(R0 << 6), r1s = opaque_const(R1 << 6);
  // second-order overflow: column 18's hi*(R1<<6) lands at weight 2^260 again.
  uint64_t top = mad64s((uint32_t)(h[8] >> 32), r1s, 0);  // weight 2^260, < 2^47
  uint32_t top_lo = (uint32_t)top, top_hi = (uint32_t)(top >> 32);
  uint32_t o[10];
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    if (k < 9) acc = mad64s((uint32_t)h[k], r0, acc);
    if (k >= 1 && k - 1 < 9) {
      acc = mad64s((uint32_t)h[k - 1], r1, acc);
      acc = mad64s((uint32_t)(h[k - 1] >> 32), r0s, acc);
    }
    if (k >= 2 && k - 2 < 8) acc = mad64s((uint32_t)(h[k - 2] >> 32), r1s, acc);
    if (k == 0) acc = mad64s(top_lo, r0, acc);
    if (k == 1) {
      acc = mad64s(top_lo, r1, acc);
      acc = mad64s(top_hi, r0s, acc);
    }
    if (k == 2) acc = mad64s(top_hi, r1s, acc);
    acc = column(k, acc);
    if (k < 9) {
      o[k] = (uint32_t)acc & M26;
      acc >>= 26;
    }
  }
  o[9] = (uint32_t)acc & M22;
  uint64_t u = acc >> 22;  // bits >= 2^256, < 2^41
  uint32_t ulo = (uint32_t)u, uhi = (uint32_t)(u >> 32);
  const uint32_t f0 = opaque_const(F0), f1 = opaque_const(F1);
  const uint32_t f0s = opaque_const(F0 << 6), f1s = opaque_const(F1 << 6);
  uint64_t s0 = mad64s(ulo, f0, o[0]);
  uint64_t s1 = mad64s(uhi, f0s, mad64s(ulo, f1, (uint64_t)o[1] + (s0 >> 26)));
  uint64_t s2 = mad64s(uhi, f1s, (uint64_t)o[2] + (s1 >> 26));
  r.n[0] = (uint32_t)s0 & M26;
  r.n[1] = (uint32_t)s1 & M26;
  r.n[2] = (uint32_t)s2;  // < 2^26 + 2^21
#pragma unroll
  for (int k = 3; k < 10; k++) r.n[k] = o[k];
}

CUDASP_HD void fe_mul(fe& r, const fe& a, const fe& b) {
  FE_CHECK_MUL(a, b, "mul");
  fe_mul_impl<false>(r, a, b);
}

CUDASP_HD void fe_sqr(fe& r, const fe& a) {
  FE_CHECK_MUL(a, a, "sqr");
  fe_mul_impl<true>(r, a, a);
}

#endif

}  // namespace cudasp
#else
#error "CUDASP_FE_LIMBS must be 9 or 10"
#endif

// ----------------------------------------------- layout-independent helpers
namespace cudasp {

CUDASP_HD void fe_set_int(fe& r, uint32_t v) {
  r.n[0] = v;
#pragma unroll
  for (int i = 1; i < FE_LIMBS; i++) r.n[i] = 0;
}

CUDASP_HD bool fe_is_zero_norm(const fe& a) {
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) z |= a.n[i];
  return z == 0;
}

CUDASP_HD bool fe_equal_norm(const fe& a, const fe& b) {
  uint32_t z = 0;
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) z |= a.n[i] ^ b.n[i];
  return z == 0;
}

CUDASP_HD void fe_sqr_n(fe& r, const fe& a, int n) {
  fe_sqr(r, a);
  for (int i = 1; i < n; i++) fe_sqr(r, r);
}

// a^(p-2) via the addition chain 223 ones | 0 | 22 ones | 0000 1 0 11 0 1
// (kept as a cross-check for tests; the kernels use fe_inv = safegcd,
// secp256k1_inv.hpp)
// (p-2 = 0xFF..FE FFFFFC2D): 255 squarings + 15 multiplications.
CUDASP_HD void fe_inv_fermat(fe& r, const fe& a) {
  fe x2, x3, x6, x9, x11, x22, x44, x88, x176, x220, x223, t;
  fe_sqr(x2, a);
  fe_mul(x2, x2, a);
  fe_sqr(x3, x2);
  fe_mul(x3, x3, a);
  fe_sqr_n(x6, x3, 3);
  fe_mul(x6, x6, x3);
  fe_sqr_n(x9, x6, 3);
  fe_mul(x9, x9, x3);
  fe_sqr_n(x11, x9, 2);
  fe_mul(x11, x11, x2);
  fe_sqr_n(x22, x11, 11);
  fe_mul(x22, x22, x11);
  fe_sqr_n(x44, x22, 22);
  fe_mul(x44, x44, x22);
  fe_sqr_n(x88, x44, 44);
  fe_mul(x88, x88, x44);
  fe_sqr_n(x176, x88, 88);
  fe_mul(x176, x176, x88);
  fe_sqr_n(x220, x176, 44);
  fe_mul(x220, x220, x44);
  fe_sqr_n(x223, x220, 3);
  fe_mul(x223, x223, x3);
  fe_sqr_n(t, x223, 23);
  fe_mul(t, t, x22);
  fe_sqr_n(t, t, 5);
  fe_mul(t, t, a);
  fe_sqr_n(t, t, 3);
  fe_mul(t, t, x2);
  fe_sqr_n(t, t, 2);
  fe_mul(r, t, a);
}

// Conditional select: r = c ? a : b (per lane).
CUDASP_HD void fe_cmov(fe& r, const fe& a, bool c) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) r.n[i] = c ? a.n[i] : r.n[i];
}

}  // namespace cudasp
