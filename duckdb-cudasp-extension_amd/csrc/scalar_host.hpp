// Host-side scalar preparation for the variable-base multiply S = d * T.
//
// The scan key d is the same for every row of a query (the reference passes it
// once, src/cudasp_gpu.cu:719-732, and replicates it n times for gECC), so its
// recoding is done once per query on the host and the kernel's control flow is
// uniform across the whole grid.  d is split with the secp256k1 endomorphism
// (GLV): d = k1 + k2 * lambda (mod n) with |k1|, |k2| < 2^129, and each half is
// recoded to width-5 NAF.  The kernel then does ~129 doublings instead of 256.
#pragma once
#include <vector>
#include <stdint.h>
#include <string.h>

namespace cudasp {
namespace host {

// Little-endian multi-precision helpers on 32-bit words (host only, not hot).
template <int W>
struct Big {
  uint32_t w[W];
};

template <int W>
static inline Big<W> big_zero() {
  Big<W> r;
  memset(r.w, 0, sizeof(r.w));
  return r;
}

template <int A, int B>
static inline Big<A + B> big_mul(const Big<A>& a, const Big<B>& b) {
  Big<A + B> r = big_zero<A + B>();
  for (int i = 0; i < A; i++) {
    uint64_t carry = 0;
    for (int j = 0; j < B; j++) {
      uint64_t t = (uint64_t)a.w[i] * b.w[j] + r.w[i + j] + carry;
      r.w[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    r.w[i + B] = (uint32_t)carry;
  }
  return r;
}

template <int W>
static inline uint32_t big_add(Big<W>& r, const Big<W>& a, const Big<W>& b) {
  uint64_t c = 0;
  for (int i = 0; i < W; i++) {
    c += (uint64_t)a.w[i] + b.w[i];
    r.w[i] = (uint32_t)c;
    c >>= 32;
  }
  return (uint32_t)c;
}

template <int W>
static inline uint32_t big_sub(Big<W>& r, const Big<W>& a, const Big<W>& b) {
  int64_t c = 0;
  for (int i = 0; i < W; i++) {
    c += (int64_t)a.w[i] - b.w[i];
    r.w[i] = (uint32_t)c;
    c >>= 32;
  }
  return (uint32_t)(c & 1);  // borrow
}

template <int W>
static inline int big_cmp(const Big<W>& a, const Big<W>& b) {
  for (int i = W - 1; i >= 0; i--) {
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  }
  return 0;
}

template <int W, int V>
static inline Big<W> big_resize(const Big<V>& a) {
  Big<W> r = big_zero<W>();
  for (int i = 0; i < W && i < V; i++) r.w[i] = a.w[i];
  return r;
}

template <int W>
static inline bool big_is_zero(const Big<W>& a) {
  for (int i = 0; i < W; i++)
    if (a.w[i]) return false;
  return true;
}

static inline Big<8> big_from_hex_be(const char* hex) {
  Big<8> r = big_zero<8>();
  int len = (int)strlen(hex);
  for (int i = 0; i < len; i++) {
    char ch = hex[len - 1 - i];
    uint32_t v = (ch >= '0' && ch <= '9') ? ch - '0' : (ch >= 'a' && ch <= 'f') ? ch - 'a' + 10 : ch - 'A' + 10;
    r.w[i / 8] |= v << (4 * (i % 8));
  }
  return r;
}

// secp256k1 group order n and GLV constants.
struct GlvConsts {
  Big<8> n, g1, g2, a1, minus_b1, a2, b2;
  GlvConsts() {
    n = big_from_hex_be("FFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141");
    // g1 = round(2^384 * b2 / n), g2 = round(2^384 * (-b1) / n)
    g1 = big_from_hex_be("3086d221a7d46bcde86c90e49284eb153daa8a1471e8ca7fe893209a45dbb031");
    g2 = big_from_hex_be("e4437ed6010e88286f547fa90abfe4c4221208ac9df506c61571b4ae8ac47f71");
    // lattice basis (a1, b1), (a2, b2) with a_i + b_i*lambda = 0 (mod n)
    a1 = big_from_hex_be("3086d221a7d46bcde86c90e49284eb15");
    minus_b1 = big_from_hex_be("e4437ed6010e88286f547fa90abfe4c3");
    a2 = big_from_hex_be("114ca50f7a8e2f3f657c1108d9d44cfd8");
    b2 = a1;
  }
};

// d mod n (d < 2^256 < 2n, so one conditional subtraction).
static inline Big<8> scalar_reduce(const Big<8>& d) {
  GlvConsts c;
  Big<8> r = d;
  if (big_cmp(r, c.n) >= 0) big_sub(r, r, c.n);
  return r;
}

// round(k * g / 2^384)
static inline Big<8> mul_shift_384(const Big<8>& k, const Big<8>& g) {
  Big<16> p = big_mul(k, g);
  // add 2^383 for rounding
  Big<16> half = big_zero<16>();
  half.w[11] = 0x80000000u;
  big_add(p, p, half);
  Big<8> r = big_zero<8>();
  for (int i = 0; i < 4; i++) r.w[i] = p.w[12 + i];
  return r;
}

struct SignedHalf {
  Big<8> mag;  // |k_i|
  bool neg;
};

// d = k1 + k2 * lambda (mod n) by Babai rounding against the reduced lattice
// basis, as two's complement 288-bit values r1 = k1, r2 = k2 (|k_i| < 2^129).
static inline void glv_split_raw(const Big<8>& d_in, Big<9>& r1, Big<9>& r2) {
  GlvConsts c;
  Big<8> d = scalar_reduce(d_in);
  Big<8> c1 = mul_shift_384(d, c.g1);
  Big<8> c2 = mul_shift_384(d, c.g2);
  // products are < 2^(130+129), keep 9 words (288 bits), two's complement.
  Big<9> c1a1 = big_resize<9>(big_mul(big_resize<4>(c1), big_resize<5>(c.a1)));
  Big<9> c2a2 = big_resize<9>(big_mul(big_resize<4>(c2), big_resize<5>(c.a2)));
  Big<9> c1b1 = big_resize<9>(big_mul(big_resize<4>(c1), big_resize<5>(c.minus_b1)));
  Big<9> c2b2 = big_resize<9>(big_mul(big_resize<4>(c2), big_resize<5>(c.b2)));
  r1 = big_resize<9>(d);
  big_sub(r1, r1, c1a1);
  big_sub(r1, r1, c2a2);   // k1 = d - c1 a1 - c2 a2
  big_sub(r2, c1b1, c2b2); // k2 = -c1 b1 - c2 b2 = c1 (-b1) - c2 b2
}

static inline void to_signed_half(const Big<9>& v, SignedHalf& out) {
  out.neg = (v.w[8] >> 31) != 0;
  Big<9> m = v;
  if (out.neg) {
    Big<9> z = big_zero<9>();
    big_sub(m, z, v);
  }
  out.mag = big_resize<8>(m);
}

static inline void glv_split(const Big<8>& d_in, SignedHalf& k1, SignedHalf& k2) {
  Big<9> r1, r2;
  glv_split_raw(d_in, r1, r2);
  to_signed_half(r1, k1);
  to_signed_half(r2, k2);
}

// r += m * v for a small signed m.
static inline void big_add_small_multiple(Big<9>& r, const Big<8>& v, int m) {
  Big<9> w = big_resize<9>(v);
  for (int i = 0; i < (m < 0 ? -m : m); i++) {
    if (m > 0)
      big_add(r, r, w);
    else
      big_sub(r, r, w);
  }
}

// Width-w NAF of a non-negative integer (< 2^256); digits[i] is the digit of
// weight 2^i, odd in (-2^(w-1), 2^(w-1)) or 0.  Returns the number of digits
// (index of the top nonzero digit + 1), 0 for k = 0, -1 if a nonzero digit
// would fall at or past max_digits.  Runs of zero digits are skipped a word
// at a time (scan_digits recodes ~580 candidates per query).
static inline int wnaf(int8_t* digits, int max_digits, const Big<8>& k_in, int w) {
  Big<9> k = big_resize<9>(k_in);
  memset(digits, 0, max_digits);
  int len = 0;
  int i = 0;
  // k >>= z (z < 32)
  auto shr = [&k](int z) {
    if (z == 0) return;
    for (int j = 0; j < 9; j++) k.w[j] = (k.w[j] >> z) | (j + 1 < 9 ? (k.w[j + 1] << (32 - z)) : 0);
  };
  for (;;) {
    // skip zero words, then zero bits
    int zw = 0;
    while (zw < 9 && k.w[zw] == 0) zw++;
    if (zw == 9) break;
    if (zw) {
      for (int j = 0; j < 9; j++) k.w[j] = j + zw < 9 ? k.w[j + zw] : 0;
      i += 32 * zw;
    }
    const int z = __builtin_ctz(k.w[0]);
    shr(z);
    i += z;
    if (i >= max_digits) return -1;
    int d = (int)(k.w[0] & ((1u << w) - 1));
    if (d >= (1 << (w - 1))) d -= (1 << w);
    Big<9> dd = big_zero<9>();
    if (d > 0) {
      dd.w[0] = (uint32_t)d;
      big_sub(k, k, dd);
    } else {
      dd.w[0] = (uint32_t)(-d);
      big_add(k, k, dd);
    }
    digits[i] = (int8_t)d;
    len = i + 1;
    shr(1);
    i++;
  }
  return len;
}

// Stage-A ladder cost of one operation (VALU instructions per doubling and per
// mixed addition incl. its table load, gfx950 build of secp256k1_group29.hpp);
// used to rank decompositions of the scan key.
constexpr int LADDER_DBL_COST = 903;
constexpr int LADDER_ADD_COST = 1600;

// The uniform signed digits of the stage-A ladder for scan key d: d = k1 +
// k2 lambda (mod n), k1 and k2 each as a width-5 NAF (digits of k_i in
// naf[i * naf_max ..], signs applied), naf_len = the longer length.  Every
// lattice point (k1, k2) + i (a1, b1) + j (a2, b2) with |i|, |j| <= search
// represents the same d; the kernels pay (naf_len - 1) doublings and
// (weight - 1) additions, so the cheapest of those is taken (the Babai
// point (0, 0) on ties).  The choice is per query and costs ~300 wNAF
// recodings on the host.  Returns 0, or -1 if no candidate fits naf_max.
static inline int scan_digits(const Big<8>& d, int8_t* naf, int naf_max, uint32_t* naf_len, int search = 8) {
  GlvConsts c;
  Big<9> r1, r2;
  glv_split_raw(d, r1, r2);
  std::vector<int8_t> t(2 * (size_t)naf_max);
  long best = -1;
  int order[2 * 64 + 1];
  int m = 0;
  order[m++] = 0;
  for (int k = 1; k <= search && k <= 64; k++) {
    order[m++] = k;
    order[m++] = -k;
  }
  for (int ii = 0; ii < m; ii++) {
    for (int jj = 0; jj < m; jj++) {
      int i = order[ii], j = order[jj];
      Big<9> v1 = r1, v2 = r2;
      big_add_small_multiple(v1, c.a1, i);
      big_add_small_multiple(v1, c.a2, j);
      big_add_small_multiple(v2, c.minus_b1, -i);
      big_add_small_multiple(v2, c.b2, j);
      SignedHalf k1, k2;
      to_signed_half(v1, k1);
      to_signed_half(v2, k2);
      int l1 = wnaf(t.data(), naf_max, k1.mag, 5);
      int l2 = wnaf(t.data() + naf_max, naf_max, k2.mag, 5);
      if (l1 < 0 || l2 < 0) continue;
      int weight = 0;
      for (int q = 0; q < 2 * naf_max; q++) weight += t[q] != 0;
      int len = l1 > l2 ? l1 : l2;
      if (weight == 0) continue;
      long cost = (long)(len - 1) * LADDER_DBL_COST + (long)(weight - 1) * LADDER_ADD_COST;
      if (best >= 0 && cost >= best) continue;
      best = cost;
      for (int q = 0; q < naf_max; q++) {
        naf[q] = k1.neg ? (int8_t)-t[q] : t[q];
        naf[naf_max + q] = k2.neg ? (int8_t)-t[naf_max + q] : t[naf_max + q];
      }
      *naf_len = (uint32_t)len;
    }
  }
  return best >= 0 ? 0 : -1;
}

}  // namespace host
}  // namespace cudasp
