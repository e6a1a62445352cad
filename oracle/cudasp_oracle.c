/*
 * cudasp_oracle.c -- CPU restatement of the reference's cudasp_scan algorithm.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker (tests/,
 * __graft_entry__.smoke()) and the CPU baseline of bench.py; the product path
 * (duckdb-cudasp-extension_amd/libcudasp_amd.so) never calls it.
 *
 * It restates, independently of the HIP code (different limb size, different
 * formulas, no endomorphism, no precomputed tables, no midstate):
 *   - the per-row pipeline of /root/reference/src/cudasp_gpu.cu
 *       S = d*T                              (:764-784, gECC ecdsa_ec_pmul)
 *       ser = 02|03 || BE(S.x) || 00000000   (:236-284)
 *       t = SHA256(H(tag)||H(tag)||ser)      (:288-314)
 *       t as a big-endian 256-bit integer, no mod-n reduction (:862-877)
 *       P0 = t*G                             (:318-354)
 *       F = P0 + B; v = int64(F.x >> 192)    (:44-71, :124-131)
 *       labels: v_j of F + L_j, in order     (:133-172)
 *   - the point arithmetic of the reference's CPU oracle
 *     /root/reference/scripts/compute_bip352_expected.py:32-93 (complete
 *     affine addition: doubling when P == Q, infinity when P == -Q);
 *   - the byte conventions of /root/reference/src/cudasp_extension.cu:59-85.
 * Pinned against the reference's own expectations by tests/test_oracle.py
* (tests/golden/ *.json fixtures, generated from the reference by make_golden.py).
 *
 * Field elements: 4 x 64-bit limbs, little-endian, fully reduced mod p.
 */
#include "cudasp_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned __int128 u128;
typedef struct { uint64_t v[4]; } fe4;

static const fe4 P_MOD = {{0xFFFFFFFEFFFFFC2FULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL, 0xFFFFFFFFFFFFFFFFULL}};
static const fe4 N_ORD = {{0xBFD25E8CD0364141ULL, 0xBAAEDCE6AF48A03BULL, 0xFFFFFFFFFFFFFFFEULL, 0xFFFFFFFFFFFFFFFFULL}};
static const fe4 GX = {{0x59F2815B16F81798ULL, 0x029BFCDB2DCE28D9ULL, 0x55A06295CE870B07ULL, 0x79BE667EF9DCBBACULL}};
static const fe4 GY = {{0x9C47D08FFB10D4B8ULL, 0xFD17B448A6855419ULL, 0x5DA4FBFC0E1108A8ULL, 0x483ADA7726A3C465ULL}};

/* ------------------------------------------------------------ 256-bit ints */
static int u256_cmp(const fe4* a, const fe4* b) {
  for (int i = 3; i >= 0; i--) {
    if (a->v[i] != b->v[i]) return a->v[i] < b->v[i] ? -1 : 1;
  }
  return 0;
}

static uint64_t u256_add(fe4* r, const fe4* a, const fe4* b) {
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (u128)a->v[i] + b->v[i];
    r->v[i] = (uint64_t)c;
    c >>= 64;
  }
  return (uint64_t)c;
}

static uint64_t u256_sub(fe4* r, const fe4* a, const fe4* b) {
  uint64_t borrow = 0;
  for (int i = 0; i < 4; i++) {
    u128 t = (u128)a->v[i] - b->v[i] - borrow;
    r->v[i] = (uint64_t)t;
    borrow = (uint64_t)(t >> 64) & 1;
  }
  return borrow;
}

static int u256_is_zero(const fe4* a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }

static void u256_from_le(fe4* r, const uint8_t* b) {
  for (int i = 0; i < 4; i++) {
    uint64_t w = 0;
    for (int k = 7; k >= 0; k--) w = (w << 8) | b[8 * i + k];
    r->v[i] = w;
  }
}

static void u256_from_be(fe4* r, const uint8_t* b) {
  for (int i = 0; i < 4; i++) {
    uint64_t w = 0;
    for (int k = 0; k < 8; k++) w = (w << 8) | b[8 * (3 - i) + k];
    r->v[i] = w;
  }
}

static void u256_to_be(uint8_t* b, const fe4* a) {
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 8; k++) b[8 * (3 - i) + k] = (uint8_t)(a->v[i] >> (56 - 8 * k));
}

static int u256_bit(const fe4* a, int i) { return (int)((a->v[i >> 6] >> (i & 63)) & 1); }

/* ------------------------------------------------------------ field mod p */
static void fp_reduce_once(fe4* a) {
  if (u256_cmp(a, &P_MOD) >= 0) u256_sub(a, a, &P_MOD);
}

static void fp_from_le(fe4* r, const uint8_t* b) {
  /* Values >= p are read modulo p, as the reference's Montgomery conversion does. */
  u256_from_le(r, b);
  fp_reduce_once(r);
}

static void fp_add(fe4* r, const fe4* a, const fe4* b) {
  uint64_t c = u256_add(r, a, b);
  if (c || u256_cmp(r, &P_MOD) >= 0) u256_sub(r, r, &P_MOD);
}

static void fp_sub(fe4* r, const fe4* a, const fe4* b) {
  if (u256_sub(r, a, b)) u256_add(r, r, &P_MOD);
}

/* 2^256 = 0x1000003D1 (mod p) */
static void fp_mul(fe4* r, const fe4* a, const fe4* b) {
  uint64_t t[8] = {0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)a->v[i] * b->v[j] + t[i + j];
      t[i + j] = (uint64_t)c;
      c >>= 64;
    }
    t[i + 4] = (uint64_t)c;
  }
  /* fold high 256 bits: lo + hi * 0x1000003D1 */
  u128 c = 0;
  uint64_t s[5];
  for (int i = 0; i < 4; i++) {
    c += (u128)t[4 + i] * 0x1000003D1ULL + t[i];
    s[i] = (uint64_t)c;
    c >>= 64;
  }
  s[4] = (uint64_t)c;
  c = (u128)s[4] * 0x1000003D1ULL + s[0];
  fe4 out;
  out.v[0] = (uint64_t)c;
  c >>= 64;
  for (int i = 1; i < 4; i++) {
    c += s[i];
    out.v[i] = (uint64_t)c;
    c >>= 64;
  }
  if (c) { /* one more wrap: add 0x1000003D1 */
    fe4 k = {{0x1000003D1ULL, 0, 0, 0}};
    u256_add(&out, &out, &k);
  }
  fp_reduce_once(&out);
  *r = out;
}

static void fp_sqr(fe4* r, const fe4* a) { fp_mul(r, a, a); }

/* a^(p-2) by plain left-to-right square-and-multiply */
static void fp_inv(fe4* r, const fe4* a) {
  fe4 e = P_MOD, two = {{2, 0, 0, 0}};
  u256_sub(&e, &e, &two);
  fe4 acc = {{1, 0, 0, 0}};
  for (int i = 255; i >= 0; i--) {
    fp_sqr(&acc, &acc);
    if (u256_bit(&e, i)) fp_mul(&acc, &acc, a);
  }
  *r = acc;
}

static int fp_eq(const fe4* a, const fe4* b) { return u256_cmp(a, b) == 0; }

/* ------------------------------------------------------ affine points */
typedef struct {
  fe4 x, y;
  int inf;
} apt;

/* point_add of scripts/compute_bip352_expected.py:32-53 (+ point_double :55-67) */
static apt pt_add(const apt* p, const apt* q) {
  if (p->inf) return *q;
  if (q->inf) return *p;
  fe4 num, den;
  if (fp_eq(&p->x, &q->x)) {
    if (!fp_eq(&p->y, &q->y)) {
      apt o;
      memset(&o, 0, sizeof(o));
      o.inf = 1;
      return o;
    }
    /* s = 3x^2 / 2y */
    fe4 x2;
    fp_sqr(&x2, &p->x);
    fp_add(&num, &x2, &x2);
    fp_add(&num, &num, &x2);
    fp_add(&den, &p->y, &p->y);
  } else {
    fp_sub(&num, &q->y, &p->y);
    fp_sub(&den, &q->x, &p->x);
  }
  fe4 inv, s, s2, x3, y3, t;
  fp_inv(&inv, &den);
  fp_mul(&s, &num, &inv);
  fp_sqr(&s2, &s);
  fp_sub(&x3, &s2, &p->x);
  fp_sub(&x3, &x3, &q->x);
  fp_sub(&t, &p->x, &x3);
  fp_mul(&y3, &s, &t);
  fp_sub(&y3, &y3, &p->y);
  apt r;
  r.x = x3;
  r.y = y3;
  r.inf = 0;
  return r;
}

/* ---------------------------------------------------- Jacobian points */
typedef struct {
  fe4 x, y, z;
  int inf;
} jpt;

static void j_double(jpt* r, const jpt* a) {
  if (a->inf || u256_is_zero(&a->y)) {
    memset(r, 0, sizeof(*r));
    r->inf = 1;
    return;
  }
  /* a = 0: S = 4 X Y^2, M = 3 X^2, X' = M^2 - 2S, Y' = M (S - X') - 8 Y^4, Z' = 2 Y Z */
  fe4 yy, s, m, x3, y3, z3, t, yyyy;
  fp_sqr(&yy, &a->y);
  fp_mul(&s, &a->x, &yy);
  fp_add(&s, &s, &s);
  fp_add(&s, &s, &s);
  fp_sqr(&t, &a->x);
  fp_add(&m, &t, &t);
  fp_add(&m, &m, &t);
  fp_sqr(&x3, &m);
  fp_sub(&x3, &x3, &s);
  fp_sub(&x3, &x3, &s);
  fp_sqr(&yyyy, &yy);
  fp_add(&yyyy, &yyyy, &yyyy);
  fp_add(&yyyy, &yyyy, &yyyy);
  fp_add(&yyyy, &yyyy, &yyyy);
  fp_sub(&t, &s, &x3);
  fp_mul(&y3, &m, &t);
  fp_sub(&y3, &y3, &yyyy);
  fp_mul(&z3, &a->y, &a->z);
  fp_add(&z3, &z3, &z3);
  r->x = x3;
  r->y = y3;
  r->z = z3;
  r->inf = 0;
}

/* complete Jacobian + Jacobian (add-1998-cmo-2 with the doubling/inverse cases) */
static void j_add(jpt* r, const jpt* a, const jpt* b) {
  if (a->inf) { *r = *b; return; }
  if (b->inf) { *r = *a; return; }
  fe4 z1z1, z2z2, u1, u2, s1, s2, t;
  fp_sqr(&z1z1, &a->z);
  fp_sqr(&z2z2, &b->z);
  fp_mul(&u1, &a->x, &z2z2);
  fp_mul(&u2, &b->x, &z1z1);
  fp_mul(&t, &b->z, &z2z2);
  fp_mul(&s1, &a->y, &t);
  fp_mul(&t, &a->z, &z1z1);
  fp_mul(&s2, &b->y, &t);
  if (fp_eq(&u1, &u2)) {
    if (fp_eq(&s1, &s2)) {
      j_double(r, a);
    } else {
      memset(r, 0, sizeof(*r));
      r->inf = 1;
    }
    return;
  }
  fe4 h, rr, hh, hhh, v, x3, y3, z3;
  fp_sub(&h, &u2, &u1);
  fp_sub(&rr, &s2, &s1);
  fp_sqr(&hh, &h);
  fp_mul(&hhh, &h, &hh);
  fp_mul(&v, &u1, &hh);
  fp_sqr(&x3, &rr);
  fp_sub(&x3, &x3, &hhh);
  fp_sub(&x3, &x3, &v);
  fp_sub(&x3, &x3, &v);
  fp_sub(&t, &v, &x3);
  fp_mul(&y3, &rr, &t);
  fp_mul(&t, &s1, &hhh);
  fp_sub(&y3, &y3, &t);
  fp_mul(&z3, &a->z, &b->z);
  fp_mul(&z3, &z3, &h);
  r->x = x3;
  r->y = y3;
  r->z = z3;
  r->inf = 0;
}

static apt j_to_affine(const jpt* a) {
  apt r;
  memset(&r, 0, sizeof(r));
  if (a->inf) {
    r.inf = 1;
    return r;
  }
  fe4 zi, zi2, zi3;
  fp_inv(&zi, &a->z);
  fp_sqr(&zi2, &zi);
  fp_mul(&zi3, &zi2, &zi);
  fp_mul(&r.x, &a->x, &zi2);
  fp_mul(&r.y, &a->y, &zi3);
  return r;
}

/* k * P, k any 256-bit integer (not reduced: n*P = O), 4-bit fixed windows.
 * Same result as point_multiply of compute_bip352_expected.py:69-83. */
static apt pt_mul(const fe4* k, const apt* p) {
  jpt tab[16];
  memset(&tab[0], 0, sizeof(jpt));
  tab[0].inf = 1;
  tab[1].x = p->x;
  tab[1].y = p->y;
  memset(&tab[1].z, 0, sizeof(fe4));
  tab[1].z.v[0] = 1;
  tab[1].inf = p->inf;
  for (int i = 2; i < 16; i++) j_add(&tab[i], &tab[i - 1], &tab[1]);
  jpt acc;
  memset(&acc, 0, sizeof(acc));
  acc.inf = 1;
  for (int w = 63; w >= 0; w--) {
    for (int d = 0; d < 4; d++) j_double(&acc, &acc);
    int nib = (int)((k->v[w >> 4] >> (4 * (w & 15))) & 15);
    if (nib) j_add(&acc, &acc, &tab[nib]);
  }
  return j_to_affine(&acc);
}

/* --------------------------------------------------------------- SHA-256 */
static const uint32_t SHA_K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_block(uint32_t h[8], const uint8_t* blk) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = ((uint32_t)blk[4 * i] << 24) | ((uint32_t)blk[4 * i + 1] << 16) | ((uint32_t)blk[4 * i + 2] << 8) |
           blk[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = hh + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + SHA_K[i] + w[i];
    uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

void cudasp_oracle_sha256(uint8_t out[32], const uint8_t* msg, size_t len) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t off = 0;
  for (; off + 64 <= len; off += 64) sha256_block(h, msg + off);
  uint8_t tail[128];
  size_t rem = len - off;
  memset(tail, 0, sizeof(tail));
  memcpy(tail, msg + off, rem);
  tail[rem] = 0x80;
  size_t tl = (rem + 9 <= 64) ? 64 : 128;
  uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; i++) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
  sha256_block(h, tail);
  if (tl == 128) sha256_block(h, tail + 64);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)(h[i] >> 24);
    out[4 * i + 1] = (uint8_t)(h[i] >> 16);
    out[4 * i + 2] = (uint8_t)(h[i] >> 8);
    out[4 * i + 3] = (uint8_t)h[i];
  }
}

/* tagged_hash of compute_bip352_expected.py:90-93 */
static void tagged_hash(uint8_t out[32], const char* tag, const uint8_t* msg, size_t len) {
  uint8_t th[32];
  cudasp_oracle_sha256(th, (const uint8_t*)tag, strlen(tag));
  uint8_t buf[64 + 256];
  memcpy(buf, th, 32);
  memcpy(buf + 32, th, 32);
  memcpy(buf + 64, msg, len);
  cudasp_oracle_sha256(out, buf, 64 + len);
}

/* --------------------------------------------------------------- pipeline */
static int64_t upper64(const fe4* x) { return (int64_t)x->v[3]; }

static apt apt_from_le64(const uint8_t* b) {
  apt p;
  fp_from_le(&p.x, b);
  fp_from_le(&p.y, b + 32);
  p.inf = 0;
  return p;
}

/* One row for output indices k = 0..K-1 (cudasp_oracle_options; the
 * reference is K = 1, no negation, int64 compare).  Per k: t_k from
 * ser(S) || ser32(k) (src/cudasp_gpu.cu:261-284 with k instead of the fixed
 * zero), F = t_k G + B (:318-354, :44-71), the base value, then F + L_j for
 * the labels in order (:133-172), then F - L_j when label_negation (the
 * "(and negated)" of :938-939).  values_out[k * (1 + L') + c]; xs_out (may be
 * NULL) the matching 32-byte BE x (zeros for infinity); t_be_out (may be NULL)
 * K digests. */
int cudasp_oracle_row_ex(const uint8_t scan_key_le[32], const uint8_t spend_key_le[64], const uint8_t* label_keys_le,
                         uint32_t label_count, const uint8_t tweak_le[64], const cudasp_oracle_options* opt,
                         uint8_t* t_be_out, uint8_t* xs_out, int64_t* values_out) {
  const uint32_t K = opt ? opt->output_count : 1;
  const int neg = opt && opt->label_negation;
  const uint32_t Lp = neg ? 2 * label_count : label_count;
  fe4 d;
  u256_from_le(&d, scan_key_le);
  apt T = apt_from_le64(tweak_le);
  apt S = pt_mul(&d, &T);
  if (S.inf) return -1;
  apt G;
  G.x = GX;
  G.y = GY;
  G.inf = 0;
  apt B = apt_from_le64(spend_key_le);
  for (uint32_t k = 0; k < K; k++) {
    uint8_t ser[37];
    ser[0] = (uint8_t)(0x02 | (S.y.v[0] & 1));
    u256_to_be(ser + 1, &S.x);
    ser[33] = (uint8_t)(k >> 24); /* ser32(k), big-endian */
    ser[34] = (uint8_t)(k >> 16);
    ser[35] = (uint8_t)(k >> 8);
    ser[36] = (uint8_t)k;
    uint8_t h[32];
    tagged_hash(h, "BIP0352/SharedSecret", ser, 37);
    if (t_be_out) memcpy(t_be_out + 32 * (size_t)k, h, 32);
    fe4 t;
    u256_from_be(&t, h);
    apt P0 = pt_mul(&t, &G);
    apt F = pt_add(&P0, &B);
    if (F.inf) return -1;
    int64_t* v = values_out + (size_t)k * (1 + Lp);
    uint8_t* xs = xs_out ? xs_out + (size_t)k * (1 + Lp) * 32 : NULL;
    v[0] = upper64(&F.x);
    if (xs) u256_to_be(xs, &F.x);
    for (uint32_t c = 0; c < Lp; c++) {
      uint32_t j = c < label_count ? c : c - label_count;
      apt Lj = apt_from_le64(label_keys_le + 64 * (size_t)j);
      if (c >= label_count) fp_sub(&Lj.y, &(fe4){{0, 0, 0, 0}}, &Lj.y); /* -L_j */
      apt FL = pt_add(&F, &Lj);
      v[1 + c] = FL.inf ? CUDASP_ORACLE_LABEL_INFINITY : upper64(&FL.x);
      if (xs) {
        if (FL.inf)
          memset(xs + 32 * (size_t)(1 + c), 0, 32);
        else
          u256_to_be(xs + 32 * (size_t)(1 + c), &FL.x);
      }
    }
  }
  return 0;
}

int cudasp_oracle_row(const uint8_t scan_key_le[32], const uint8_t spend_key_le[64], const uint8_t* label_keys_le,
                      uint32_t label_count, const uint8_t tweak_le[64], uint8_t t_be_out[32], int64_t* values_out) {
  return cudasp_oracle_row_ex(scan_key_le, spend_key_le, label_keys_le, label_count, tweak_le, NULL, t_be_out, NULL,
                              values_out);
}

static int contains(const int64_t* outs, uint32_t off, uint32_t len, int64_t v) {
  for (uint32_t k = 0; k < len; k++)
    if (outs[(size_t)off + k] == v) return 1;
  return 0;
}

static int contains_x(const uint8_t* outs_x, uint32_t off, uint32_t len, const uint8_t x[32]) {
  for (uint32_t k = 0; k < len; k++)
    if (memcmp(outs_x + 32 * ((size_t)off + k), x, 32) == 0) return 1;
  return 0;
}

typedef struct {
  const uint8_t *scan, *spend, *labels, *tweaks;
  uint32_t label_count, begin, end;
  cudasp_oracle_options opt;
  const void* outputs;
  const uint32_t *offs, *lens;
  uint8_t* flags;
  int64_t* values;
  int rc;
} job_t;

static void* run_job(void* arg) {
  job_t* j = (job_t*)arg;
  const uint32_t K = j->opt.output_count;
  const uint32_t W = 1 + (j->opt.label_negation ? 2 : 1) * j->label_count; /* values per output index */
  int64_t* v = (int64_t*)malloc(sizeof(int64_t) * K * W);
  uint8_t* xs = (uint8_t*)malloc(32 * (size_t)K * W);
  j->rc = 0;
  for (uint32_t r = j->begin; r < j->end; r++) {
    if (cudasp_oracle_row_ex(j->scan, j->spend, j->labels, j->label_count, j->tweaks + 64 * (size_t)r, &j->opt,
                             NULL, xs, v) != 0) {
      j->rc = -1;
      if (j->flags) j->flags[r] = 0;
      continue;
    }
    if (j->values) memcpy(j->values + (size_t)r * K * W, v, sizeof(int64_t) * K * W);
    if (j->flags) {
      /* CheckMatchesWithLabelsKernel: base value first, then labels in order;
       * a row matches if any output index does */
      int hit = 0;
      for (uint32_t q = 0; !hit && q < K * W; q++) {
        if (q % W != 0 && v[q] == CUDASP_ORACLE_LABEL_INFINITY) continue;
        hit = j->opt.full_x ? contains_x((const uint8_t*)j->outputs, j->offs[r], j->lens[r], xs + 32 * (size_t)q)
                            : contains((const int64_t*)j->outputs, j->offs[r], j->lens[r], v[q]);
      }
      j->flags[r] = (uint8_t)hit;
    }
  }
  free(v);
  free(xs);
  return NULL;
}

int cudasp_oracle_scan_ex(const uint8_t scan_key_le[32], const uint8_t spend_key_le[64], const uint8_t* label_keys_le,
                          uint32_t label_count, const uint8_t* tweaks_le, uint32_t n, const cudasp_oracle_options* opt,
                          const void* outputs, const uint32_t* offsets, const uint32_t* lengths, uint8_t* flags_out,
                          int64_t* values_out, int threads) {
  cudasp_oracle_options o = {1, 0, 0};
  if (opt) o = *opt;
  if (o.output_count < 1) return -2;
  if (threads < 1) threads = 1;
  if ((uint32_t)threads > n) threads = n ? (int)n : 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  job_t* jobs = (job_t*)malloc(sizeof(job_t) * threads);
  for (int i = 0; i < threads; i++) {
    job_t* j = &jobs[i];
    j->scan = scan_key_le; j->spend = spend_key_le; j->labels = label_keys_le; j->tweaks = tweaks_le;
    j->label_count = label_count;
    j->opt = o;
    j->begin = (uint32_t)((uint64_t)n * i / threads);
    j->end = (uint32_t)((uint64_t)n * (i + 1) / threads);
    j->outputs = outputs; j->offs = offsets; j->lens = lengths;
    j->flags = flags_out; j->values = values_out;
    pthread_create(&th[i], NULL, run_job, j);
  }
  int rc = 0;
  for (int i = 0; i < threads; i++) {
    pthread_join(th[i], NULL);
    if (jobs[i].rc) rc = jobs[i].rc;
  }
  free(th);
  free(jobs);
  return rc;
}

int cudasp_oracle_scan(const uint8_t scan_key_le[32], const uint8_t spend_key_le[64], const uint8_t* label_keys_le,
                       uint32_t label_count, const uint8_t* tweaks_le, uint32_t n, const int64_t* outputs,
                       const uint32_t* offsets, const uint32_t* lengths, uint8_t* flags_out, int64_t* values_out,
                       int threads) {
  return cudasp_oracle_scan_ex(scan_key_le, spend_key_le, label_keys_le, label_count, tweaks_le, n, NULL, outputs,
                               offsets, lengths, flags_out, values_out, threads);
}

/* Synthetic tweak of bench/test tables: T_i = (s0 + i) * G,
 * s0 given as 32 LE bytes (already reduced), written as 64 LE bytes x || y. */
int cudasp_oracle_synth_tweak(const uint8_t s0_le[32], uint64_t index, uint8_t out_le[64]) {
  fe4 s, add = {{index, 0, 0, 0}};
  u256_from_le(&s, s0_le);
  if (u256_add(&s, &s, &add) || u256_cmp(&s, &N_ORD) >= 0) u256_sub(&s, &s, &N_ORD);
  apt G;
  G.x = GX;
  G.y = GY;
  G.inf = 0;
  apt T = pt_mul(&s, &G);
  if (T.inf) return -1;
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 8; k++) {
      out_le[8 * i + k] = (uint8_t)(T.x.v[i] >> (8 * k));
      out_le[32 + 8 * i + k] = (uint8_t)(T.y.v[i] >> (8 * k));
    }
  return 0;
}

/* Field multiply mod p on LE byte strings, for cross-checks. */
void cudasp_oracle_fp_mul(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]) {
  fe4 x, y, r;
  fp_from_le(&x, a);
  fp_from_le(&y, b);
  fp_mul(&r, &x, &y);
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 8; k++) out[8 * i + k] = (uint8_t)(r.v[i] >> (8 * k));
}
