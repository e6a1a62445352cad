// Host-side preparation of one query's constants for the scan kernels
// (the bind-time work of CudaspScanBind + LaunchBatchScan in the reference,
// src/cudasp_extension.cu:420-509 and src/cudasp_gpu.cu:445-669): SHA-256
// midstate of the tag block, GLV split + wNAF of the scan key, the spend key
// with 2^256 G (and -G) folded in, normalized label keys, and the window bases
// 2^(16 i) G of the fixed-base table.  Shared by the HIP library and the CPU
// emulation harness (tests/native), so both run the same host logic.
#pragma once
#include <stdint.h>
#include <string.h>

#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "../../include/cudasp_abi.h"
#include "scalar_host.hpp"
#include "scan_rows.hpp"

namespace cudasp {
namespace {

// Complete affine addition on the host (normalized inputs), inf flags.
struct HPoint {
  ge p;
  bool inf;
};

HPoint hp_add(const HPoint& a, const HPoint& b) {
  if (a.inf) return b;
  if (b.inf) return a;
  fe num, den;
  if (fe_equal_norm(a.p.x, b.p.x)) {
    if (!fe_equal_norm(a.p.y, b.p.y)) return HPoint{ge{}, true};
    fe_sqr(num, a.p.x);
    fe_mul_int(num, num, 3);
    fe_add(den, a.p.y, a.p.y);
  } else {
    fe_sub<1>(num, b.p.y, a.p.y);
    fe_sub<1>(den, b.p.x, a.p.x);
  }
  fe inv, lam, x3, y3, t;
  fe_inv(inv, den);
  fe_mul(lam, num, inv);
  fe_sqr(x3, lam);
  fe_sub<1>(x3, x3, a.p.x);
  fe_sub<1>(x3, x3, b.p.x);
  fe_normalize(x3);
  fe_sub<1>(t, a.p.x, x3);
  fe_mul(y3, lam, t);
  fe_sub<1>(y3, y3, a.p.y);
  fe_normalize(y3);
  HPoint r;
  r.p.x = x3;
  r.p.y = y3;
  r.inf = false;
  return r;
}

HPoint hp_neg(const HPoint& a) {
  HPoint r = a;
  if (!a.inf) {
    fe_negate<1>(r.p.y, a.p.y);
    fe_normalize(r.p.y);
  }
  return r;
}

void hp_words(uint32_t w[16], const HPoint& a) {
  fe_to_u32x8(w, a.p.x);
  fe_to_u32x8(w + 8, a.p.y);
}

HPoint hp_from_bytes(const uint8_t b[64]) {
  uint32_t w[16];
  for (int i = 0; i < 16; i++)
    w[i] = (uint32_t)b[4 * i] | ((uint32_t)b[4 * i + 1] << 8) | ((uint32_t)b[4 * i + 2] << 16) |
           ((uint32_t)b[4 * i + 3] << 24);
  HPoint r;
  fe_from_u32x8(r.p.x, w);
  fe_from_u32x8(r.p.y, w + 8);
  fe_normalize(r.p.x);
  fe_normalize(r.p.y);
  r.inf = false;
  return r;
}

HPoint hp_generator() {
  static const uint8_t gbytes[64] = {
      // x = 79BE667E F9DCBBAC 55A06295 CE870B07 029BFCDB 2DCE28D9 59F2815B 16F81798 (LE)
      0x98, 0x17, 0xf8, 0x16, 0x5b, 0x81, 0xf2, 0x59, 0xd9, 0x28, 0xce, 0x2d, 0xdb, 0xfc, 0x9b, 0x02,
      0x07, 0x0b, 0x87, 0xce, 0x95, 0x62, 0xa0, 0x55, 0xac, 0xbb, 0xdc, 0xf9, 0x7e, 0x66, 0xbe, 0x79,
      // y = 483ADA77 26A3C465 5DA4FBFC 0E1108A8 FD17B448 A6855419 9C47D08F FB10D4B8 (LE)
      0xb8, 0xd4, 0x10, 0xfb, 0x8f, 0xd0, 0x47, 0x9c, 0x19, 0x54, 0x85, 0xa6, 0x48, 0xb4, 0x17, 0xfd,
      0xa8, 0x08, 0x11, 0x0e, 0xfc, 0xfb, 0xa4, 0x5d, 0x65, 0xc4, 0xa3, 0x26, 0x77, 0xda, 0x3a, 0x48};
  return hp_from_bytes(gbytes);
}

void sha256_bytes(uint8_t out[32], const uint8_t* msg, size_t len) {
  uint32_t s[8];
  sha256_init(s);
  std::vector<uint8_t> buf(msg, msg + len);
  buf.push_back(0x80);
  while (buf.size() % 64 != 56) buf.push_back(0);
  uint64_t bits = (uint64_t)len * 8;
  for (int i = 7; i >= 0; i--) buf.push_back((uint8_t)(bits >> (8 * i)));
  for (size_t off = 0; off < buf.size(); off += 64) {
    uint32_t w[16];
    for (int i = 0; i < 16; i++)
      w[i] = ((uint32_t)buf[off + 4 * i] << 24) | ((uint32_t)buf[off + 4 * i + 1] << 16) |
             ((uint32_t)buf[off + 4 * i + 2] << 8) | buf[off + 4 * i + 3];
    sha256_compress(s, w);
  }
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)(s[i] >> 24);
    out[4 * i + 1] = (uint8_t)(s[i] >> 16);
    out[4 * i + 2] = (uint8_t)(s[i] >> 8);
    out[4 * i + 3] = (uint8_t)s[i];
  }
}

// SHA-256 state after the constant block SHA256(tag) || SHA256(tag).
void bip352_midstate(uint32_t mid[8]) {
  static const char tag[] = "BIP0352/SharedSecret";
  uint8_t th[32];
  sha256_bytes(th, (const uint8_t*)tag, 20);
  uint32_t w[16];
  for (int i = 0; i < 8; i++) {
    w[i] = ((uint32_t)th[4 * i] << 24) | ((uint32_t)th[4 * i + 1] << 16) | ((uint32_t)th[4 * i + 2] << 8) |
           th[4 * i + 3];
    w[8 + i] = w[i];
  }
  sha256_init(mid);
  sha256_compress(mid, w);
}


// Fixed-base window bases 2^(bits i) G, i = 0 .. windows - 1, as 16
// normalized words each (host, once per table build).
inline std::vector<uint32_t> fb_window_bases(int bits = FB_BITS) {
  const int windows = (256 + bits - 1) / bits;
  std::vector<uint32_t> bases((size_t)windows * 16);
  HPoint cur = hp_generator();
  for (int i = 0; i < windows; i++) {
    hp_words(&bases[(size_t)i * 16], cur);
    for (int d = 0; d < bits; d++) cur = hp_add(cur, cur);
  }
  return bases;
}

// The same bases with their doubles: 32 words per window, 2^(bits i) G then
// 2^(bits i + 1) G (k_fb_build_runs: the step between consecutive odd
// multiples).
inline std::vector<uint32_t> fb_window_bases_doubled(int bits) {
  const int windows = (256 + bits - 1) / bits;
  std::vector<uint32_t> out((size_t)windows * 32);
  HPoint cur = hp_generator();
  for (int i = 0; i < windows; i++) {
    const HPoint two = hp_add(cur, cur);
    hp_words(&out[(size_t)i * 32], cur);
    hp_words(&out[(size_t)i * 32 + 16], two);
    cur = two;
    for (int d = 1; d < bits; d++) cur = hp_add(cur, cur);
  }
  return out;
}

// Overwrite memory that held key material (not optimised away).
inline void wipe_bytes(void* p, size_t n) {
  volatile uint8_t* v = static_cast<volatile uint8_t*>(p);
  for (size_t i = 0; i < n; i++) v[i] = 0;
}

// A small process-wide cache of scan_digits: the search over ~290 GLV
// decompositions costs ~0.3 ms of host time per key, paid at every new
// scanner's bind otherwise (a wallet's key is scanned query after query).
// The key itself is not stored: entries are found by SHA-256(salt || d) with
// a per-process random salt, compared in constant time.  The digits are
// equivalent to the key, so entries are wiped on eviction and by
// scan_digits_cache_clear (cudasp_tf_release_pool, library unload).
struct ScanDigitsCache {
  struct Entry {
    uint8_t tag[32];
    std::vector<int8_t> naf;
    uint32_t len;
  };
  std::mutex mu;
  std::vector<Entry> entries;  // most recent last, at most 16
  uint8_t salt[32];
  ScanDigitsCache() {
    std::random_device rd;
    for (int i = 0; i < 32; i += 4) {
      const uint32_t v = rd();
      memcpy(salt + i, &v, 4);
    }
  }
  ~ScanDigitsCache() { clear(); }
  static void wipe(Entry& e) {
    wipe_bytes(e.tag, sizeof(e.tag));
    if (!e.naf.empty()) wipe_bytes(e.naf.data(), e.naf.size());
    e.len = 0;
  }
  void clear() {
    std::lock_guard<std::mutex> lk(mu);
    for (Entry& e : entries) wipe(e);
    entries.clear();
  }
  void tag_of(const host::Big<8>& d, uint8_t tag[32]) const {
    uint8_t buf[64];
    memcpy(buf, salt, 32);
    for (int i = 0; i < 8; i++) memcpy(buf + 32 + 4 * i, &d.w[i], 4);
    sha256_bytes(tag, buf, sizeof(buf));
    wipe_bytes(buf, sizeof(buf));
  }
  static bool tag_eq(const uint8_t* a, const uint8_t* b) {
    uint8_t x = 0;
    for (int i = 0; i < 32; i++) x |= a[i] ^ b[i];
    return x == 0;
  }
};

inline ScanDigitsCache& scan_digits_cache() {
  static ScanDigitsCache c;
  return c;
}

inline void scan_digits_cache_clear() { scan_digits_cache().clear(); }

inline bool scan_digits_cached(const host::Big<8>& d, std::vector<int8_t>& naf, uint32_t* naf_len) {
  ScanDigitsCache& c = scan_digits_cache();
  uint8_t tag[32];
  c.tag_of(d, tag);
  {
    std::lock_guard<std::mutex> lk(c.mu);
    int hit = -1;
    for (size_t i = 0; i < c.entries.size(); i++)  // every entry compared: no early exit on the key
      if (ScanDigitsCache::tag_eq(c.entries[i].tag, tag)) hit = (int)i;
    if (hit >= 0) {
      naf = c.entries[hit].naf;
      *naf_len = c.entries[hit].len;
      wipe_bytes(tag, sizeof(tag));
      return true;
    }
  }
  if (host::scan_digits(d, naf.data(), NAF_MAX, naf_len) != 0) return false;
  std::lock_guard<std::mutex> lk(c.mu);
  if (c.entries.size() >= 16) {
    ScanDigitsCache::wipe(c.entries.front());
    c.entries.erase(c.entries.begin());
  }
  ScanDigitsCache::Entry e;
  memcpy(e.tag, tag, 32);
  e.naf = naf;
  e.len = *naf_len;
  c.entries.push_back(std::move(e));
  wipe_bytes(tag, sizeof(tag));
  return true;
}

// opt (may be NULL = the reference's semantics): K and full_x go to the
// constants; with label_negation the label buffer holds L_0..L_(L-1) then
// -L_0..-L_(L-1) and k.label_count = 2 L.
inline int prepare_scan(const uint8_t scan_private_key[32], const uint8_t spend_public_key[64],
                        const uint8_t* label_keys, uint32_t label_count, ScanConsts& k, std::vector<int8_t>& naf,
                        std::vector<uint32_t>& labels, std::string& err, const cudasp_scan_options* opt = nullptr) {
  const uint32_t K = opt ? opt->output_count : 1u;
  if (K < 1 || K > CUDASP_MAX_OUTPUT_COUNT) {
    err = "output_count must be between 1 and " + std::to_string(CUDASP_MAX_OUTPUT_COUNT);
    return CUDASP_ERR_INVALID_ARG;
  }
  const bool negate = opt && opt->label_negation;
  host::Big<8> d = host::big_zero<8>();
  for (int i = 0; i < 32; i++) d.w[i / 4] |= (uint32_t)scan_private_key[i] << (8 * (i % 4));
  d = host::scalar_reduce(d);
  if (host::big_is_zero(d)) {
    err = "scan_private_key is 0 mod n";
    return CUDASP_ERR_INVALID_ARG;
  }
  naf.assign(2 * NAF_MAX, 0);
  uint32_t naf_len = 0;
  if (!scan_digits_cached(d, naf, &naf_len)) {
    err = "GLV split out of range";
    return CUDASP_ERR_INVALID_ARG;
  }
  memset(&k, 0, sizeof(k));
  bip352_midstate(k.mid);
  k.naf_len = naf_len;
  k.label_count = negate ? 2 * label_count : label_count;
  k.output_count = K;
  k.full_x = opt && opt->full_x ? 1u : 0u;
  hp_words(k.spend, hp_from_bytes(spend_public_key));
  labels.assign(16 * (size_t)(k.label_count ? k.label_count : 1), 0);
  for (uint32_t j = 0; j < label_count; j++) {
    HPoint Lj = hp_from_bytes(label_keys + 64 * (size_t)j);
    hp_words(&labels[16 * j], Lj);
    if (negate) hp_words(&labels[16 * ((size_t)label_count + j)], hp_neg(Lj));
  }
  return CUDASP_OK;
}

}  // namespace
}  // namespace cudasp
