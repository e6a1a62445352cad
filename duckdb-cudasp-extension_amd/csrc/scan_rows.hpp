// Per-row bodies of the cudasp_scan hot path, written once as
// __host__ __device__ code: the HIP kernels in scan_kernels.hip are thin
// grid-stride wrappers around them, and tests/native/cudasp_emu.cpp runs the
// very same functions on the CPU (with magnitude checks) to debug the kernel
// math without a GPU.
//
// Pipeline per row (semantics of /root/reference/src/cudasp_gpu.cu):
//   stage A  row_shared_secret  S = d*T, ser = 02|03 || x || 00000000,
//            t = SHA256(H(tag)||H(tag)||ser)                     (:236-314,:784)
//   stage B  row_match          F = t*G + B, v = int64(F.x >> 192), labels
//            v_j = int64((F + L_j).x >> 192), compare with outputs   (:74-178,:318-354)
#pragma once
#include "secp256k1_group.hpp"
#include "sha256.hpp"

namespace cudasp {

// Variable-base window: odd multiples 1,3,...,15 of T (width-5 NAF digits).
constexpr int VB_ENTRIES = 8;
constexpr int NAF_MAX = 136;
// Fixed-base table: W windows of w-bit odd digits, each with 2^(w-1) odd
// multiples (2j+1) 2^(w i) G, 64 bytes per entry.  The odd representative t'
// of t mod n is sum_i d_i 2^(w i) (fixed_base_mul), so P0 = t G costs W
// gathers and W - 1 mixed additions.  The width is a per-scanner runtime
// choice among the prebuilt widths (FbWidth below; cudasp_scanner_set_fixed_base_bits):
//   22 bits: 12 windows, 1.5 GiB per device  (the default, CUDASP_FB_BITS)
//   26 bits: 10 windows, 21.5 GB per device  (~1.5% faster end to end,
//            profiles/r01_stage_ab_fb_windows26.txt: 22 -> 24 -> 26 bits
//            158.4 -> 160.2 -> 160.9 M tx/s, stage B -13%)
// FB_BITS / FB_WINDOWS / FB_ENTRIES name the default width.
#ifndef CUDASP_FB_BITS
#define CUDASP_FB_BITS 22
#endif
template <int BITS>
struct FbWidth {
  static_assert(BITS >= 4 && BITS <= 27, "fixed-base window width");
  static constexpr int WINDOWS = (256 + BITS - 1) / BITS;
  static constexpr uint32_t ENTRIES = 1u << (BITS - 1);
  // entries of the top window a scalar below 2^256 can reach: its digit is
  // 2 b + 1 with b = t' >> (BITS (WINDOWS - 1) + 1) < 2^(255 - BITS (WINDOWS - 1))
  static constexpr uint32_t TOP_ENTRIES = 1u << (255 - BITS * (WINDOWS - 1));
};
constexpr int FB_BITS = CUDASP_FB_BITS;
static_assert(FB_BITS == 22 || FB_BITS == 26, "default fixed-base width must be a prebuilt one (22 or 26)");
constexpr int FB_WINDOWS = FbWidth<FB_BITS>::WINDOWS;
constexpr uint32_t FB_ENTRIES = FbWidth<FB_BITS>::ENTRIES;
constexpr int FB_WORDS = 16;

// Per-query constants, passed to the kernels by value.
struct ScanConsts {
  uint32_t mid[8];      // SHA-256 state after the constant block H(tag)||H(tag)
  uint32_t spend[16];   // B, the spend public key (normalized)
  uint32_t naf_len;     // digits in each GLV half
  uint32_t label_count; // label keys in the label buffer (negated copies included)
  // Protocol variants (cudasp_scan_options, include/cudasp_abi.h; the reference
  // is output_count 1, full_x 0):
  uint32_t output_count;  // K: output indices k = 0..K-1 hashed per row
  uint32_t full_x;        // outputs are 32-byte big-endian x-only keys
  // The spend key folded into the fixed-base table's top window (nullptr:
  // added on its own): TOP_ENTRIES entries (2j+1) 2^(w (W-1)) G + B, then as
  // many with - B (fixed_base_mul, fb_fold_entry).  Set by the scanner for an
  // on-curve B and an HBM width only; never by prepare_scan.
  const uint32_t* fb_top;
};

// beta, a primitive cube root of unity mod p: (beta*x, y) = lambda*(x, y).
CUDASP_HD void fe_beta(fe& r) {
  const uint32_t w[8] = {0x719501eeu, 0xc1396c28u, 0x12f58995u, 0x9cf04975u,
                         0xac3434e9u, 0x6e64479eu, 0x657c0710u, 0x7ae96a2bu};
  fe_from_u32x8(r, w);
}

// Column-major scratch: element k of a row lives at s[k * stride + slot].
struct Scratch {
  uint32_t* s;
  uint32_t stride;
  uint32_t slot;
#if defined(__HIP_DEVICE_COMPILE__)
  __amdgpu_buffer_rsrc_t rsrc;
#endif
};

// Word w of a slot lives at s[w * stride + slot] (coalesced across a wave).
// On the device every access is a buffer load/store with the column offset
// w * stride * 4 in a scalar register and the lane offset slot * 4 in a VGPR:
// no 64-bit per-lane address exists for the compiler to hoist out of the loops
// and keep live (that spilled registers in stage A).  The scanner keeps each
// scratch buffer below 4 GiB (32-bit offsets).
CUDASP_HD Scratch make_scratch(uint32_t* s, uint32_t stride, uint32_t slot) {
  Scratch sc;
  sc.s = s;
  sc.stride = stride;
  sc.slot = slot;
#if defined(__HIP_DEVICE_COMPILE__)
  // word 3 = 0x00020000: raw 32-bit buffer access on gfx9-family (CDNA) parts
  sc.rsrc = __builtin_amdgcn_make_buffer_rsrc(s, 0, (int)0xFFFFFFFFu, 0x00020000);
#endif
  return sc;
}

// Cache policy of the scratch loads / stores (gfx950 CPol bits: 1 = sc0,
// 2 = nt, 16 = sc1).
#ifndef CUDASP_SCR_LOAD_CPOL
#define CUDASP_SCR_LOAD_CPOL 0
#endif
#ifndef CUDASP_SCR_STORE_CPOL
#define CUDASP_SCR_STORE_CPOL 0
#endif

CUDASP_HD void scr_store(const Scratch& sc, int base, const fe& a) {
#pragma unroll
  for (int l = 0; l < FE_LIMBS; l++) {
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_raw_buffer_store_b32(a.n[l], sc.rsrc, sc.slot * 4u, (uint32_t)(base + l) * sc.stride * 4u, CUDASP_SCR_STORE_CPOL);
#else
    sc.s[(size_t)(base + l) * sc.stride + sc.slot] = a.n[l];
#endif
  }
}

CUDASP_HD void scr_load(fe& a, const Scratch& sc, int base) {
#pragma unroll
  for (int l = 0; l < FE_LIMBS; l++) {
#if defined(__HIP_DEVICE_COMPILE__)
    a.n[l] = __builtin_amdgcn_raw_buffer_load_b32(sc.rsrc, sc.slot * 4u, (uint32_t)(base + l) * sc.stride * 4u,
                                                  CUDASP_SCR_LOAD_CPOL);
#else
    a.n[l] = sc.s[(size_t)(base + l) * sc.stride + sc.slot];
#endif
  }
}

// Scratch layout of stage A (u32 words per row).
// (FE_LIMBS words per field element)
constexpr int FW = FE_LIMBS;
// Stage-A ladder in the doubled-Y form (secp256k1_group29.hpp, 9 x 29 only).
#ifndef LADDER_YH
#define LADDER_YH (CUDASP_FE_LIMBS == 9)
#endif
constexpr int VB_ENTRY_X(int e) { return e * 2 * FW; }
constexpr int VB_ENTRY_Y(int e) { return e * 2 * FW + FW; }
constexpr int VB_ZR(int i) { return VB_ENTRIES * 2 * FW + i * FW; }
constexpr int VB_CZ = VB_ENTRIES * 2 * FW + (VB_ENTRIES - 1) * FW;
// beta * x of every entry (the x of phi(entry)), when CUDASP_PHI_TABLE.
#ifndef CUDASP_PHI_TABLE
#define CUDASP_PHI_TABLE 1
#endif
constexpr int VB_ENTRY_XB(int e) { return VB_CZ + FW + e * FW; }
constexpr int VB_SCRATCH_WORDS = VB_CZ + FW + (CUDASP_PHI_TABLE ? VB_ENTRIES * FW : 0);

CUDASP_HD int8_t uniform_digit(const int8_t* p, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
  return (int8_t)__builtin_amdgcn_readfirstlane((int)p[i]);
#else
  return p[i];
#endif
}

// Where the odd-multiple table's y coordinates live (row_shared_secret_point_t).
// ScrY: all in scratch.  LdsY<N>: entries 0 .. N-1 in the workgroup's LDS
// (word w of this thread at p[w * stride], stride = the threads sharing the
// array -- the block's, or the wave's 64 -- so a wave's accesses are
// conflict-free), the rest in scratch: y is read by every
// addition (x only by its half's), so an LDS word of y saves the most
// scratch traffic, which costs clock under the power cap.
struct ScrY {
  CUDASP_HD bool has(int) const { return false; }
  CUDASP_HD void store(int, const fe&) const {}
  CUDASP_HD void load(fe&, int) const {}
};

template <int N>
struct LdsY {
  uint32_t* p;
  uint32_t stride;
  CUDASP_HD bool has(int e) const { return e < N; }
  CUDASP_HD void store(int e, const fe& a) const {
#pragma unroll
    for (int l = 0; l < FE_LIMBS; l++) p[(uint32_t)(e * FE_LIMBS + l) * stride] = a.n[l];
  }
  CUDASP_HD void load(fe& a, int e) const {
#pragma unroll
    for (int l = 0; l < FE_LIMBS; l++) a.n[l] = p[(uint32_t)(e * FE_LIMBS + l) * stride];
  }
};

template <class YTab>
CUDASP_HD void tab_store_y(const Scratch& sc, const YTab& yt, int e, const fe& a) {
  if (yt.has(e)) yt.store(e, a);
  else scr_store(sc, VB_ENTRY_Y(e), a);
}

template <class YTab>
CUDASP_HD void tab_load_y(fe& a, const Scratch& sc, const YTab& yt, int e) {
  if (yt.has(e)) yt.load(a, e);
  else scr_load(a, sc, VB_ENTRY_Y(e));
}

// A ladder hook that does nothing (row_shared_secret_point_t).
struct NoTick {
  CUDASP_HD void ladder(int, uint32_t) const {}
};

// Stage A, first half: S = d T as a Jacobian point of the original curve.
// tx, ty: the tweak point, 8 LE u32 words each (normal form, the reference's
// layout).  naf: 2 * NAF_MAX digits (GLV half 1, then half 2, signs folded in).
// tick.ladder(i, naf_len) runs every 16 ladder steps, i the digits still to
// go (the persistent kernels re-prioritise their waves there).
template <class Tick, class YTab = ScrY>
CUDASP_HD void row_shared_secret_point_t(gej& R, const uint32_t tx[8], const uint32_t ty[8], const int8_t* naf,
                                         uint32_t naf_len, const Scratch& sc, const Tick& tick,
                                         const YTab& yt = YTab()) {
  ge T;
  fe_from_u32x8(T.x, tx);
  fe_from_u32x8(T.y, ty);

  // --- odd multiples {1,3,...,15} T with one shared Z (no inversion) --------
  fe beta;
  fe_beta(beta);
  // Co-Z arithmetic (Meloni): DBLU gives D = 2T and T with a common Z, then
  // each ZADDU adds D to the last odd multiple and moves D to the new Z (5M+2S
  // per entry instead of a mixed addition's 8M+3S).  The entries, each with its
  // own Z, are then brought to the Z of the last one (Zg) through the recorded
  // Z ratios.  With Zg taken as 1 every entry is affine on an isomorphic curve,
  // the main loop uses mixed additions only, and the final Z is multiplied back
  // by Zg.
  {
    gej D, acc;
    gej_dblu(D, acc, T);
    scr_store(sc, VB_ENTRY_X(0), acc.x);
    tab_store_y(sc, yt, 0, acc.y);
    for (int e = 1; e < VB_ENTRIES; e++) {
      fe zr;
      gej nxt;
      gej_zaddu(nxt, D, acc, &zr);
      acc = nxt;
      if (e == VB_ENTRIES - 1) {  // the only entry not rescaled below
        fe_normalize_weak(acc.x);
        fe_normalize_weak(acc.y);
#if LADDER_YH
        fe_add(acc.y, acc.y, acc.y);
#endif
#if CUDASP_PHI_TABLE
        fe xb;
        fe_mul(xb, acc.x, beta);
        scr_store(sc, VB_ENTRY_XB(e), xb);
#endif
      }
      scr_store(sc, VB_ENTRY_X(e), acc.x);
      tab_store_y(sc, yt, e, acc.y);
      scr_store(sc, VB_ZR(e - 1), zr);
    }
    scr_store(sc, VB_CZ, acc.z);  // Zg
  }
  {
    fe ratio;
    scr_load(ratio, sc, VB_ZR(VB_ENTRIES - 2));
    for (int e = VB_ENTRIES - 2; e >= 0; e--) {
      fe x, y, r2, r3;
      scr_load(x, sc, VB_ENTRY_X(e));
      tab_load_y(y, sc, yt, e);
      fe_sqr(r2, ratio);
      fe_mul(r3, r2, ratio);
      fe_mul(x, x, r2);
#if LADDER_YH
      fe_add(r3, r3, r3);  // entries hold 2y (the ladder's Yh form)
#endif
      fe_mul(y, y, r3);
      scr_store(sc, VB_ENTRY_X(e), x);
      tab_store_y(sc, yt, e, y);
#if CUDASP_PHI_TABLE
      fe_mul(x, x, beta);
      scr_store(sc, VB_ENTRY_XB(e), x);
#endif
      if (e > 0) {
        fe z;
        scr_load(z, sc, VB_ZR(e - 1));
        fe_mul(ratio, ratio, z);
      }
    }
  }

  // --- S'' = k1*T'' + k2*phi(T'') with uniform NAF digits -------------------
  // LADDER_YH: R holds (X, 2Y, Z) of sgn * R_true; the doubling returns the
  // negated double, so sgn flips with every doubling and an addition adds the
  // entry with its digit's sign times sgn (wave-uniform, like the digits).
  bool inf = true;
  bool sgn_neg = false;
#if LADDER_YH && CUDASP_PHI_TABLE && CUDASP_PREFETCH_ENTRY
  // The table entry of an iteration's first addition is loaded BEFORE its
  // doubling, so the load's latency runs under the doubling's ~900
  // instructions (the digits are wave-uniform, so is the choice).
  for (int i = (int)naf_len - 1; i >= 0; --i) {
    if ((i & 15) == 0) tick.ladder(i, naf_len);
    const int d0 = uniform_digit(naf, i), d1 = uniform_digit(naf, NAF_MAX + i);
    const int hf = d0 != 0 ? 0 : (d1 != 0 ? 1 : -1);
    ge Pn;
    if (hf >= 0) {
      const int d = hf ? d1 : d0;
      const int e = (d < 0 ? -d : d) >> 1;
      scr_load(Pn.x, sc, hf ? VB_ENTRY_XB(e) : VB_ENTRY_X(e));
      tab_load_y(Pn.y, sc, yt, e);
    }
    if (!inf) {
      gej_double_neg_yh(R, R);
      sgn_neg = !sgn_neg;
    }
#pragma unroll
    for (int half = 0; half < 2; half++) {
      const int d = half ? d1 : d0;
      if (d != 0) {
        ge P;
        if (half == hf) {
          P = Pn;
        } else {
          const int e = (d < 0 ? -d : d) >> 1;
          scr_load(P.x, sc, VB_ENTRY_XB(e));
          tab_load_y(P.y, sc, yt, e);
        }
        if ((d < 0) != sgn_neg) fe_negate<2>(P.y, P.y);
        if (inf) {
          gej_set_ge(R, P);
          fe_normalize_weak(R.y);
          inf = false;
        } else {
          gej_add_ge_yh(R, R, P);
        }
      }
    }
  }
#else
  for (int i = (int)naf_len - 1; i >= 0; --i) {
    if ((i & 15) == 0) tick.ladder(i, naf_len);
#if LADDER_YH
    if (!inf) {
      gej_double_neg_yh(R, R);
      sgn_neg = !sgn_neg;
    }
#else
    if (!inf) gej_double(R, R);
#endif
#pragma unroll
    for (int half = 0; half < 2; half++) {
      int d = uniform_digit(naf, half * NAF_MAX + i);
      if (d != 0) {
        int e = (d < 0 ? -d : d) >> 1;
        ge P;
#if CUDASP_PHI_TABLE
        scr_load(P.x, sc, half ? VB_ENTRY_XB(e) : VB_ENTRY_X(e));
#else
        scr_load(P.x, sc, VB_ENTRY_X(e));
        if (half) fe_mul(P.x, P.x, beta);
#endif
        tab_load_y(P.y, sc, yt, e);
#if LADDER_YH
        if ((d < 0) != sgn_neg) fe_negate<2>(P.y, P.y);
        if (inf) {
          gej_set_ge(R, P);
          fe_normalize_weak(R.y);
          inf = false;
        } else {
          gej_add_ge_yh(R, R, P);
        }
#else
        if (d < 0) ge_neg(P, P);
        if (inf) {
          gej_set_ge(R, P);
          inf = false;
        } else {
          gej_add_ge(R, R, P);
        }
#endif
      }
    }
  }
#endif  // CUDASP_PREFETCH_ENTRY
#if LADDER_YH
  fe_half(R.y, R.y);                              // Y = Yh / 2
  if (sgn_neg) fe_negate<2>(R.y, R.y);            // R_true
#endif


  // --- back to the original curve: Z times the common table Z -------------
  fe cz;
  scr_load(cz, sc, VB_CZ);
  fe_mul(R.z, R.z, cz);
}

CUDASP_HD void row_shared_secret_point(gej& R, const uint32_t tx[8], const uint32_t ty[8], const int8_t* naf,
                                       uint32_t naf_len, const Scratch& sc) {
  row_shared_secret_point_t(R, tx, ty, naf, naf_len, sc, NoTick());
}

// Stage A, second half: from S (Jacobian) and 1/Z, the affine x (8 LE words)
// and the parity of y.
CUDASP_HD uint32_t row_shared_secret_affine(uint32_t sx[8], const gej& R, const fe& zi) {
  ge S;
  gej_to_ge_zinv(S, R, zi);
  uint32_t sy[8];
  fe_to_u32x8(sx, S.x);
  fe_to_u32x8(sy, S.y);
  return sy[0] & 1u;
}

// Serialize and hash (output index 0, the reference's).  Writes t (8 LE words
// of the BE digest read as an integer).
CUDASP_HD void row_shared_secret_finish(uint32_t t_out[8], const gej& R, const fe& zi, const uint32_t mid[8]) {
  uint32_t sx[8];
  uint32_t y_odd = row_shared_secret_affine(sx, R, zi);
  bip352_shared_secret_hash(t_out, mid, sx, y_odd);
}

// Stage A for one row (one inversion per row).
CUDASP_HD void row_shared_secret(uint32_t t_out[8], const uint32_t tx[8], const uint32_t ty[8],
                                 const int8_t* naf, uint32_t naf_len, const uint32_t mid[8],
                                 const Scratch& sc) {
  gej R;
  row_shared_secret_point(R, tx, ty, naf, naf_len, sc);
  fe zi;
  fe_inv(zi, R.z);
  row_shared_secret_finish(t_out, R, zi, mid);
}

// --- pending points: K rows per thread share one field inversion ------------
// Per pending row j, PEND_WORDS scratch words from `base`: X, Y, Z, then the
// prefix product (replaced by 1/Z by pend_invert).
constexpr int PEND_WORDS = 4 * FW;
CUDASP_HD int PEND_X(int base, int j) { return base + PEND_WORDS * j; }
CUDASP_HD int PEND_Y(int base, int j) { return base + PEND_WORDS * j + FW; }
CUDASP_HD int PEND_Z(int base, int j) { return base + PEND_WORDS * j + 2 * FW; }
CUDASP_HD int PEND_ZI(int base, int j) { return base + PEND_WORDS * j + 3 * FW; }

CUDASP_HD void pend_store(const Scratch& sc, int base, int j, const gej& R) {
  scr_store(sc, PEND_X(base, j), R.x);
  scr_store(sc, PEND_Y(base, j), R.y);
  scr_store(sc, PEND_Z(base, j), R.z);
}

CUDASP_HD void pend_load(gej& R, const Scratch& sc, int base, int j) {
  scr_load(R.x, sc, PEND_X(base, j));
  scr_load(R.y, sc, PEND_Y(base, j));
  scr_load(R.z, sc, PEND_Z(base, j));
}

// 1/Z of the pending rows j < count (Montgomery's trick: 3 multiplications per
// row and one inversion).  A zero Z gets 0, exactly like fe_inv per row: if the
// product is 0, every row falls back to its own inversion.  One fe_inv call
// site, so the (large) inversion is inlined once.
template <int K>
CUDASP_HD void pend_invert(const Scratch& sc, int base, int count) {
  fe acc, z;
  fe_set_int(acc, 1);
#pragma unroll 1
  for (int j = 0; j < count; j++) {
    scr_store(sc, PEND_ZI(base, j), acc);  // prefix product of Z_0 .. Z_(j-1)
    scr_load(z, sc, PEND_Z(base, j));
    fe_mul(acc, acc, z);
  }
  fe accn = acc;
  fe_normalize(accn);
  const bool zero = fe_is_zero_norm(accn);
  const int rounds = zero ? count : 1;
#pragma unroll 1
  for (int r = 0; r < rounds; r++) {
    fe x, xi;
    if (zero)
      scr_load(x, sc, PEND_Z(base, r));
    else
      x = acc;
    fe_inv(xi, x);
    if (zero) {
      scr_store(sc, PEND_ZI(base, r), xi);
    } else {
      // xi = 1 / (Z_0 ... Z_(count-1)); peel the rows off from the last one.
#pragma unroll 1
      for (int j = count - 1; j >= 0; j--) {
        fe pre, zi;
        scr_load(pre, sc, PEND_ZI(base, j));
        fe_mul(zi, xi, pre);
        scr_store(sc, PEND_ZI(base, j), zi);
        scr_load(z, sc, PEND_Z(base, j));
        fe_mul(xi, xi, z);
      }
    }
  }
}

CUDASP_HD void ge_from_words(ge& r, const uint32_t* w) {
  fe_from_u32x8(r.x, w);
  fe_from_u32x8(r.y, w + 8);
}

// Upper 64 bits of a fully normalized x as the reference's signed BIGINT
// (ExtractUpper64, src/cudasp_gpu.cu:67-71).
CUDASP_HD int64_t fe_upper64(const fe& x) {
  uint32_t w[8];
  fe_to_u32x8(w, x);
  return (int64_t)(((uint64_t)w[7] << 32) | w[6]);
}

// CheckValueMatch (src/cudasp_gpu.cu:29-41).
CUDASP_HD bool outputs_contain(const int64_t* outputs, uint32_t off, uint32_t len, int64_t v) {
  for (uint32_t k = 0; k < len; k++)
    if (outputs[(size_t)off + k] == v) return true;
  return false;
}

// Full-x compare (cudasp_scan_options.full_x): outputs are 32-byte big-endian
// x-only keys, 8 u32 words each; x is a fully normalized field element.
CUDASP_HD uint32_t bswap32(uint32_t v) {
  return (v >> 24) | ((v >> 8) & 0xff00u) | ((v << 8) & 0xff0000u) | (v << 24);
}

CUDASP_HD bool outputs_contain_x(const uint32_t* outputs_x, uint32_t off, uint32_t len, const fe& x) {
  uint32_t w[8];
  fe_to_u32x8(w, x);
  for (uint32_t k = 0; k < len; k++) {
    const uint32_t* o = outputs_x + ((size_t)off + k) * 8;
    uint32_t diff = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) diff |= bswap32(o[q]) ^ w[7 - q];
    if (diff == 0) return true;
  }
  return false;
}

CUDASP_HD bool outputs_match(const ScanConsts& k, const int64_t* outputs, uint32_t off, uint32_t len, const fe& x,
                             int64_t v) {
  return k.full_x ? outputs_contain_x(reinterpret_cast<const uint32_t*>(outputs), off, len, x)
                  : outputs_contain(outputs, off, len, v);
}

// Value reported for a label whose sum F + L is the point at infinity (F = -L):
// no x coordinate exists, the row cannot match through it.
constexpr int64_t LABEL_INFINITY = (int64_t)0x8000000000000000ull;

// Entry for the digit d = 2 b + 1 - 2^BITS of window `window` (b = the
// window's BITS bits): |d| = 2j + 1, negated when b < 2^(BITS-1).
template <int BITS = FB_BITS>
CUDASP_HD void fb_entry(ge& P, const uint32_t* table, int window, uint32_t bits) {
  constexpr uint32_t ENTRIES = FbWidth<BITS>::ENTRIES;
  bool neg = (bits & ENTRIES) == 0;
  uint32_t j = (bits ^ (neg ? ENTRIES - 1 : 0u)) & (ENTRIES - 1);
  const uint32_t* e = table + ((size_t)window * ENTRIES + j) * FB_WORDS;
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t w[16];
  const uint4* e4 = reinterpret_cast<const uint4*>(e);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    uint4 v = e4[q];
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
  ge_from_words(P, w);
#else
  ge_from_words(P, e);
#endif
  if (neg) ge_neg(P, P);
}

// secp256k1 group order n, 8 LE words.
CUDASP_HD uint32_t order_word(int i) {
  const uint32_t n[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                         0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  return n[i];
}

// The odd representative of a scalar for the odd-digit recoding: t = in mod n
// (in < 2^256 < 2n: one conditional subtraction; in >= n has probability
// ~2^-128), then n - t when t is even (n is odd, and (n - t) G = -t G).
// Returns whether the result stands for -t (the caller negates the point).
// Branch-free: lanes of a wave differ in parity.
CUDASP_HD bool scalar_odd_rep(uint32_t t[8], const uint32_t in[8]) {
  uint32_t d[8];
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t x = (uint64_t)in[i] - order_word(i) - borrow;
    d[i] = (uint32_t)x;
    borrow = x >> 63;
  }
  const bool ge = borrow == 0;
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = ge ? d[i] : in[i];
  const bool even = (t[0] & 1u) == 0;
  borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t x = (uint64_t)order_word(i) - t[i] - borrow;
    d[i] = (uint32_t)x;
    borrow = x >> 63;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = even ? d[i] : t[i];
  return even;
}

// P = t*G (Jacobian) from the fixed-base table.  t: 8 LE words, any 256-bit
// value (not reduced mod n, like the reference, src/cudasp_gpu.cu:862-877;
// n*G = O makes that irrelevant).  W gathers and W - 1 mixed additions (W the
// windows of the BITS-bit table), no constant term.
// fb_top (optional): the top window with a point B folded in (ScanConsts::
// fb_top): the result is then t G + B.  A lane whose odd representative
// stands for -t (negated at the end) reads the - B half, so the final
// negation gives -(t' G - B) = t G + B as well.
template <int BITS = FB_BITS>
CUDASP_HD void fixed_base_mul(gej& R, const uint32_t t_in[8], const uint32_t* fb_table,
                              const uint32_t* fb_top = nullptr) {
  constexpr int WINDOWS = FbWidth<BITS>::WINDOWS;
  constexpr uint32_t ENTRIES = FbWidth<BITS>::ENTRIES;
  uint32_t t[9];
  const bool negate = scalar_odd_rep(t, t_in);
  t[8] = 0;
  // odd t' < n = 1 + sum_{i<W} 2 b_i 2^(w i), b_i = bits [w i + 1, w i + w] of
  // t' (w = BITS, W = WINDOWS), written with signed odd digits
  // d_i = 2 b_i + 1 - 2^w below the top window and the positive top digit
  // d_(W-1) = 2 b_(W-1) + 1: the (1 - 2^w) 2^(w i) terms telescope to
  // 1 - 2^(w (W-1)), which the top digit's + 2^(w (W-1)) cancels, so
  // t' = sum d_i 2^(w i) exactly.  t' < 2^256 keeps b_(W-1) < 2^(w-1), a valid
  // table index.
  // The window loop is not unrolled (the mixed additions would blow the
  // instruction cache), so t is consumed by shifting instead of indexing a
  // register array with the loop counter (that would spill to scratch).
#pragma unroll 1
  for (int i = 0; i < WINDOWS; i++) {
    uint32_t bits = (t[0] >> 1) & ((ENTRIES << 1) - 1);
#pragma unroll
    for (int q = 0; q < 8; q++) t[q] = (t[q] >> BITS) | (t[q + 1] << (32 - BITS));
    t[8] >>= BITS;
    ge P;
    if (i < WINDOWS - 1)
      fb_entry<BITS>(P, fb_table, i, bits);
    else if (fb_top)  // positive digit, entry bits of the folded top window (+ B or - B)
      fb_entry<BITS>(P, fb_top + (negate ? (size_t)FbWidth<BITS>::TOP_ENTRIES * FB_WORDS : 0), 0, bits | ENTRIES);
    else
      fb_entry<BITS>(P, fb_table, i, bits | ENTRIES);  // positive digit 2 bits + 1: entry bits
    if (i == 0) {
      gej_set_ge(R, P);
    } else {
      gej_add_ge(R, R, P);
    }
  }
  // -P0 for an even t: y negated (a per-lane select; magnitudes differ per
  // layout, so normalize first)
  fe ny = R.y;
  fe_normalize_weak(ny);
  fe_negate<1>(ny, ny);
  if (negate) R.y = ny;
}

// Stage B, first half: F = t G + B as a Jacobian point.
template <int BITS = FB_BITS>
CUDASP_HD void row_match_point(gej& R, const uint32_t t_in[8], const uint32_t* fb_table, const ScanConsts& k) {
  if (k.fb_top) {
    // an on-curve B folded into the top window: F = t G + B with one mixed
    // addition fewer (the group law makes it the same point as the chord
    // addition below)
    fixed_base_mul<BITS>(R, t_in, fb_table, k.fb_top);
    return;
  }
  fixed_base_mul<BITS>(R, t_in, fb_table);  // P0 = t*G
  // B added on its own: F = P0 + B is the same single chord addition as the
  // reference's, also for a spend key that is not on the curve.
  ge B;
  ge_from_words(B, k.spend);
  gej_add_ge(R, R, B);  // F = P0 + B (Jacobian)
}

// Stage B, second half: from F (Jacobian) and 1/Z, the compare values and the
// match.  Returns whether the row matches; if values != nullptr, writes the
// base value and one value per label (values[j * vstride]).  sc: the label
// scratch (10 L words per slot).
CUDASP_HD bool row_match_finish(const gej& R, const fe& zi, const ScanConsts& k, const uint32_t* labels,
                                const int64_t* outputs, uint32_t off, uint32_t len, const Scratch& sc,
                                int64_t* values, uint32_t vstride) {
  ge F;
  gej_to_ge_zinv(F, R, zi);
  int64_t v = fe_upper64(F.x);  // F is normalized by gej_to_ge_zinv
  if (values) values[0] = v;
  bool hit = outputs_match(k, outputs, off, len, F.x, v);

  uint32_t L = k.label_count;
  if (L == 0) return hit;

  // --- labels: x of F + L_j for all j with one batched inversion -------------
  // The reference adds each label with its own inversion and stops at the
  // first hit (src/cudasp_gpu.cu:153-172); the flag is the same OR.
  // Exceptional sums are handled like the reference's Python oracle
  // (scripts/compute_bip352_expected.py:42-46): F == L doubles, F == -L is O.
  fe accp;
  fe_set_int(accp, 1);
  for (uint32_t j = 0; j < L; j++) {
    ge Lj;
    ge_from_words(Lj, labels + (size_t)j * 16);
    fe d;
    if (!fe_equal_norm(Lj.x, F.x)) {
      fe_sub<1>(d, Lj.x, F.x);
    } else if (fe_equal_norm(Lj.y, F.y)) {
      fe_add(d, F.y, F.y);
    } else {
      fe_set_int(d, 1);
    }
    scr_store(sc, (int)j * FW, accp);
    fe_mul(accp, accp, d);
  }
  fe inv;
  fe_inv(inv, accp);
  for (int j = (int)L - 1; j >= 0; j--) {
    ge Lj;
    ge_from_words(Lj, labels + (size_t)j * 16);
    fe d, num, pre, dinv;
    bool xeq = fe_equal_norm(Lj.x, F.x);
    bool infinity = false;
    if (!xeq) {
      fe_sub<1>(d, Lj.x, F.x);
      fe_sub<1>(num, Lj.y, F.y);
    } else if (fe_equal_norm(Lj.y, F.y)) {
      fe_add(d, F.y, F.y);
      fe_sqr(num, F.x);
      fe_mul_int(num, num, 3);
    } else {
      fe_set_int(d, 1);
      fe_set_int(num, 0);
      infinity = true;
    }
    scr_load(pre, sc, j * FW);
    fe_mul(dinv, inv, pre);
    fe_mul(inv, inv, d);
    fe lam, x3;
    fe_mul(lam, num, dinv);
    fe_sqr(x3, lam);
    fe_sub<1>(x3, x3, F.x);
    fe_sub<1>(x3, x3, Lj.x);
    fe_normalize(x3);
    int64_t vj = infinity ? LABEL_INFINITY : fe_upper64(x3);
    if (values) values[(size_t)(1 + j) * vstride] = vj;
    if (!infinity) hit = hit || outputs_match(k, outputs, off, len, x3, vj);
  }
  return hit;
}

// Denominator (and numerator) of the label sum F + L (F, L affine,
// normalized): L.x - F.x and L.y - F.y for a chord; 2 F.y and 3 F.x^2 when
// F == L (doubling); d = 1, num = 0 and `true` (infinity) when F == -L --
// the reference's Python oracle's cases (scripts/compute_bip352_expected.py:42-46).
CUDASP_HD bool label_terms(fe& d, fe* num, const ge& F, const ge& L) {
  if (!fe_equal_norm(L.x, F.x)) {
    fe_sub<1>(d, L.x, F.x);
    if (num) fe_sub<1>(*num, L.y, F.y);
    return false;
  }
  if (fe_equal_norm(L.y, F.y)) {
    fe_add(d, F.y, F.y);
    if (num) {
      fe_sqr(*num, F.x);
      fe_mul_int(*num, *num, 3);
    }
    return false;
  }
  fe_set_int(d, 1);
  if (num) fe_set_int(*num, 0);
  return true;
}

// Stage B, base half of a pending row: F affine from (R, 1/Z), the base
// compare value and match; F is written back over the row's pending X / Y
// words for match_labels_rows.
CUDASP_HD bool row_match_base(const gej& R, const fe& zi, const ScanConsts& k, const int64_t* outputs,
                              uint32_t off, uint32_t len, const Scratch& sc, int pb, int j, int64_t* value) {
  ge F;
  gej_to_ge_zinv(F, R, zi);
  scr_store(sc, PEND_X(pb, j), F.x);
  scr_store(sc, PEND_Y(pb, j), F.y);
  int64_t v = fe_upper64(F.x);
  if (value) *value = v;
  return outputs_match(k, outputs, off, len, F.x, v);
}

// Label sums F_j + L_l of a thread's rows j < count, first half: the count x L
// denominators' prefix products at scratch words lb + (j L + l) FW, and their
// product in acc (Montgomery's trick).  f_at(j, F) loads row j's affine F.
template <class FAt>
CUDASP_HD void labels_forward(fe& acc, const ScanConsts& k, const uint32_t* labels, int count, const Scratch& sc,
                              int lb, const FAt& f_at) {
  const int L = (int)k.label_count;
  fe_set_int(acc, 1);
  for (int j = 0; j < count; j++) {
    ge F;
    f_at(j, F);
    for (int l = 0; l < L; l++) {
      ge Ll;
      ge_from_words(Ll, labels + (size_t)l * 16);
      fe d;
      label_terms(d, nullptr, F, Ll);
      scr_store(sc, lb + (j * L + l) * FW, acc);
      fe_mul(acc, acc, d);
    }
  }
}

// Second half, from inv = 1 / acc: x of every sum, the values and the
// compares.  Returns the rows with a label hit as a bit mask.  row_out(j,
// outputs, off, len, vrow, vstride) gives row j's outputs list and, if
// vrow != nullptr, where its label values go (vrow[(1 + l) vstride]).
template <class FAt, class RowOut>
CUDASP_HD uint32_t labels_backward(fe inv, const ScanConsts& k, const uint32_t* labels, int count, const Scratch& sc,
                                   int lb, const FAt& f_at, const RowOut& row_out) {
  const int L = (int)k.label_count;
  uint32_t hits = 0;
  for (int j = count - 1; j >= 0; j--) {
    const int64_t* outputs;
    uint32_t off, len, vstride;
    int64_t* vrow;
    row_out(j, outputs, off, len, vrow, vstride);
    ge F;
    f_at(j, F);
    bool hit = false;
    for (int l = L - 1; l >= 0; l--) {
      ge Ll;
      ge_from_words(Ll, labels + (size_t)l * 16);
      fe d, num, pre, dinv;
      const bool infinity = label_terms(d, &num, F, Ll);
      scr_load(pre, sc, lb + (j * L + l) * FW);
      fe_mul(dinv, inv, pre);
      fe_mul(inv, inv, d);
      fe lam, x3;
      fe_mul(lam, num, dinv);
      fe_sqr(x3, lam);
      fe_sub<1>(x3, x3, F.x);
      fe_sub<1>(x3, x3, Ll.x);
      fe_normalize(x3);
      const int64_t vl = infinity ? LABEL_INFINITY : fe_upper64(x3);
      if (vrow) vrow[(size_t)(1 + l) * vstride] = vl;
      if (!infinity) hit = hit || outputs_match(k, outputs, off, len, x3, vl);
    }
    if (hit) hits |= 1u << j;
  }
  return hits;
}

// Label sums F_j + L_l of a thread's pending rows j < count (F affine in the
// pending slots' X / Y words), all with ONE batched inversion over the
// count x L denominators instead of one per row.  Same values and hits as
// row_match_finish.
template <class RowOut>
CUDASP_HD uint32_t match_labels_core(const ScanConsts& k, const uint32_t* labels, int count, const Scratch& sc, int pb,
                                     int lb, const RowOut& row_out) {
  const auto f_at = [&](int j, ge& F) {
    scr_load(F.x, sc, PEND_X(pb, j));
    scr_load(F.y, sc, PEND_Y(pb, j));
  };
  fe acc, inv;
  labels_forward(acc, k, labels, count, sc, lb, f_at);
  fe_inv(inv, acc);
  return labels_backward(inv, k, labels, count, sc, lb, f_at, row_out);
}

// match_labels_core for the rows g + j G of one batch (k_match, the
// emulation): outputs lists by input row (virtual row mod n_rows), label
// values (with `values`, then outputs/offs/lens unused) to
// values[(1 + l) n + row]; label prefix products from scratch word 0.
CUDASP_HD uint32_t match_labels_rows(const ScanConsts& k, const uint32_t* labels, const int64_t* outputs,
                                     const uint32_t* offs, const uint32_t* lens, uint32_t g, uint32_t G, uint32_t n,
                                     uint32_t n_rows, int count, const Scratch& sc, int pb, int64_t* values) {
  return match_labels_core(k, labels, count, sc, pb, 0,
                           [&](int j, const int64_t*& o, uint32_t& off, uint32_t& len, int64_t*& vrow,
                               uint32_t& vstride) {
                             const uint32_t row = g + (uint32_t)j * G;
                             const uint32_t orow = n == n_rows ? row : row % n_rows;
                             o = outputs;
                             off = values ? 0u : offs[orow];
                             len = values ? 0u : lens[orow];
                             vrow = values ? values + row : nullptr;
                             vstride = n;
                           });
}

// Stage B for one row (one inversion per row).
template <int BITS = FB_BITS>
CUDASP_HD bool row_match(const uint32_t t_in[8], const uint32_t* fb_table, const ScanConsts& k,
                         const uint32_t* labels, const int64_t* outputs, uint32_t off, uint32_t len,
                         const Scratch& sc, int64_t* values, uint32_t vstride) {
  gej R;
  row_match_point<BITS>(R, t_in, fb_table, k);
  fe zi;
  fe_inv(zi, R.z);
  return row_match_finish(R, zi, k, labels, outputs, off, len, sc, values, vstride);
}

// Fixed-base table entry (2j+1) Q of a window with base Q = 2^(w window) G.
// Affine P + Q (normalized words) given inv = 1 / (Q.x - P.x).
CUDASP_HD void affine_add_inv(uint32_t out[16], const ge& P, const ge& Q, const fe& inv) {
  fe num, lam, x3, y3, t;
  fe_sub<1>(num, Q.y, P.y);
  fe_mul(lam, num, inv);
  fe_sqr(x3, lam);
  fe_sub<1>(x3, x3, P.x);
  fe_sub<1>(x3, x3, Q.x);
  fe_normalize(x3);
  fe_sub<1>(t, P.x, x3);
  fe_mul(y3, lam, t);
  fe_sub<1>(y3, y3, P.y);
  fe_normalize(y3);
  fe_to_u32x8(out, x3);
  fe_to_u32x8(out + 8, y3);
}

// One entry P of the fixed-base table's top window with the spend key folded
// in (ScanConsts::fb_top): out_pos = P + B, out_neg = P - B, both affine and
// normalized, from one inversion (the two denominators are the same).
// P, B normalized.  False when x(P) = x(B): a sum would be a doubling or the
// point at infinity (probability ~2^-230 for a real key); the scanner then
// adds B on its own.
CUDASP_HD bool fb_fold_entry(uint32_t out_pos[16], uint32_t out_neg[16], const ge& P, const ge& B) {
  fe den, dn, inv;
  fe_sub<1>(den, B.x, P.x);
  dn = den;
  fe_normalize(dn);
  if (fe_is_zero_norm(dn)) return false;
  fe_inv(inv, dn);
  affine_add_inv(out_pos, P, B, inv);
  ge nB;
  nB.x = B.x;
  fe_negate<1>(nB.y, B.y);
  fe_normalize(nB.y);
  affine_add_inv(out_neg, P, nB, inv);
  return true;
}

// y^2 = x^3 + 7 for normalized words (the fold needs the group law, so only
// an on-curve spend key is folded).
CUDASP_HD bool on_curve_words(const uint32_t w[16]) {
  fe x, y, y2, x3;
  fe_from_u32x8(x, w);
  fe_from_u32x8(y, w + 8);
  fe_sqr(y2, y);
  fe_sqr(x3, x);
  fe_mul(x3, x3, x);
  fe seven;
  fe_set_int(seven, 7);
  fe_add(x3, x3, seven);
  fe_normalize(y2);
  fe_normalize(x3);
  return fe_equal_norm(y2, x3);
}

CUDASP_HD void fb_build_entry(uint32_t out[16], const ge& Q, uint32_t j) {
  uint32_t m = 2 * j + 1;  // 1 .. 2^w - 1
  int top = 31 - __builtin_clz(m);
  gej R;
  gej_set_ge(R, Q);
  for (int b = top - 1; b >= 0; b--) {
    gej_double(R, R);
    if ((m >> b) & 1u) gej_add_ge(R, R, Q);
  }
  fe zi;
  fe_inv(zi, R.z);
  ge A;
  gej_to_ge_zinv(A, R, zi);
  fe_to_u32x8(out, A.x);
  fe_to_u32x8(out + 8, A.y);
}

}  // namespace cudasp
