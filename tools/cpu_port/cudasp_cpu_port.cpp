// Optimized CPU baseline ("port-optimized"): the product's own per-row
// pipeline (duckdb-cudasp-extension_amd/csrc/scan_rows.hpp -- GLV + width-5
// wNAF with co-Z odd multiples, one shared inversion per group of rows,
// one-compression tagged SHA-256, batched label inversions) compiled for the
// host CPU at -O3 without the emulation build's magnitude checks, run on
// std::threads.  The fixed-base table is sized for a CPU cache instead of HBM:
// 8-bit windows (32 windows x 128 odd multiples, 256 KB) instead of the GPU's
// 22/26-bit HBM tables.  Used only by bench.py's cpu_baseline leg as a
// reported baseline next to the plain C oracle; never part of the product path
// (the product is libcudasp_amd.so on a gfx950 device).
#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "../../duckdb-cudasp-extension_amd/csrc/scan_prepare.hpp"

using namespace cudasp;

namespace {

constexpr int CPU_FB_BITS = 8;
constexpr int ROWS = 8;  // rows per group sharing one inversion (stage A and stage B)

struct CpuTable {
  std::vector<uint32_t> t;
  CpuTable() {
    const int W = FbWidth<CPU_FB_BITS>::WINDOWS;
    const uint32_t E = FbWidth<CPU_FB_BITS>::ENTRIES;
    t.resize((size_t)W * E * FB_WORDS);
    std::vector<uint32_t> bases = fb_window_bases(CPU_FB_BITS);
    for (int w = 0; w < W; w++) {
      ge Q;
      ge_from_words(Q, &bases[(size_t)w * 16]);
      for (uint32_t j = 0; j < E; j++) fb_build_entry(&t[((size_t)w * E + j) * FB_WORDS], Q, j);
    }
  }
};

const CpuTable& cpu_table() {
  static CpuTable tab;
  return tab;
}

void words_from_row(uint32_t x[8], uint32_t y[8], const uint8_t* row) {
  for (int i = 0; i < 8; i++) {
    x[i] = (uint32_t)row[4 * i] | ((uint32_t)row[4 * i + 1] << 8) | ((uint32_t)row[4 * i + 2] << 16) |
           ((uint32_t)row[4 * i + 3] << 24);
    const uint8_t* r = row + 32;
    y[i] = (uint32_t)r[4 * i] | ((uint32_t)r[4 * i + 1] << 8) | ((uint32_t)r[4 * i + 2] << 16) |
           ((uint32_t)r[4 * i + 3] << 24);
  }
}

// Rows [g, g + count) of one thread: stage A (shared inversion) then stage B
// (shared Z inversion, batched label inversion), as k_shared_secret / k_match.
void scan_group(const ScanConsts& k, const int8_t* naf, const uint32_t* labels, const uint32_t* fb,
                const uint8_t* tweaks, const int64_t* outputs, const uint32_t* offs, const uint32_t* lens, uint32_t g,
                int count, uint32_t n, const Scratch& sa, const Scratch& sb, uint8_t* flags) {
  constexpr int PA = VB_SCRATCH_WORDS;
  uint32_t t[ROWS][8];
  for (int j = 0; j < count; j++) {
    uint32_t x[8], y[8];
    words_from_row(x, y, tweaks + 64 * (size_t)(g + j));
    gej P;
    row_shared_secret_point(P, x, y, naf, k.naf_len, sa);
    pend_store(sa, PA, j, P);
  }
  pend_invert<ROWS>(sa, PA, count);
  for (int j = 0; j < count; j++) {
    gej P;
    fe zi;
    pend_load(P, sa, PA, j);
    scr_load(zi, sa, PEND_ZI(PA, j));
    uint32_t sx[8];
    const uint32_t y_odd = row_shared_secret_affine(sx, P, zi);
    bip352_shared_secret_hash(t[j], k.mid, sx, y_odd, 0);
  }
  const int PB = FW * (int)k.label_count * ROWS;
  for (int j = 0; j < count; j++) {
    gej P;
    row_match_point<CPU_FB_BITS>(P, t[j], fb, k);
    pend_store(sb, PB, j, P);
  }
  pend_invert<ROWS>(sb, PB, count);
  uint32_t hits = 0;
  for (int j = 0; j < count; j++) {
    const uint32_t row = g + (uint32_t)j;
    gej P;
    fe zi;
    pend_load(P, sb, PB, j);
    scr_load(zi, sb, PEND_ZI(PB, j));
    if (row_match_base(P, zi, k, outputs, offs[row], lens[row], sb, PB, j, nullptr)) hits |= 1u << j;
  }
  if (k.label_count) hits |= match_labels_rows(k, labels, outputs, offs, lens, g, 1, n, n, count, sb, PB, nullptr);
  for (int j = 0; j < count; j++) flags[g + j] = (hits >> j) & 1u;
}

}  // namespace

extern "C" {

// Flags of n rows (tweaks: n x 64-byte LE x||y blobs; outputs CSR), the
// reference's semantics; threads <= 0 means 1.  Returns 0 or a negative code.
int cudasp_cpu_port_scan(const uint8_t scan[32], const uint8_t spend[64], const uint8_t* label_keys,
                         uint32_t label_count, const uint8_t* tweaks, uint32_t n, const int64_t* outputs,
                         const uint32_t* offs, const uint32_t* lens, uint8_t* flags, int threads) {
  ScanConsts k;
  std::vector<int8_t> naf;
  std::vector<uint32_t> labels;
  std::string err;
  int rc = prepare_scan(scan, spend, label_keys, label_count, k, naf, labels, err);
  if (rc != CUDASP_OK) return rc;
  const uint32_t* fb = cpu_table().t.data();
  if (threads <= 0) threads = 1;
  std::atomic<uint32_t> next{0};
  const uint32_t chunk = 64 * ROWS;
  auto work = [&]() {
    std::vector<uint32_t> va(VB_SCRATCH_WORDS + PEND_WORDS * ROWS);
    std::vector<uint32_t> vb((size_t)(FW * k.label_count + PEND_WORDS) * ROWS);
    Scratch sa{va.data(), 1, 0}, sb{vb.data(), 1, 0};
    for (;;) {
      const uint32_t c0 = next.fetch_add(chunk);
      if (c0 >= n) break;
      const uint32_t c1 = c0 + chunk < n ? c0 + chunk : n;
      for (uint32_t g = c0; g < c1; g += ROWS) {
        const int count = (int)(c1 - g < (uint32_t)ROWS ? c1 - g : (uint32_t)ROWS);
        scan_group(k, naf.data(), labels.data(), fb, tweaks, outputs, offs, lens, g, count, n, sa, sb, flags);
      }
    }
  };
  std::vector<std::thread> th;
  for (int i = 1; i < threads; i++) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  return 0;
}

}  // extern "C"
