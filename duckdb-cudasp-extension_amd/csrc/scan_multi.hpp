// Work distribution of the multi-batch persistent scan (k_scan_multi,
// scan_kernels.hip), written once as __host__ __device__ code so that
// tests/native/cudasp_emu.cpp can replay the schedule on the CPU and check
// that every row of every batch is scanned exactly once.
//
// The batches' rows form a virtual row space of 64-row wave-rows: batch b
// occupies wave-rows [first_wr, first_wr + ceil(n / 64)), so a wave-row never
// spans two batches and the last one of a batch is padded.
#pragma once
#include <stdint.h>

#include "secp256k1_fe.hpp"  // CUDASP_HD

namespace cudasp {

// Device descriptor of one batch (cudasp_device_batch plus its first wave-row).
struct MultiBatch {
  const uint32_t* tx;
  const uint32_t* ty;
  const int64_t* outputs;
  const uint32_t* offs;
  const uint32_t* lens;
  uint8_t* flags;
  uint32_t* match_rows;
  uint32_t* match_count;
  uint32_t n;
  uint32_t first_wr;
};

// The batch holding wave-row w (w wave-uniform): the last batch with
// first_wr <= w.
CUDASP_HD uint32_t multi_batch_of(const MultiBatch* __restrict__ bd, uint32_t nb, uint32_t w) {
  uint32_t lo = 0, hi = nb;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (bd[mid].first_wr <= w) lo = mid; else hi = mid;
  }
  return lo;
}

// Row of this lane in wave-row w of batch `b`; *active = false for the padding
// of the batch's last wave-row (which then reads batch row 0).
CUDASP_HD uint32_t multi_row(const MultiBatch& b, uint32_t w, uint32_t lane, bool* active) {
  const uint32_t r = (w - b.first_wr) * 64u + lane;
  *active = r < b.n;
  return *active ? r : 0u;
}

// Wave-rows of the next piece (= rows per thread) with `rem` wave-rows left:
// guided self-scheduling, rem / g1 rows (at least 1, at most rmax; g1 = the
// grid's waves for the classic rule), so a piece is never longer than the
// time the other waves need for what remains and the waves run out of work
// together; rmax while more than g2 wave-rows remain (g2 = 0: the rule
// throughout), and rmax throughout when g1 = 0.
CUDASP_HD uint32_t multi_piece_rows(uint32_t rem, uint32_t g1, uint32_t g2, uint32_t rmax) {
  if (g1 == 0 || (g2 != 0 && rem > g2)) return rmax;
  const uint32_t r = rem / g1;
  return r < 1u ? 1u : (r > rmax ? rmax : r);
}

// The adaptive form: a wave that has already claimed `mine` wave-rows of the
// `prev` claimed by all sizes its next piece by its own share of the work done,
// rem x mine / prev rows (at least 1, at most rmax), so that the piece ends
// when the other waves finish what remains, however unevenly the SIMDs share
// their issue slots among resident waves (the oldest wave of a SIMD issues
// first: on gfx950 the three waves of a SIMD progress at ~1 : 0.3 : 0.05).
// A wave's first piece is one wave-row (its speed is not known yet); g1 = 0
// (a fused single-batch launch) keeps rmax throughout.
//
// `young`: the wave is its SIMD's youngest (the persistent grid's last third
// of blocks: the dispatcher places blocks 0 .. cus - 1 first on every CU,
// then the next cus, then the last; tools/multi_trace.py finds the last third
// the slowest on all 1024 SIMDs).  It issues last, at ~4% of its SIMD while the
// older two work, so a wave-row it claims late is the last work of its SIMD
// and runs alone there in the drain.  In a launch of fewer than 10 x g1
// wave-rows (~2M rows on the full grid: while a young wave does one wave-row
// at ~4% of its SIMD, the GPU does ~25 per SIMD) it takes no piece at all: 0
// (= leave).  Leaving later as well, once its share of the rows left drops
// under one wave-row, costs more than the straggler it saves (its issue share
// lost for the second half of a 4M-row launch: -0.5%).
// The older waves keep the rules above, so every row is still claimed.
CUDASP_HD uint32_t multi_piece_rows_adaptive(uint32_t rem, uint32_t prev, uint32_t mine, uint32_t g1, uint32_t g2,
                                             uint32_t rmax, bool young = false) {
  if (g1 == 0) return rmax;
  if (mine == 0 || prev == 0) return young && rem < 10ull * g1 ? 0u : 1u;
  const uint64_t r = (uint64_t)rem * mine / prev;
  return r < 1u ? 1u : (r > rmax ? rmax : (uint32_t)r);
}

}  // namespace cudasp
