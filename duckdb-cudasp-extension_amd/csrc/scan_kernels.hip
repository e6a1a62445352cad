// cudasp_scan hot path for MI355X (gfx950): kernels, per-device fixed-base
// table, scanner objects and the C ABI declared in include/cudasp_abi.h.
//
// Kernel pipeline for one batch of n rows (all device-resident):
//   k_shared_secret   stage A of scan_rows.hpp: reads tweak columns (8 x n u32
//                     each, column-major), writes t (8 x n u32).
//   k_match           stage B: reads t, gathers from the per-device fixed-base
//                     table (22-bit windows: 1.5 GiB, 26-bit: 21.5 GB; a
//                     per-scanner choice, scan_rows.hpp), compares with the outputs CSR, writes one flag per
//                     row and (optionally) the compacted row indices via a
//                     per-wavefront ballot + one atomic per wave.
// Replaces the reference's ec_pmul + serialize + hash + host round trip +
// fixed-point + check sequence (src/cudasp_gpu.cu:764-956), which crosses PCIe
// twice per batch; here nothing leaves the device between the two kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <memory>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/cudasp_abi.h"
#include "scan_prepare.hpp"
#include "scan_multi.hpp"
#include "scan_stream.hpp"

using namespace cudasp;

#define CUDASP_VERSION_STRING "cudasp-mi355x 0.1.0 (gfx950)"

// ----------------------------------------------------------------- errors
namespace {
thread_local std::string g_last_error;

int set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define HIP_TRY(expr)                                                                          \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      return set_error(CUDASP_ERR_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), \
                       __FILE__, __LINE__);                                                    \
  } while (0)

constexpr int BLOCK = 256;
// Minimum waves per SIMD requested for the two hot kernels (register budget:
// 2 -> 256 VGPRs, 3 -> 168, 4 -> 128).  Tuned on MI355X; see DESIGN.md.
#ifndef CUDASP_WAVES_A
#define CUDASP_WAVES_A 3
#endif
#ifndef CUDASP_WAVES_B
#define CUDASP_WAVES_B 3
#endif
// Measurement-only A/B (never in a product build): CUDASP_AB_SCRATCH_ALIAS=S
// maps every thread's scratch slot onto slot mod S, so the per-row scratch of
// both stages (odd-multiple table, Z ratios, pending rows, label prefix
// products) stays inside an L2-sized region: the HBM traffic of the scratch
// disappears while the instruction stream is unchanged.  Threads then race on
// shared slots, so results are wrong -- the build only times the kernels.
#ifdef CUDASP_AB_SCRATCH_ALIAS
__device__ __forceinline__ Scratch ab_scratch(uint32_t* s, uint32_t stride, uint32_t slot) {
  // never more slots than the buffer holds (stride = the launch's thread count)
  const uint32_t a = stride < CUDASP_AB_SCRATCH_ALIAS ? stride : CUDASP_AB_SCRATCH_ALIAS;
  return make_scratch(s, a, slot % a);
}
#define SCAN_SCRATCH ab_scratch
#else
#define SCAN_SCRATCH make_scratch
#endif
// Grid cap for the grid-stride kernels; also bounds the per-slot scratch.
constexpr uint32_t MAX_BLOCKS = 4096;
// Rows per thread in stage A / stage B: the rows of a thread share one field
// inversion (Montgomery's trick, pend_invert in scan_rows.hpp).  Tuned on
// MI355X; see DESIGN.md.
#ifndef CUDASP_ROWS_A
#define CUDASP_ROWS_A 4
#endif
#ifndef CUDASP_ROWS_B
#define CUDASP_ROWS_B 6
#endif
constexpr int ROWS_A = CUDASP_ROWS_A;
constexpr int ROWS_B = CUDASP_ROWS_B;
static_assert(ROWS_A >= 1 && ROWS_A <= 8 && ROWS_B >= 1 && ROWS_B <= 8, "rows per thread");
// Scratch words per slot: stage A's odd-multiple table + its pending rows;
// stage B's label prefix products (FW L per row of the thread: one batched
// inversion for all its rows' labels) + its pending rows.
constexpr uint32_t vscratch_words(int rows) { return VB_SCRATCH_WORDS + PEND_WORDS * (uint32_t)rows; }
constexpr uint32_t VSCRATCH_WORDS = vscratch_words(ROWS_A);
inline uint32_t lscratch_words(uint32_t label_count, int rows = ROWS_B) {
  return (FW * label_count + PEND_WORDS) * (uint32_t)rows;
}
}  // namespace

// ----------------------------------------------------------------- kernels

// t of output index kk of row `row`: virtual row kk * n + row of the 8 x (K n)
// column-major t array (K = k.output_count, 1 in the reference's semantics).
__device__ __forceinline__ void store_t(uint32_t* __restrict__ t_out, uint32_t n, uint32_t K, uint32_t row,
                                        const uint32_t sx[8], uint32_t y_odd, const uint32_t mid[8]) {
  const size_t N = (size_t)K * n;
#pragma unroll 1
  for (uint32_t kk = 0; kk < K; kk++) {
    uint32_t t[8];
    bip352_shared_secret_hash(t, mid, sx, y_odd, kk);
#pragma unroll
    for (int w = 0; w < 8; w++) t_out[(size_t)w * N + (size_t)kk * n + row] = t[w];
  }
}

// The odd-multiple table's y of entries 0 .. N-1 in LDS (LdsY, scan_rows.hpp;
// 0: all in scratch).  Three blocks per CU leave room for 5 (45 KB of the 53 KB
// a block may have; k_scan_stream's prefetch transpose shares the area).  The
// scratch traffic they take off (~25%) is energy under the power cap: +0.9%
// config 4 device-resident (k_scan_multi, at a higher clock), +1.0% end to end
// (k_scan_stream; profiles/r06_lds_y_ab.txt).  k_shared_secret (the per-slot
// launches' stage A) uses CUDASP_MULTI_LDS_Y too.
#ifndef CUDASP_MULTI_LDS_Y
#define CUDASP_MULTI_LDS_Y 5
#endif
#ifndef CUDASP_STREAM_LDS_Y
#define CUDASP_STREAM_LDS_Y 5
#endif
static_assert(CUDASP_WAVES_A * CUDASP_MULTI_LDS_Y * FW * BLOCK * 4 <= 160 * 1024,
              "k_scan_multi's LDS y table must leave CUDASP_WAVES_A blocks per CU");

// Stage A: thread `slot` takes the rows g, g + G, ... (G = ceil(n / R)) of
// each of its groups g, so every row access stays coalesced.  R = ROWS_A rows
// per thread share one inversion; launches too small to fill the GPU use 2 or
// 1 (rows_a_for), which shortens the launch (its rows run in sequence).
template <int R>
__global__ __launch_bounds__(BLOCK, CUDASP_WAVES_A) void k_shared_secret(const uint32_t* __restrict__ tx,
                                                         const uint32_t* __restrict__ ty, uint32_t n,
                                                         const int8_t* __restrict__ naf, ScanConsts k,
                                                         uint32_t* __restrict__ vscr,
                                                         uint32_t* __restrict__ t_out) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t stride = gridDim.x * blockDim.x;
  const Scratch sc = SCAN_SCRATCH(vscr, stride, slot);
  // A/B builds may fold only the odd-multiple table or only the pending rows
  // (the two regions never overlap: table words < VB_SCRATCH_WORDS).
#if defined(CUDASP_AB_ALIAS_TABLE_ONLY)
  const Scratch sc_tab = SCAN_SCRATCH(vscr, stride, slot), sc_pend = make_scratch(vscr, stride, slot);
#elif defined(CUDASP_AB_ALIAS_PEND_ONLY)
  const Scratch sc_tab = make_scratch(vscr, stride, slot), sc_pend = SCAN_SCRATCH(vscr, stride, slot);
#else
  const Scratch& sc_tab = sc;
  const Scratch& sc_pend = sc;
#endif
#if CUDASP_MULTI_LDS_Y
  __shared__ uint32_t ytab[CUDASP_MULTI_LDS_Y * FW][BLOCK];
  const LdsY<CUDASP_MULTI_LDS_Y> yt{&ytab[0][threadIdx.x], BLOCK};
#else
  const ScrY yt;
#endif
  if constexpr (R == 1) {
    for (uint32_t row = slot; row < n; row += stride) {
      uint32_t x[8], y[8];
#pragma unroll
      for (int w = 0; w < 8; w++) {
        x[w] = tx[(size_t)w * n + row];
        y[w] = ty[(size_t)w * n + row];
      }
      gej P;
      row_shared_secret_point_t(P, x, y, naf, k.naf_len, sc, NoTick(), yt);
      fe zi;
      fe_inv(zi, P.z);
      uint32_t sx[8];
      const uint32_t y_odd = row_shared_secret_affine(sx, P, zi);
      store_t(t_out, n, k.output_count, row, sx, y_odd, k.mid);
    }
    return;
  }
  const uint32_t G = (n + R - 1) / R;
  constexpr int PB = VB_SCRATCH_WORDS;
  for (uint32_t g = slot; g < G; g += stride) {
    int count = 0;
#pragma unroll 1
    for (int j = 0; j < R; j++) {
      const uint32_t row = g + (uint32_t)j * G;
      if (row >= n) break;
      uint32_t x[8], y[8];
#pragma unroll
      for (int w = 0; w < 8; w++) {
        x[w] = tx[(size_t)w * n + row];
        y[w] = ty[(size_t)w * n + row];
      }
      gej P;
      row_shared_secret_point_t(P, x, y, naf, k.naf_len, sc_tab, NoTick(), yt);
      pend_store(sc_pend, PB, j, P);
      count = j + 1;
    }
    pend_invert<R>(sc_pend, PB, count);
#pragma unroll 1
    for (int j = 0; j < count; j++) {
      const uint32_t row = g + (uint32_t)j * G;
      gej P;
      fe zi;
      pend_load(P, sc_pend, PB, j);
      scr_load(zi, sc_pend, PEND_ZI(PB, j));
      uint32_t sx[8];
      const uint32_t y_odd = row_shared_secret_affine(sx, P, zi);
      store_t(t_out, n, k.output_count, row, sx, y_odd, k.mid);
    }
  }
}

// Stage B: rows g, g + G, ... (G = ceil(n / R)) per thread as in stage A
// (R = ROWS_B, or 2 for launches too small to fill the GPU: rows_b_for); the
// block walks its groups together so that the compaction ballots see
// consecutive rows of full waves.  n counts virtual rows kk * n_rows + row
// (K output indices per input row; n == n_rows when K = 1): t, flags and
// values are indexed by the virtual row, the outputs lists by the input row.
template <bool VALUES, int R, int FBB>
__device__ __forceinline__ void match_body(const uint32_t* __restrict__ t_in, uint32_t n, uint32_t n_rows,
                                           const uint32_t* __restrict__ fb, const ScanConsts& k,
                                           const uint32_t* __restrict__ labels,
                                           const int64_t* __restrict__ outputs,
                                           const uint32_t* __restrict__ offs,
                                           const uint32_t* __restrict__ lens,
                                           uint32_t* __restrict__ lscr, uint8_t* __restrict__ flags,
                                           uint32_t* __restrict__ match_rows,
                                           uint32_t* __restrict__ match_count,
                                           int64_t* __restrict__ values) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t stride = gridDim.x * blockDim.x;
  const Scratch sc = SCAN_SCRATCH(lscr, stride, slot);
  const uint32_t G = (n + R - 1) / R;
  const int PB = FW * (int)k.label_count * R;
  for (uint32_t g0 = blockIdx.x * blockDim.x; g0 < G; g0 += stride) {
    const uint32_t g = g0 + threadIdx.x;
    int count = 0;
    uint32_t hits = 0;  // R > 1: bit j = row j matches
    if (R > 1 && g < G) {
#pragma unroll 1
      for (int j = 0; j < R; j++) {
        const uint32_t row = g + (uint32_t)j * G;
        if (row >= n) break;
        uint32_t t[8];
#pragma unroll
        for (int w = 0; w < 8; w++) t[w] = t_in[(size_t)w * n + row];
        gej P;
        row_match_point<FBB>(P, t, fb, k);
        pend_store(sc, PB, j, P);
        count = j + 1;
      }
      pend_invert<R>(sc, PB, count);
      // base values of all rows, then the labels of all rows with one
      // batched inversion (match_labels_rows)
#pragma unroll 1
      for (int j = 0; j < count; j++) {
        const uint32_t row = g + (uint32_t)j * G;
        const uint32_t orow = n == n_rows ? row : row % n_rows;
        gej P;
        fe zi;
        pend_load(P, sc, PB, j);
        scr_load(zi, sc, PEND_ZI(PB, j));
        const uint32_t off = VALUES ? 0u : offs[orow];
        const uint32_t len = VALUES ? 0u : lens[orow];
        if (row_match_base(P, zi, k, outputs, off, len, sc, PB, j, VALUES ? values + row : nullptr)) hits |= 1u << j;
      }
      if (k.label_count)
        hits |= match_labels_rows(k, labels, outputs, offs, lens, g, G, n, n_rows, count, sc, PB,
                                  VALUES ? values : nullptr);
    }
#pragma unroll 1
    for (int j = 0; j < R; j++) {
      const uint32_t row = g + (uint32_t)j * G;
      bool hit = false;
      if (R == 1 && g < n) {
        uint32_t t[8];
#pragma unroll
        for (int w = 0; w < 8; w++) t[w] = t_in[(size_t)w * n + row];
        const uint32_t orow = n == n_rows ? row : row % n_rows;
        uint32_t off = VALUES ? 0u : offs[orow];
        uint32_t len = VALUES ? 0u : lens[orow];
        hit = row_match<FBB>(t, fb, k, labels, outputs, off, len, sc, VALUES ? values + row : nullptr, n);
        if (!VALUES) flags[row] = hit ? 1 : 0;
      } else if (j < count) {
        hit = (hits >> j) & 1u;
        if (!VALUES) flags[row] = hit ? 1 : 0;
      }
      if (!VALUES && match_rows != nullptr) {
        const uint64_t m = __ballot(hit);
        if (m) {
          const uint32_t lane = threadIdx.x & 63u;
          uint32_t base = 0;
          if (lane == 0) base = atomicAdd(match_count, (uint32_t)__popcll(m));
          base = __shfl(base, 0);
          if (hit) match_rows[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = row;
        }
      }
    }
  }
}

#define MATCH_PARAMS                                                                                        \
  const uint32_t *__restrict__ t_in, uint32_t n, uint32_t n_rows, const uint32_t *__restrict__ fb, ScanConsts k, \
      const uint32_t *__restrict__ labels, const int64_t *__restrict__ outputs, const uint32_t *__restrict__ offs, \
      const uint32_t *__restrict__ lens, uint32_t *__restrict__ lscr, uint8_t *__restrict__ flags,               \
      uint32_t *__restrict__ match_rows, uint32_t *__restrict__ match_count, int64_t *__restrict__ values
#define MATCH_ARGS t_in, n, n_rows, fb, k, labels, outputs, offs, lens, lscr, flags, match_rows, match_count, values

// Stage B with the fixed-base table in HBM (22- or 26-bit windows).
template <bool VALUES, int R, int FBB>
__global__ __launch_bounds__(BLOCK, CUDASP_WAVES_B) void k_match(MATCH_PARAMS) {
  match_body<VALUES, R, FBB>(MATCH_ARGS);
}

// Stage B with LDS-staged fixed-base windows (the north star's layout): the
// 7-bit table (37 windows x 64 odd multiples x 64 B = 151.5 KB) is copied from
// HBM into the workgroup's LDS, then t*G reads its 37 entries per row from
// LDS.  One 768-thread workgroup per CU (12 waves, 3 per SIMD).  Selected by
// a scanner's fixed-base width 7; measured against the HBM tables:
// 36 mixed additions per row instead of 9 cost far more than the 10 HBM
// gathers they replace.
constexpr int LDS_BLOCK = 768;
constexpr int LDS_FB_BITS = 7;
constexpr uint32_t LDS_FB_WORDS = FbWidth<LDS_FB_BITS>::WINDOWS * FbWidth<LDS_FB_BITS>::ENTRIES * FB_WORDS;
template <bool VALUES, int R>
__global__ __launch_bounds__(LDS_BLOCK, 1) void k_match_lds(MATCH_PARAMS) {
  __shared__ uint4 tab[LDS_FB_WORDS / 4];
  const uint4* src = reinterpret_cast<const uint4*>(fb);
  for (uint32_t i = threadIdx.x; i < LDS_FB_WORDS / 4; i += blockDim.x) tab[i] = src[i];
  __syncthreads();
  const uint32_t* lfb = reinterpret_cast<const uint32_t*>(tab);
  match_body<VALUES, R, LDS_FB_BITS>(t_in, n, n_rows, lfb, k, labels, outputs, offs, lens, lscr, flags, match_rows,
                                     match_count, values);
}

// K > 1 output indices: a row matches when any of its K virtual rows does;
// flags and the ballot compaction of k_match, over the input rows.
__global__ __launch_bounds__(BLOCK) void k_or_flags(const uint8_t* __restrict__ vflags, uint32_t n, uint32_t K,
                                                    uint8_t* __restrict__ flags, uint32_t* __restrict__ match_rows,
                                                    uint32_t* __restrict__ match_count) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t r0 = blockIdx.x * blockDim.x; r0 < n; r0 += stride) {
    const uint32_t row = r0 + threadIdx.x;
    bool hit = false;
    if (row < n) {
      for (uint32_t kk = 0; kk < K; kk++) hit = hit || vflags[(size_t)kk * n + row] != 0;
      flags[row] = hit ? 1 : 0;
    }
    if (match_rows != nullptr) {
      const uint64_t m = __ballot(hit);
      if (m) {
        const uint32_t lane = threadIdx.x & 63u;
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(match_count, (uint32_t)__popcll(m));
        base = __shfl(base, 0);
        if (hit) match_rows[base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = row;
      }
    }
  }
}

// ------------------------------------------------ multi-batch persistent scan
// cudasp_scan_device_batches: both stages of every row of several resident
// batches in ONE persistent kernel.  The batches' rows form a virtual row
// space in 64-row "wave-rows" (batch b starts at wave-row first_wr; its last
// wave-row is padded, padding lanes compute batch row 0 and store nothing).
// Each wavefront takes R consecutive wave-rows from a device counter (one
// atomic per piece) of R rows per thread, 1 .. rmax (<= MULTI_RMAX): by
// default the wave's share of the work left, rem x (rows it has claimed) /
// (rows all have claimed) (multi_piece_rows_adaptive: the waves of a SIMD
// progress at very different rates, so each is sized by its own), else
// guided self-scheduling, rem / (grid waves) (multi_piece_rows) -- no piece
// outlasts the work left to the other waves and the GPU stays full to the end
// (a fused single-batch launch uses g1 = 0: rmax rows per thread throughout).  A
// thread's R rows share one Z inversion in stage A (t stays in the thread),
// then one Z inversion and one label inversion in stage B.  PIPE (the default): a wave finishes a piece's
// stage B one iteration later and its labels one more iteration later, so the
// piece's stage-B Z inversion and its label inversion join the following
// pieces' stage-A inversions -- one inversion per piece instead of two (three
// with labels).  Exit: every wave leaves when the counter passes the last
// wave-row and its last pieces are finished.
#ifndef CUDASP_MULTI_RMAX
#define CUDASP_MULTI_RMAX 6
#endif
constexpr int MULTI_RMAX = CUDASP_MULTI_RMAX;  // rows per thread while much work remains (tuned)
static_assert(MULTI_RMAX >= 2 && MULTI_RMAX <= 16, "multi-batch rows per thread");
static_assert(ROWS_A <= MULTI_RMAX, "the fused single-batch launch runs ROWS_A rows per thread in k_scan_multi");
// Scratch of a k_scan_multi thread (u32 words from the slot's base): the
// stage-A table, then the pending slots -- one piece's, or with the pipelined
// schedule (PIPE) the previous piece's F points beside the new piece's S
// points plus one slot for the label product of the piece before that --,
// the label prefix products of one piece, and (PIPE with labels) that piece's
// affine F points and label product while their inversion is pending.
constexpr int multi_pend_slots(bool pipe) { return pipe ? 2 * MULTI_RMAX + 1 : MULTI_RMAX; }
constexpr uint32_t multi_scratch_words(uint32_t label_count, bool pipe) {
  return VB_SCRATCH_WORDS + PEND_WORDS * multi_pend_slots(pipe) + FW * label_count * MULTI_RMAX +
         (pipe && label_count ? 2 * FW * MULTI_RMAX + FW : 0);
}

// Wave-row w of the batches as (descriptor, batch row) of this lane.
__device__ __forceinline__ const MultiBatch& multi_locate(const MultiBatch* __restrict__ bd, uint32_t nb, uint32_t w,
                                                          uint32_t lane, uint32_t* r, bool* active) {
  const MultiBatch& b = bd[multi_batch_of(bd, nb, w)];
  *r = multi_row(b, w, lane, active);
  return b;
}

// Flags of rows base .. base + count - 1 (hits: bit j = row j matched) and
// their compaction, one wave-row (= one batch) at a time.
__device__ __forceinline__ void multi_emit(const MultiBatch* __restrict__ bd, uint32_t nb, uint32_t base, int count,
                                           uint32_t lane, uint32_t hits) {
#pragma unroll 1
  for (int j = 0; j < count; j++) {
    uint32_t r;
    bool active;
    const MultiBatch& b = multi_locate(bd, nb, base + (uint32_t)j, lane, &r, &active);
    const bool hit = active && ((hits >> j) & 1u);
    if (active) b.flags[r] = hit ? 1 : 0;
    if (b.match_rows != nullptr) {
      const uint64_t m = __ballot(hit);
      if (m) {
        uint32_t at = 0;
        if (lane == 0) at = atomicAdd(b.match_count, (uint32_t)__popcll(m));
        at = __shfl(at, 0);
        if (hit) b.match_rows[at + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = r;
      }
    }
  }
}

// Stage B's second half for the `count` rows from wave-row `base` whose F
// points wait in pending slots 0 .. count - 1 with their 1/Z: base compare,
// labels (one batched inversion), flags and compaction.
__device__ __forceinline__ void multi_finish(const MultiBatch* __restrict__ bd, uint32_t nb, uint32_t base, int count,
                                             uint32_t lane, const ScanConsts& k, const uint32_t* __restrict__ labels,
                                             const Scratch& sc, int pb, int lb) {
  uint32_t hits = 0;
#pragma unroll 1
  for (int j = 0; j < count; j++) {
    uint32_t r;
    bool active;
    const MultiBatch& b = multi_locate(bd, nb, base + (uint32_t)j, lane, &r, &active);
    gej P;
    fe zi;
    pend_load(P, sc, pb, j);
    scr_load(zi, sc, PEND_ZI(pb, j));
    if (row_match_base(P, zi, k, b.outputs, b.offs[r], b.lens[r], sc, pb, j, nullptr)) hits |= 1u << j;
  }
  if (k.label_count)
    hits |= match_labels_core(k, labels, count, sc, pb, lb,
                              [&](int j, const int64_t*& o, uint32_t& off, uint32_t& len, int64_t*& vrow,
                                  uint32_t& vstride) {
                                uint32_t r;
                                bool active;
                                const MultiBatch& b = multi_locate(bd, nb, base + (uint32_t)j, lane, &r, &active);
                                o = b.outputs;
                                off = b.offs[r];
                                len = b.lens[r];
                                vrow = nullptr;
                                vstride = 0;
                              });
  multi_emit(bd, nb, base, count, lane, hits);
}

// Measurement builds only (-DCUDASP_MULTI_TRACE=1, tools/multi_trace.py): per
// wave of the last k_scan_multi launch, its start and end (s_memrealtime
// ticks), pieces and wave-rows, its placement (HW_ID | XCC_ID << 32), when it
// first found the counter exhausted, shader-clock ticks (s_memtime) over its
// life and when its last stage-A row ended, read back by
// cudasp_debug_multi_trace.
#ifndef CUDASP_MULTI_TRACE
#define CUDASP_MULTI_TRACE 0
#endif
#if CUDASP_MULTI_TRACE
constexpr uint32_t MULTI_TRACE_WAVES = 8192;
constexpr uint32_t MULTI_TRACE_WORDS = 8;
__device__ uint64_t g_multi_trace[MULTI_TRACE_WAVES * MULTI_TRACE_WORDS];
__device__ __forceinline__ uint64_t trace_placement() {
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  return (uint64_t)hw | ((uint64_t)xcc << 32);
}
#endif

// The wave's issue priority, 0 .. 3 (s_setprio takes an immediate).
__device__ __forceinline__ void set_wave_prio(uint32_t level) {
  switch (level) {
    case 0:
      __builtin_amdgcn_s_setprio(0);
      break;
    case 1:
      __builtin_amdgcn_s_setprio(1);
      break;
    case 2:
      __builtin_amdgcn_s_setprio(2);
      break;
    default:
      __builtin_amdgcn_s_setprio(3);
      break;
  }
}

// The ladder hook of k_scan_multi (the drain): once the work counter has run
// out, the SIMDs' waves issue youngest first.  Until then the oldest wave of a
// SIMD issues first and the youngest gets ~4% of it, so the youngest's last
// piece is the SIMD's last work and runs alone (1 wave on the SIMD) after the
// others have left: tools/multi_trace.py finds the youngest wave ending last
// on 77-100% of the SIMDs, its stage A ending ~0.6 ms after the counter ran
// out at 4M rows.  Reversed, it finishes while the older waves fill its
// stalls, and the older ones (whose last pieces are short: they claim most
// often) finish after it.  The wave's tier comes from its block (the
// dispatcher places a CU-count of blocks at a time: `young_from` = 2 x CUs on
// the full grid, ~0 otherwise); the priority is set once, at the first ladder
// tick or claim that finds the counter out.  Claims and piece sizes are
// untouched.
struct MultiTick {
  const uint32_t* counter;
  uint32_t total_wr;
  bool* out;       // the counter has run out (sticky, wave-uniform)
  uint32_t level;  // the priority to take then (0: none)
  __device__ __forceinline__ void ladder(int, uint32_t) const {
    if (level == 0 || *out) return;
    const uint32_t c = __hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((uint32_t)__builtin_amdgcn_readfirstlane((int)c) < total_wr) return;
    *out = true;
    set_wave_prio(level);
  }
};


// The shader clock of the last k_scan_multi launch (cudasp_debug_multi_clock,
// measurement only: the bench line's clock, which differs by a few percent
// between boxes): the grid's first wave's s_memtime and s_memrealtime at its
// start and end (it is its SIMD's oldest wave and runs until the drain).
__device__ uint64_t g_multi_clock[4];

template <int FBB, bool PIPE>
__global__ __launch_bounds__(BLOCK, CUDASP_WAVES_A) void k_scan_multi(const MultiBatch* __restrict__ bd, uint32_t nb,
                                                                   uint32_t total_wr, const int8_t* __restrict__ naf,
                                                                   ScanConsts k, const uint32_t* __restrict__ fb,
                                                                   const uint32_t* __restrict__ labels,
                                                                   uint32_t* __restrict__ scr,
                                                                   uint32_t* __restrict__ counter, uint32_t g1,
                                                                   uint32_t g2, uint32_t rmax, uint32_t adaptive,
                                                                   uint32_t young_from, uint32_t tier_blocks) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  const Scratch sc = make_scratch(scr, gridDim.x * blockDim.x, slot);
  const uint32_t lane = threadIdx.x & 63u;
#if CUDASP_MULTI_LDS_Y
  // the y of odd multiples 0 .. CUDASP_MULTI_LDS_Y - 1 (LdsY): 45 KB per block
  // at 5, so three blocks per CU fit the 160 KB
  __shared__ uint32_t ytab[CUDASP_MULTI_LDS_Y * FW][BLOCK];
#endif
  constexpr int PB = VB_SCRATCH_WORDS;                             // pending rows
  constexpr int LB = VB_SCRATCH_WORDS + PEND_WORDS * multi_pend_slots(PIPE);  // label prefix products
  const int QF = LB + FW * (int)k.label_count * MULTI_RMAX;  // PIPE: piece Q's affine F (x, y per row)
  const int QACC = QF + 2 * FW * MULTI_RMAX;                 // PIPE: piece Q's label product
  // PIPE: piece P's F points wait in slots 0 .. count_p - 1 for their 1/Z;
  // with labels, piece Q (base compared, label prefix products formed) waits
  // for the inverse of its label product.  Each joins the next iteration's
  // inversion, so a piece costs one inversion instead of three.
  uint32_t base_p = 0, base_q = 0, hits_q = 0;
  int count_p = 0, count_q = 0;
  bool more = true;
  uint32_t mine = 0;  // wave-rows this wave has claimed (lane 0)
  bool out = false;   // MultiTick: the counter has run out
  const bool clock_wave = blockIdx.x == 0 && threadIdx.x == 0u;  // (nothing held across the loop)
  if (clock_wave) {
    g_multi_clock[0] = __builtin_amdgcn_s_memtime();
    g_multi_clock[1] = wall_clock64();
  }
  // MultiTick's priority: youngest first (blocks from 2 x tier_blocks), then
  // the middle tier (from tier_blocks); the oldest keep 0; tier_blocks = 0: off
  const uint32_t drain_level = tier_blocks == 0u                  ? 0u
                               : blockIdx.x >= 2u * tier_blocks   ? 3u
                               : blockIdx.x >= tier_blocks        ? 2u
                                                                  : 0u;
#if CUDASP_MULTI_TRACE
  const uint64_t trace_t0 = wall_clock64(), trace_c0 = __builtin_amdgcn_s_memtime();
  uint64_t trace_tx = 0, trace_ta = 0;
  uint32_t trace_pieces = 0, trace_rows = 0;
#endif
  for (;;) {
    uint32_t base = 0;
    int count = 0;
    if (more) {
      uint32_t R = 1;
      if (lane == 0) {
        const uint32_t prev = __hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t rem = prev < total_wr ? total_wr - prev : 0u;
        R = adaptive ? multi_piece_rows_adaptive(rem, prev, mine, g1, g2, rmax, blockIdx.x >= young_from)
                     : multi_piece_rows(rem, g1, g2, rmax);
        base = R ? atomicAdd(counter, R) : total_wr;  // R = 0: this wave leaves
        mine += R;
      }
      base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
      R = (uint32_t)__builtin_amdgcn_readfirstlane((int)R);
      if (base >= total_wr) {
        more = false;
        if (drain_level && !out) {  // MultiTick's drain priority
          out = true;
          set_wave_prio(drain_level);
        }
      } else {
        count = (int)(R < total_wr - base ? R : total_wr - base);
      }
#if CUDASP_MULTI_TRACE
      if (!more) trace_tx = wall_clock64();
#endif
    }
    if (count == 0 && count_p == 0 && count_q == 0) break;
#if CUDASP_MULTI_TRACE
    trace_pieces += count ? 1u : 0u;
    trace_rows += (uint32_t)count;
#endif
    // stage A: S = d T of the piece's rows (after the previous piece's F points)
#pragma unroll 1
    for (int j = 0; j < count; j++) {
      uint32_t r;
      bool active;
      const MultiBatch& b = multi_locate(bd, nb, base + (uint32_t)j, lane, &r, &active);
      uint32_t x[8], y[8];
#pragma unroll
      for (int q = 0; q < 8; q++) {
        x[q] = b.tx[(size_t)q * b.n + r];
        y[q] = b.ty[(size_t)q * b.n + r];
      }
      gej P;
#if CUDASP_MULTI_LDS_Y
      row_shared_secret_point_t(P, x, y, naf, k.naf_len, sc, MultiTick{counter, total_wr, &out, drain_level},
                                LdsY<CUDASP_MULTI_LDS_Y>{&ytab[0][threadIdx.x], BLOCK});
#else
      row_shared_secret_point_t(P, x, y, naf, k.naf_len, sc,
                                MultiTick{counter, total_wr, &out, drain_level});
#endif
      pend_store(sc, PB, count_p + j, P);
    }
#if CUDASP_MULTI_TRACE
    if (count) trace_ta = wall_clock64();
#endif
    if constexpr (!PIPE) {
      pend_invert<MULTI_RMAX>(sc, PB, count);
    } else {
      // one inversion: the new S points, piece P's F points, piece Q's label product
      int ninv = count_p + count;
      if (count_q) {
        fe acc;
        scr_load(acc, sc, QACC);
        scr_store(sc, PEND_Z(PB, ninv), acc);
        ninv++;
      }
      pend_invert<2 * MULTI_RMAX + 1>(sc, PB, ninv);
      const auto qf_at = [&](int j, ge& F) {
        scr_load(F.x, sc, QF + 2 * FW * j);
        scr_load(F.y, sc, QF + 2 * FW * j + FW);
      };
      const auto q_out = [&](int j, const int64_t*& o, uint32_t& off, uint32_t& len, int64_t*& vrow,
                             uint32_t& vstride) {
        uint32_t r;
        bool active;
        const MultiBatch& b = multi_locate(bd, nb, base_q + (uint32_t)j, lane, &r, &active);
        o = b.outputs;
        off = b.offs[r];
        len = b.lens[r];
        vrow = nullptr;
        vstride = 0;
      };
      if (count_q) {  // piece Q: its labels, then its flags
        fe inv;
        scr_load(inv, sc, PEND_ZI(PB, ninv - 1));
        hits_q |= labels_backward(inv, k, labels, count_q, sc, LB, qf_at, q_out);
        multi_emit(bd, nb, base_q, count_q, lane, hits_q);
        count_q = 0;
      }
      if (count_p) {  // piece P: affine F, base compare; its labels wait one iteration
        uint32_t hits = 0;
#pragma unroll 1
        for (int j = 0; j < count_p; j++) {
          uint32_t r;
          bool active;
          const MultiBatch& b = multi_locate(bd, nb, base_p + (uint32_t)j, lane, &r, &active);
          gej P;
          fe zi;
          pend_load(P, sc, PB, j);
          scr_load(zi, sc, PEND_ZI(PB, j));
          ge F;
          gej_to_ge_zinv(F, P, zi);
          if (k.label_count) {
            scr_store(sc, QF + 2 * FW * j, F.x);
            scr_store(sc, QF + 2 * FW * j + FW, F.y);
          }
          if (outputs_match(k, b.outputs, b.offs[r], b.lens[r], F.x, fe_upper64(F.x))) hits |= 1u << j;
        }
        if (k.label_count) {
          fe acc;
          labels_forward(acc, k, labels, count_p, sc, LB, qf_at);
          scr_store(sc, QACC, acc);
          base_q = base_p;
          count_q = count_p;
          hits_q = hits;
        } else {
          multi_emit(bd, nb, base_p, count_p, lane, hits);
        }
      }
    }
    // t of each row, then stage B's F = t G + B into slot j
#pragma unroll 1
    for (int j = 0; j < count; j++) {
      gej P;
      fe zi;
      pend_load(P, sc, PB, count_p + j);
      scr_load(zi, sc, PEND_ZI(PB, count_p + j));
      uint32_t sx[8], t[8];
      const uint32_t y_odd = row_shared_secret_affine(sx, P, zi);
      bip352_shared_secret_hash(t, k.mid, sx, y_odd);
      gej F;
      row_match_point<FBB>(F, t, fb, k);
      pend_store(sc, PB, j, F);  // slot count_p + j' (j' < j) is consumed already
    }
    if constexpr (PIPE) {
      base_p = base;
      count_p = count;
    } else {
      pend_invert<MULTI_RMAX>(sc, PB, count);
      multi_finish(bd, nb, base, count, lane, k, labels, sc, PB, LB);
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0u) {
    g_multi_clock[2] = __builtin_amdgcn_s_memtime();
    g_multi_clock[3] = wall_clock64();
  }
#if CUDASP_MULTI_TRACE
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64u;
  const uint64_t trace_c1 = __builtin_amdgcn_s_memtime(), trace_t1 = wall_clock64();
  if (lane == 0 && wave < MULTI_TRACE_WAVES) {
    uint64_t* rec = g_multi_trace + (size_t)wave * MULTI_TRACE_WORDS;
    rec[0] = trace_t0;
    rec[1] = trace_t1;
    rec[2] = trace_pieces;
    rec[3] = trace_rows;
    rec[4] = trace_placement();
    rec[5] = trace_tx;
    rec[6] = trace_c1 - trace_c0;
    rec[7] = trace_ta;
  }
#endif
}

// ------------------------------------------------------------ streaming scan
// k_scan_stream: k_scan_multi's pipelined body over batches the host publishes
// while the kernel runs (scan_stream.hpp: zero-copy inputs from pinned host
// memory, ticket claims and batch lookups in a device mirror of the host's
// descriptor ring, per-batch completion words).

__device__ __forceinline__ uint32_t sys_load_u32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t sys_load_u64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t dev_load_u32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t dev_load_u64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32);
}

// Measurement builds only (-DCUDASP_STREAM_TRACE=1, tools/stream_trace.py):
// timestamped events of k_scan_stream (wave starts with their hardware
// placement, claims, pieces, iteration ends, exits, batches mirrored and
// completed), appended by cudasp_stream_finish to $CUDASP_STREAM_TRACE_FILE.
#ifndef CUDASP_STREAM_TRACE
#define CUDASP_STREAM_TRACE 0
#endif
#if CUDASP_STREAM_TRACE
struct StreamTraceEv {
  uint64_t t, a;
  uint32_t wave, kind, b, c;
};
enum { ST_START = 1, ST_CLAIM, ST_PIECE, ST_ITER_END, ST_EXIT, ST_PUB, ST_DONE };
constexpr uint32_t STREAM_TRACE_CAP = 1u << 21;
__device__ uint32_t g_st_n;
__device__ StreamTraceEv g_st_ev[STREAM_TRACE_CAP];
__device__ __forceinline__ void st_ev(uint32_t kind, uint32_t wave, uint64_t a, uint32_t b, uint32_t c) {
  const uint32_t i = atomicAdd(&g_st_n, 1u);
  if (i < STREAM_TRACE_CAP) {
    StreamTraceEv e;
    e.t = wall_clock64();
    e.a = a;
    e.wave = wave;
    e.kind = kind;
    e.b = b;
    e.c = c;
    g_st_ev[i] = e;
  }
}
#define ST_EV(...) st_ev(__VA_ARGS__)
// host-side events of the same query (wave = ~0u, t = steady_clock ns)
static std::mutex g_st_host_mu;
static std::vector<StreamTraceEv> g_st_host;
extern "C" void cudasp_internal_trace_host(uint32_t kind, uint64_t a, uint32_t b) {
  StreamTraceEv e;
  e.t = (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
            std::chrono::steady_clock::now().time_since_epoch())
            .count();
  e.a = a;
  e.wave = ~0u;
  e.kind = kind;
  e.b = b;
  e.c = 0;
  std::lock_guard<std::mutex> lk(g_st_host_mu);
  g_st_host.push_back(e);
}
#define ST_HOST(...) cudasp_internal_trace_host(__VA_ARGS__)
#else
#define ST_EV(...) ((void)0)
#define ST_HOST(...) ((void)0)
#endif

// A wave-row's batch, wave-uniform.
struct StreamRow {
  const uint8_t* rows;
  const int64_t* outputs;
  const uint32_t* offs;
  const uint32_t* lens;
  uint8_t* flags;
  uint32_t* matches;
  int64_t* mirror;
  uint64_t first_wr;
  uint32_t n;
  uint32_t nwr;
  uint32_t b;
};

// The batch holding published wave-row w, searched forward from `hint` (the
// batch of an earlier wave-row of this wave's tickets).  A ring entry holding
// another sequence number was reused: that batch is complete, hence before
// w's (w is this wave's and not done yet).  The walk starts no earlier than
// pub - STREAM_RING: the host publishes batch X only once X - STREAM_RING is
// done, so every batch below that is done and w's lies at or above it (a
// wave's first hint is 0, which once the ring has wrapped twice would leave
// a walk from the hint short of w's batch).  A stale `pub` lowers the start
// by at most one poller pass (STREAM_RING batches), so three passes of the
// ring bound the walk.
__device__ __forceinline__ uint32_t stream_batch_of(StreamDev* dev, uint32_t hint, uint64_t w) {
  uint32_t b = hint;
  const uint32_t pub = dev_load_u32(&dev->pub);
  if (pub > STREAM_RING && b < pub - STREAM_RING) b = pub - STREAM_RING;
  for (uint32_t i = 0; i < 3 * STREAM_RING; i++, b++) {
    // seqlock read: the poller rewrites an entry (batch b + STREAM_RING,
    // once b is done) with its seq invalidated first and set last, so a
    // range read between two equal seq loads belongs to batch b; an entry
    // rewritten meanwhile held a done batch, not w's
    // (agent-scope loads are served by the L2, so ordering them with vmcnt
    // waits is the acquire; no cache of the CU is invalidated)
    const StreamBatch* d = &dev->desc[b % STREAM_RING];
    if (dev_load_u64(&d->seq) != b) continue;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint64_t end = dev_load_u64(&d->first_wr) + dev_load_u32(&d->nwr);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (dev_load_u64(&d->seq) != b) continue;
    if (w < end) break;
  }
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
}

__device__ __forceinline__ StreamRow stream_row(StreamDev* dev, uint32_t& hint, uint64_t w) {
  const uint32_t b = stream_batch_of(dev, hint, w);
  hint = b;
  const StreamBatch* d = &dev->desc[b % STREAM_RING];
  StreamRow r;
  const auto ptr = [&](auto* const* f) {
    using T = std::remove_reference_t<decltype(**f)>;
    return reinterpret_cast<T*>(uniform_u64(dev_load_u64(reinterpret_cast<const uint64_t*>(f))));
  };
  r.rows = ptr(&d->rows);
  r.outputs = ptr(&d->outputs);
  r.offs = ptr(&d->offs);
  r.lens = ptr(&d->lens);
  r.flags = ptr(&d->flags);
  r.matches = ptr(&d->matches);
  r.mirror = ptr(&d->mirror);
  r.first_wr = uniform_u64(dev_load_u64(&d->first_wr));
  r.n = (uint32_t)__builtin_amdgcn_readfirstlane((int)dev_load_u32(&d->n));
  r.nwr = (uint32_t)__builtin_amdgcn_readfirstlane((int)dev_load_u32(&d->nwr));
  r.b = b;
  return r;
}

// The poller (lane 0 of one wave per kernel): mirrors new batches of the
// host's control block into the device state -- descriptors first, then the
// counts behind an agent-scope release -- and `closed` after the last one.
// Leaves once closed is mirrored, or once the kernel has had nothing to do
// for idle_ticks (no new batch, every published row claimed): it then sets
// `idle`, the workers leave as they drain, and the GPU is free until the
// host's next publish or wait relaunches the kernel (cudasp_stream_*).
__device__ void stream_poll(StreamCtrl* ctrl, StreamDev* dev, uint64_t idle_ticks) {
  uint32_t seen = dev_load_u32(&dev->pub);
  uint64_t last = wall_clock64();
  uint64_t polls = 0;
  for (;;) {
    // the control block is uncached host memory (MTYPE UC): relaxed
    // system-scope loads read it fresh without invalidating any cache; the
    // wait keeps `published` read after `closed`
    const uint32_t cl = sys_load_u32(&ctrl->closed);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t pub = sys_load_u32(&ctrl->published);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the descriptors are read after `published`
    const uint64_t now = wall_clock64();
    if (pub != seen) {
      uint64_t pub_wr = 0;
      uint32_t b = seen;
      for (; b != pub; b++) {
        const uint64_t* src = reinterpret_cast<const uint64_t*>(&ctrl->desc[b % STREAM_RING]);
        StreamBatch* de = &dev->desc[b % STREAM_RING];
        uint64_t* dst = reinterpret_cast<uint64_t*>(de);
        StreamBatch d;
        uint64_t* dw = reinterpret_cast<uint64_t*>(&d);
        // seqlock write (stream_batch_of): seq invalid, the fields, then seq.
        // Every store is an agent-scope relaxed one (global_store sc1: written
        // through to memory, the line dropped from this XCD's L2) and each
        // step waits for the previous one's stores to complete (vmcnt), which
        // orders them for the workers' sc1 loads on any XCD -- no release
        // fence: on gfx950 that is buffer_wbl2, a write-back of the whole
        // L2's dirty lines (here the workers' scratch), stalling this XCD's
        // memory traffic several times per mirrored batch (round 4)
        static_assert(offsetof(StreamBatch, seq) + 8 == sizeof(StreamBatch), "seq is the descriptor's last word");
        __hip_atomic_store(&de->seq, ~0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int i = 0; i < (int)(sizeof(StreamBatch) / 8); i++) dw[i] = sys_load_u64(src + i);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int i = 0; i < (int)(sizeof(StreamBatch) / 8) - 1; i++)
          __hip_atomic_store(dst + i, dw[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&de->seq, d.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the rows mirrored so far (not the host's published_wr, which may
        // already count a batch published after `pub` was read)
        pub_wr = d.first_wr + d.nwr;
      }
      if (b != seen) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the descriptors before the counts
        __hip_atomic_store(&dev->pub_wr, pub_wr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&dev->pub, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ST_EV(ST_PUB, 0u, pub_wr, b, seen);
        seen = b;
        last = now;
      }
    }
    if (cl && seen == pub) {  // `published` was read after `closed`: every batch is mirrored
      __hip_atomic_store(&dev->closed, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    if (dev_load_u64(&dev->ticket) < dev_load_u64(&dev->pub_wr)) {
      last = now;  // rows still unclaimed: not idle
    } else if (now - last > idle_ticks) {
      __hip_atomic_store(&dev->idle, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      atomicAdd(&dev->stat[STREAM_STAT_IDLE_EXITS], 1ull);
      break;
    }
    polls++;
    __builtin_amdgcn_s_sleep(32);
  }
  atomicAdd(&dev->stat[STREAM_STAT_POLLER_POLLS], (unsigned long long)polls);
}

// The batch-complete word's release (stream_emit): 1 = a system-scope
// release fence before it (A/B; see the comment there).
#ifndef CUDASP_STREAM_RELEASE_FENCE
#define CUDASP_STREAM_RELEASE_FENCE 1
#endif

// Raw scratch words (column-major like scr_load / scr_store).
__device__ __forceinline__ void scr_store_w(const Scratch& sc, int w, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_raw_buffer_store_b32(v, sc.rsrc, sc.slot * 4u, (uint32_t)w * sc.stride * 4u, CUDASP_SCR_STORE_CPOL);
#else
  sc.s[(size_t)w * sc.stride + sc.slot] = v;
#endif
}
__device__ __forceinline__ uint32_t scr_load_w(const Scratch& sc, int w) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_raw_buffer_load_b32(sc.rsrc, sc.slot * 4u, (uint32_t)w * sc.stride * 4u,
                                              CUDASP_SCR_LOAD_CPOL);
#else
  return sc.s[(size_t)w * sc.stride + sc.slot];
#endif
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o));
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// Scratch of a k_scan_stream thread (u32 words from the slot's base):
// k_scan_multi's pipelined layout, then the new piece's row blobs (16 words
// per wave-row), the offsets and lengths of the three pieces in flight (new,
// P, Q: 2 words per wave-row each) and, with output_count > 1, the new
// piece's affine shared-secret x and y parity (9 words per row).
constexpr int STREAM_STG_WORDS = 16 * MULTI_RMAX;
constexpr int STREAM_META_WORDS = 3 * 2 * MULTI_RMAX;
constexpr int STREAM_SXA_WORDS = 9 * MULTI_RMAX;
constexpr uint32_t stream_scratch_words(uint32_t label_count) {
  return multi_scratch_words(label_count, true) + STREAM_STG_WORDS + STREAM_META_WORDS + STREAM_SXA_WORDS;
}

// Host pointers of a piece's wave-rows, kept in LDS during its prefetch.
struct StreamPf {
  const uint8_t* rows;
  const int64_t* outputs;
  const uint32_t* offs;
  const uint32_t* lens;
};

// Outputs words [q0, q1) of one batch into its device mirror, the whole wave
// copying (lane-strided, 4 loads in flight per lane).
// A store into a batch's device mirror of its outputs: written through to
// memory (agent scope: global_store sc1, the line not kept in this XCD's L2).
// A mirror is rewritten whenever its slot carries a newer batch, by waves on
// any XCD; a plain store leaves the line dirty in its XCD's L2, and a
// write-back of such a line after the slot's next batch had rewritten it
// undid that batch's outputs (matches lost with 4 slots even behind the
// per-iteration acquire; profiles/r05_stream_acquire.txt).
__device__ __forceinline__ void mirror_store(int64_t* p, int64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void stream_copy_range(int64_t* mirror, const int64_t* outputs, uint32_t q0, uint32_t q1,
                                                  uint32_t lane) {
#pragma unroll 1
  for (uint32_t q = q0 + lane; q < q1; q += 4 * 64) {
    int64_t v[4];
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (q + 64u * i < q1) v[i] = outputs[q + 64u * i];
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (q + 64u * i < q1) mirror_store(mirror + q + 64u * i, v[i]);
  }
}

// Prefetch of a new piece (count wave-rows from `base`): each wave-row's
// batch looked up once (its StreamWr to LDS), then the row blobs into the
// staging words `stg`, the offsets and lengths into `meta` (0 for padding
// lanes) and the rows' outputs into the batch's device mirror -- all loads
// of up to 3 wave-rows in flight together, and one cooperative copy per
// group of wave-rows of one batch whose outputs lie close together (else
// each lane copies its own row's) -- so the piece's PCIe latencies are paid
// here, a few per piece, and nothing later reads host memory.
// coal: the row blobs are read lane-contiguously (lane i the i-th 16 bytes
// of each 1 KB of the wave-row's 4 KB, so every 4 lanes make one 64-byte
// request) and transposed through the wave's 4 KB of LDS (`tr`), instead of
// each lane reading its own 64-byte row in 16-byte pieces (64-byte-strided
// lanes: over uncached pinned memory every piece is a request of its own).
__device__ __forceinline__ void stream_prefetch(StreamDev* dev, uint32_t& hint, uint64_t base, int count,
                                                uint32_t lane, StreamWr* wr, StreamPf* pf, const Scratch& sc,
                                                int stg, int meta, uint32_t ow, bool coal, uint4* tr) {
#pragma unroll 1
  for (int j = 0; j < count; j++) {
    if (j > 0 && wr[j - 1].r0 / 64u + 1u < wr[j - 1].nwr) {
      // the next wave-row of the previous one's batch: no lookup (the
      // batch's descriptor cannot change while this wave holds its rows)
      StreamWr w = wr[j - 1];
      w.r0 += 64u;
      wr[j] = w;
      pf[j] = pf[j - 1];
      continue;
    }
    const StreamRow sr = stream_row(dev, hint, base + (uint32_t)j);
    StreamWr w;
    w.mirror = sr.mirror;
    w.flags = sr.flags;
    w.matches = sr.matches;
    w.r0 = (uint32_t)(base + (uint32_t)j - sr.first_wr) * 64u;
    w.n = sr.n;
    w.nwr = sr.nwr;
    w.b = sr.b;
    wr[j] = w;  // every lane stores the same (wave-uniform) values
    StreamPf p;
    p.rows = sr.rows;
    p.outputs = sr.outputs;
    p.offs = sr.offs;
    p.lens = sr.lens;
    pf[j] = p;
  }
#pragma unroll 1
  for (int g = 0; g < count; g += 3) {
    uint4 v[3][4];
    uint32_t of[3], ln[3];
    bool act[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
      act[i] = false;
      of[i] = ln[i] = 0;
      if (g + i < count) {
        const uint32_t r0 = wr[g + i].r0;
        act[i] = r0 + lane < wr[g + i].n;
        const uint32_t r = act[i] ? r0 + lane : 0u;
        if (coal) {
          // 16-byte pieces lane + 64 q of the wave-row's rows (only those of
          // rows the batch has: the last wave-row may be partial)
          const uint32_t pieces = (wr[g + i].n - r0 < 64u ? wr[g + i].n - r0 : 64u) * 4u;
          const uint4* src = reinterpret_cast<const uint4*>(pf[g + i].rows + (size_t)r0 * 64);
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const uint32_t idx = lane + 64u * q;
            v[i][q] = idx < pieces ? src[idx] : make_uint4(0, 0, 0, 0);
          }
        } else {
          const uint4* src = reinterpret_cast<const uint4*>(pf[g + i].rows + (size_t)r * 64);
#pragma unroll
          for (int q = 0; q < 4; q++) v[i][q] = src[q];
        }
        // lengths, or none: Arrow list offsets (n + 1 of them, a row's list
        // from offs[r] to offs[r + 1]; cudasp_stream_batch)
        const uint32_t* lp = pf[g + i].lens;
        of[i] = pf[g + i].offs[r];
        ln[i] = lp != nullptr ? lp[r] : pf[g + i].offs[r + 1] - of[i];
      }
    }
#pragma unroll
    for (int i = 0; i < 3; i++) {
      if (g + i < count) {
        const int s0 = stg + 16 * (g + i);
        if (coal) {  // transpose: piece lane + 64 q to LDS, then this lane's row
#pragma unroll
          for (int q = 0; q < 4; q++) tr[lane + 64 * q] = v[i][q];
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int q = 0; q < 4; q++) v[i][q] = tr[4 * lane + q];
          __builtin_amdgcn_wave_barrier();
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
          scr_store_w(sc, s0 + 4 * q, v[i][q].x);
          scr_store_w(sc, s0 + 4 * q + 1, v[i][q].y);
          scr_store_w(sc, s0 + 4 * q + 2, v[i][q].z);
          scr_store_w(sc, s0 + 4 * q + 3, v[i][q].w);
        }
        if (!act[i]) ln[i] = 0;
        scr_store_w(sc, meta + 2 * (g + i), of[i]);
        scr_store_w(sc, meta + 2 * (g + i) + 1, ln[i]);
      }
    }
    // the outputs: runs of wave-rows of one batch whose lists span at most
    // 48 words per lane are copied by the whole wave; anything else (a
    // scattered CSR) lane by lane.
#ifdef CUDASP_AB_STREAM_ANY_MEMORY
    // measurement builds only (tools/stream_probe.py --device-inputs): a
    // batch whose outputs already are its device mirror needs no copy
    bool resident = true;
#pragma unroll
    for (int i = 0; i < 3; i++)
      if (g + i < count) resident = resident && wr[g + i].mirror == pf[g + i].outputs;
    if (resident) continue;
#endif
#ifdef CUDASP_AB_NO_OUTCOPY
    continue;  // measurement only: compares read a stale mirror
#endif
    uint32_t lo = ~0u, hi = 0;
    int i0 = 0;
#pragma unroll
    for (int i = 0; i <= 3; i++) {
      const bool in = g + i < count && i < 3;
      const bool flush = !in || (i > i0 && wr[g + i].b != wr[g + i0].b);
      if (flush && i > i0) {
        int64_t* mir = wr[g + i0].mirror;
        const int64_t* out = pf[g + i0].outputs;
        if (hi > lo && (uint64_t)(hi - lo) * ow <= 48u * 64u) {
          stream_copy_range(mir, out, lo * ow, hi * ow, lane);
        } else if (hi > lo) {
#pragma unroll
          for (int t = 0; t < 3; t++)
            if (t >= i0 && t < i) {
#pragma unroll 1
              for (uint32_t q = of[t] * ow; q < (of[t] + ln[t]) * ow; q++) mirror_store(mir + q, out[q]);
            }
        }
        lo = ~0u;
        hi = 0;
        i0 = i;
      }
      if (in) {
        lo = min(lo, wave_min_u32(ln[i] ? of[i] : ~0u));
        hi = max(hi, wave_max_u32(ln[i] ? of[i] + ln[i] : 0u));
      }
    }
  }
}

// Results of the piece's wave-rows (wr: their StreamWr, hits: bit j = row j
// of this lane matched) into the pinned slots -- one flag per row and/or the
// matching rows' indices (ballot compaction: one atomic per wave-row with a
// match) -- then each batch's completion: the wave's stores are complete
// before its wave-rows count, and the wave whose count finishes a batch
// writes the batch's match count and, behind a system-scope release, its
// done word.
__device__ __forceinline__ void stream_emit(StreamCtrl* ctrl, StreamDev* dev, const StreamWr* wr, int count,
                                            uint32_t lane, uint32_t hits) {
#pragma unroll 1
  for (int j = 0; j < count; j++) {
    const uint32_t r = wr[j].r0 + lane;
    const bool active = r < wr[j].n;
    const bool hit = active && ((hits >> j) & 1u);
    // system-scope stores: written through to host memory whatever the
    // caching type of the pinned pages
    uint8_t* flags = wr[j].flags;
    if (flags != nullptr && active)
      __hip_atomic_store(flags + r, (uint8_t)(hit ? 1 : 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* matches = wr[j].matches;
    if (matches != nullptr) {
      const uint64_t m = __ballot(hit);
      if (m) {
        uint32_t at = 0;
        if (lane == 0) at = atomicAdd(&dev->nmatch[wr[j].b % STREAM_RING], (uint32_t)__popcll(m));
        at = (uint32_t)__shfl((int)at, 0);
        if (hit)
          __hip_atomic_store(matches + at + (uint32_t)__popcll(m & ((1ull << lane) - 1ull)), r, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
#ifndef CUDASP_AB_NO_EMIT_WAIT
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the wave's stores are written before its rows count
#endif
  if (lane == 0) {
    // one count per run of wave-rows of one batch (a piece's usually are)
#pragma unroll 1
    for (int j = 0; j < count;) {
      int j1 = j + 1;
      while (j1 < count && wr[j1].b == wr[j].b) j1++;
      const uint32_t run = (uint32_t)(j1 - j);
      const uint32_t e = wr[j].b % STREAM_RING;
      const uint32_t nwr = wr[j].nwr;
      const uint32_t before = atomicAdd(&dev->wr_done[e], run);
      if (before + run == nwr) {
        // the entry's counts back to 0 for batch b + STREAM_RING (published
        // only after the host has seen this batch done); the subtraction
        // commutes with that batch's counts however late it lands
        atomicSub(&dev->wr_done[e], nwr);
        const uint32_t nm = atomicExch(&dev->nmatch[e], 0u);
        __hip_atomic_store(&ctrl->nmatch[e], nm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        // system-scope release, then the done word: the host's acquire of
        // `done` sees the match count and every result store before it
#if CUDASP_STREAM_RELEASE_FENCE
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
#endif
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(&ctrl->done[e], wr[j].b + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        ST_EV(ST_DONE, 0u, (uint64_t)nm, wr[j].b, nwr);
      }
      j = j1;
    }
  }
}

// The ladder hook of k_scan_stream: the wave's issue priority by the age of
// its oldest unfinished piece (stream_prio), refreshed every 16 ladder steps
// so that a starved wave rises while it is still in its ladder.
struct StreamTick {
  volatile StreamWave* me;
  uint64_t step;
  __device__ __forceinline__ void operator()() const {
#ifdef CUDASP_AB_NO_TICK
    return;
#endif
    if (step == 0) return;
    const uint64_t t_old = uniform_u64(me->t_old);
    set_wave_prio(stream_prio(wall_clock64() - t_old, step));
  }
  __device__ __forceinline__ void ladder(int, uint32_t) const { (*this)(); }
};

// Row bits of a label pass's unit bits (unit u = row u / K, index u % K).
__device__ __forceinline__ uint32_t stream_unit_rows(uint32_t uh, int K) {
  if (K == 1) return uh;
  uint32_t r = 0;
#pragma unroll 1
  for (int u = 0; u < MULTI_RMAX; u++)
    if ((uh >> u) & 1u) r |= 1u << (u / K);
  return r;
}

// WIDE: output_count K > MULTI_RMAX (one row per piece, its indices in groups
// of MULTI_RMAX, no pipelining) -- a separate instance, so the default
// instance's register allocation is the pipelined body's alone.
template <int FBB, bool WIDE>
__global__ __launch_bounds__(BLOCK, CUDASP_WAVES_A) void k_scan_stream(StreamCtrl* ctrl, StreamDev* dev,
                                                                    const int8_t* __restrict__ naf, ScanConsts k,
                                                                    const uint32_t* __restrict__ fb,
                                                                    const uint32_t* __restrict__ labels,
                                                                    uint32_t* __restrict__ scr, uint32_t rmax,
                                                                    uint64_t idle_ticks,
                                                                    unsigned long long* __restrict__ wstat,
                                                                    uint64_t prio_ticks, uint32_t pf_coal) {
  const uint32_t slot = blockIdx.x * blockDim.x + threadIdx.x;
  const Scratch sc = SCAN_SCRATCH(scr, gridDim.x * blockDim.x, slot);
  const uint32_t lane = threadIdx.x & 63u;
  if (blockIdx.x == 0 && threadIdx.x < 64) {  // one wave of the grid is the poller
    if (lane == 0) stream_poll(ctrl, dev, idle_ticks);
    return;
  }
  constexpr int PB = VB_SCRATCH_WORDS;
  constexpr int LB = VB_SCRATCH_WORDS + PEND_WORDS * multi_pend_slots(true);
  const int QF = LB + FW * (int)k.label_count * MULTI_RMAX;
  const int QACC = QF + 2 * FW * MULTI_RMAX;
  const int STG = (int)multi_scratch_words(k.label_count, true);
  const int META = STG + STREAM_STG_WORDS;  // piece area a: META + 2 MULTI_RMAX a
  const int SXA = META + STREAM_META_WORDS;
  // 1 .. CUDASP_MAX_OUTPUT_COUNT; K <= MULTI_RMAX: K x rmax <= MULTI_RMAX
  // units in the pipelined schedule; K > MULTI_RMAX (`wide`): one row per
  // piece, its K indices in groups of MULTI_RMAX, unpipelined (stream_wide)
  const int K = (int)k.output_count;
  constexpr bool wide = WIDE;
  const bool with_labels = k.label_count != 0;
  const uint32_t ow = k.full_x ? 4u : 1u;
  // pieces of the pipelined schedule: P (F points pending), Q (labels
  // pending), each with its wave-rows' StreamWr and offsets/lengths in piece
  // area pp / pq; the new piece's go to area pn
  int count_p = 0, count_q = 0;
  int pn = 0, pp = 1, pq = 2;
  uint32_t hint = 0, hits_q = 0;
  // lane 0's ticket and counters live in LDS, so none of them is held in
  // registers through a piece's ladders
  __shared__ StreamWave waves[BLOCK / 64];
  __shared__ StreamWr wrs[BLOCK / 64][3][MULTI_RMAX];
  __shared__ StreamPf pfs[BLOCK / 64][MULTI_RMAX];
  const uint32_t wid = threadIdx.x >> 6;
#if CUDASP_STREAM_LDS_Y
  // LdsY as in k_scan_multi, wave-major (a wave's y entries are one contiguous
  // area, 11.25 KB at 5), whose first 4 KB double as the prefetch's transpose
  // buffer: the prefetch runs between pieces, when no row's table is live, and a
  // wave's LDS operations complete in order
  constexpr int YW = CUDASP_STREAM_LDS_Y * FW * 64 > 1024 ? CUDASP_STREAM_LDS_Y * FW * 64 : 1024;
  __shared__ uint4 ywave[BLOCK / 64][YW / 4];
  uint4* const pftr_w = ywave[wid];  // the row blobs' transpose (stream_prefetch, coal)
  const LdsY<CUDASP_STREAM_LDS_Y> ytab{reinterpret_cast<uint32_t*>(ywave[wid]) + lane, 64};
#else
  __shared__ uint4 pftr[BLOCK / 64][256];  // the row blobs' transpose (stream_prefetch, coal)
  uint4* const pftr_w = pftr[wid];
#endif
  volatile StreamWave& me = waves[wid];
  if (lane == 0) {
    // the first ticket: one wave-row, worker w's at first_wr + w (k_stream_start)
    me.tk = dev_load_u64(&dev->first_wr) + (slot / 64u - 1u);
    me.tr = me.have = me.mine = 1;
    me.t_start = wall_clock64();
    me.busy = me.pieces = me.rows = me.polls = me.drains = 0;
    me.t_p = me.t_q = me.t_old = 0;
  }
  const StreamTick tick{&me, prio_ticks};
#if CUDASP_STREAM_TRACE
  const uint32_t st_wave = slot / 64u;
  if (lane == 0) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    ST_EV(ST_START, st_wave, (uint64_t)hw | ((uint64_t)xcc << 32), 0u, 0u);
  }
#endif
  bool stop = false;  // closed or idle, nothing published left in the ticket: leave once drained
  for (;;) {
    const uint64_t t_it = wall_clock64();
    uint32_t status = 0, cnt = 0;  // 0: nothing to do now; 1: cnt published rows of the ticket; 2: leave
    uint64_t tbase = 0;
    if (lane == 0 && !stop) {
      // the device state is read with agent-scope loads, which the L2 serves
      // (no L1 copy): ordering the loads (vmcnt) is all an acquire needs here,
      // and no cache of the CU is invalidated
      const uint32_t fin = dev_load_u32(&dev->closed) | dev_load_u32(&dev->idle);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // pub_wr is final once closed / idle is seen
      const uint64_t pw = dev_load_u64(&dev->pub_wr);
      if (!me.have) {
        // claim only while published rows are unclaimed: the wave's share of
        // them (k_scan_multi's adaptive rule).  A single atomicAdd, never a
        // retry (a compare-and-swap claim contends: 5M retries at 9.4M rows,
        // profiles/r03_stream_cas_claims.txt), so concurrent claims may pass
        // pub_wr; such a ticket waits for the host's next batch
        const uint64_t cur = dev_load_u64(&dev->ticket);
        if (pw > cur) {
          const uint32_t tr = stream_piece_rows(pw - cur, cur, me.mine, rmax);
          me.tk = atomicAdd(reinterpret_cast<unsigned long long*>(&dev->ticket), (unsigned long long)tr);
          me.tr = tr;
          me.mine = me.mine + tr;
          me.have = 1;
          ST_EV(ST_CLAIM, st_wave, me.tk, tr, (uint32_t)(pw - cur));
        }
      }
      const uint64_t tk = me.tk;
      if (me.have && tk < pw) {
        // the published part of the ticket now; an unpublished rest stays
        // the wave's ticket (the host may wait for this part's batch before
        // it publishes more)
        status = 1;
        const uint32_t tr = me.tr;
        cnt = tk + tr <= pw ? tr : (uint32_t)(pw - tk);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the mirrored descriptors after pub_wr
        tbase = tk;
        me.tk = tk + cnt;
        me.tr = tr - cnt;
        me.have = tr != cnt;
      } else if (fin) {
        // closed: the ticket lies past the last row; idle: its rows were
        // never published to this kernel (pub_wr is final), so none of them
        // is processed and the relaunch hands them out again from pub_wr
        status = 2;
        me.have = 0;
      }
    }
    status = (uint32_t)__builtin_amdgcn_readfirstlane((int)status);
    const int count = __builtin_amdgcn_readfirstlane((int)cnt);
    const uint64_t base = uniform_u64(tbase);
    if (status == 2) stop = true;
    if (count == 0 && count_p == 0 && count_q == 0) {
      if (stop) break;  // closed (or idle) and nothing left
      if (lane == 0) me.polls = me.polls + 1;
      __builtin_amdgcn_s_sleep(32);
      continue;
    }
    if (lane == 0) {
      if (count == 0) me.drains = me.drains + 1;
      if (count) {
        me.pieces = me.pieces + 1;
        me.rows = me.rows + (uint32_t)count;
      }
      ST_EV(ST_PIECE, st_wave, base, (uint32_t)count, (uint32_t)count_p | ((uint32_t)count_q << 8));
      // the oldest piece this wave holds: Q's, else P's, else the new one's
      me.t_old = count_q ? me.t_q : (count_p ? me.t_p : t_it);
    }
    tick();
    // A system-scope acquire (buffer_inv sc0 sc1: this CU's L1 and this XCD's
    // L2) before the iteration's reads of the new piece's pinned slots and of
    // the pending pieces' output mirrors.  A slot the host rewrote for a newer
    // batch, or a mirror rewritten for one (slot reuse), was otherwise read
    // from stale cached lines: rows scanned with another batch's tweaks or
    // compared against its outputs, matches lost (a streaming feed of 4 slots
    // lost 8-25% of its planted matches; tools/soak_host.py,
    // profiles/r05_stream_acquire.txt).  The batch's publication was observed
    // before this (pub_wr, then the mirrored ring).
#ifndef CUDASP_AB_PF_NO_ACQUIRE
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
#endif
    StreamWr* const wn = wrs[wid][pn];
    const int meta_n = META + 2 * MULTI_RMAX * pn;
    if (count) stream_prefetch(dev, hint, base, count, lane, wn, pfs[wid], sc, STG, meta_n, ow, pf_coal != 0, pftr_w);
    const int np = count_p * K;  // F points of piece P in pending slots 0 .. np - 1
    // stage A: S = d T of the new piece's rows (staged by the prefetch)
#pragma unroll 1
    for (int j = 0; j < count; j++) {
      uint32_t w[16];
#pragma unroll
      for (int q = 0; q < 16; q++) w[q] = scr_load_w(sc, STG + 16 * j + q);
      gej P;
#if CUDASP_STREAM_LDS_Y
      row_shared_secret_point_t(P, w, w + 8, naf, k.naf_len, sc, tick, ytab);
#else
      row_shared_secret_point_t(P, w, w + 8, naf, k.naf_len, sc, tick);
#endif
      pend_store(sc, PB, np + j, P);
    }
    // one inversion: the new S points, piece P's F points, piece Q's label product
    int ninv = np + count;
    if (count_q) {
      fe acc;
      scr_load(acc, sc, QACC);
      scr_store(sc, PEND_Z(PB, ninv), acc);
      ninv++;
    }
    pend_invert<2 * MULTI_RMAX + 1>(sc, PB, ninv);
    const auto qf_at = [&](int u, ge& F) {
      scr_load(F.x, sc, QF + 2 * FW * u);
      scr_load(F.y, sc, QF + 2 * FW * u + FW);
    };
    if (!wide && count_q) {  // piece Q: its labels against the mirrored outputs, then its results
      const StreamWr* wq = wrs[wid][pq];
      const int meta_q = META + 2 * MULTI_RMAX * pq;
      const auto q_out = [&](int u, const int64_t*& o, uint32_t& off, uint32_t& len, int64_t*& vrow,
                             uint32_t& vstride) {
        const int j = u / K;
        o = wq[j].mirror;
        off = scr_load_w(sc, meta_q + 2 * j);
        len = scr_load_w(sc, meta_q + 2 * j + 1);  // 0 for padding lanes
        vrow = nullptr;
        vstride = 0;
      };
      fe inv;
      scr_load(inv, sc, PEND_ZI(PB, ninv - 1));
      hits_q |= stream_unit_rows(labels_backward(inv, k, labels, count_q * K, sc, LB, qf_at, q_out), K);
      stream_emit(ctrl, dev, wq, count_q, lane, hits_q);
      count_q = 0;
    }
    if (!wide && count_p) {  // piece P: affine F, base compare; its labels wait one iteration
      const StreamWr* wp = wrs[wid][pp];
      const int meta_p = META + 2 * MULTI_RMAX * pp;
      uint32_t hits = 0;
#pragma unroll 1
      for (int u = 0; u < np; u++) {
        const int j = u / K;
        gej P;
        fe zi;
        pend_load(P, sc, PB, u);
        scr_load(zi, sc, PEND_ZI(PB, u));
        ge F;
        gej_to_ge_zinv(F, P, zi);
        if (with_labels) {
          scr_store(sc, QF + 2 * FW * u, F.x);
          scr_store(sc, QF + 2 * FW * u + FW, F.y);
        }
        const uint32_t off = scr_load_w(sc, meta_p + 2 * j);
        const uint32_t len = scr_load_w(sc, meta_p + 2 * j + 1);  // 0 for padding lanes
        if (outputs_match(k, wp[j].mirror, off, len, F.x, fe_upper64(F.x))) hits |= 1u << j;
      }
      if (with_labels) {
        fe acc;
        labels_forward(acc, k, labels, np, sc, LB, qf_at);
        scr_store(sc, QACC, acc);
        const int t = pq;  // P's wave-rows and offsets become Q's
        pq = pp;
        pp = t;
        if (lane == 0) me.t_q = me.t_p;
        count_q = count_p;
        hits_q = hits;
      } else {
        stream_emit(ctrl, dev, wp, count_p, lane, hits);
      }
    }
    // t of each new row (K output indices), then stage B's F = t G + B into
    // slots u = j K + kk
    if constexpr (wide) {
      // K > MULTI_RMAX: the piece (count rows, rmax 1: one) is finished here,
      // its indices in groups of g <= MULTI_RMAX F points with one inversion
      // each (the S points were inverted above, alone: P and Q stay empty).
      // Its rows' output mirrors were written in this iteration, lane-strided
      // by stream_prefetch (agent-scope write-through stores): wait for those
      // stores and drop this CU's L1 before any lane reads them (the
      // pipelined path reads a mirror one iteration later, after the next
      // iteration's system-scope acquire).
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const StreamWr* wn = wrs[wid][pn];
      const int meta_n = META + 2 * MULTI_RMAX * pn;
      uint32_t hits = 0;
#pragma unroll 1
      for (int j = 0; j < count; j++) {
        uint32_t sx[8];
        {
          gej P;
          fe zi;
          pend_load(P, sc, PB, j);
          scr_load(zi, sc, PEND_ZI(PB, j));
          const uint32_t y_odd = row_shared_secret_affine(sx, P, zi);
#pragma unroll
          for (int q = 0; q < 8; q++) scr_store_w(sc, SXA + q, sx[q]);
          scr_store_w(sc, SXA + 8, y_odd);
        }
        const uint32_t off = scr_load_w(sc, meta_n + 2 * j);
        const uint32_t len = scr_load_w(sc, meta_n + 2 * j + 1);  // 0 for padding lanes
        const auto out = [&](int, const int64_t*& o, uint32_t& of, uint32_t& ln, int64_t*& vrow, uint32_t& vstride) {
          o = wn[j].mirror;
          of = off;
          ln = len;
          vrow = nullptr;
          vstride = 0;
        };
        const auto f_at = [&](int u, ge& F) {
          scr_load(F.x, sc, PEND_X(PB, u));
          scr_load(F.y, sc, PEND_Y(PB, u));
        };
        bool hit = false;
#pragma unroll 1
        for (int kk0 = 0; kk0 < K; kk0 += MULTI_RMAX) {
          const int g = K - kk0 < MULTI_RMAX ? K - kk0 : MULTI_RMAX;
#pragma unroll 1
          for (int u = 0; u < g; u++) {
            uint32_t t[8];
#pragma unroll
            for (int q = 0; q < 8; q++) sx[q] = scr_load_w(sc, SXA + q);
            bip352_shared_secret_hash(t, k.mid, sx, scr_load_w(sc, SXA + 8), (uint32_t)(kk0 + u));
            gej F;
            row_match_point<FBB>(F, t, fb, k);
            pend_store(sc, PB, u, F);
          }
          pend_invert<2 * MULTI_RMAX + 1>(sc, PB, g);
#pragma unroll 1
          for (int u = 0; u < g; u++) {
            gej F;
            fe zi;
            pend_load(F, sc, PB, u);
            scr_load(zi, sc, PEND_ZI(PB, u));
            // F affine over the slot's X / Y (the labels read it there)
            if (row_match_base(F, zi, k, wn[j].mirror, off, len, sc, PB, u, nullptr)) hit = true;
          }
          if (with_labels) {
            // the g x L label sums with one more inversion: their product
            // goes through pend_invert in pending slot g (same instance)
            fe acc, inv;
            labels_forward(acc, k, labels, g, sc, LB, f_at);
            scr_store(sc, PEND_Z(PB, g), acc);
            pend_invert<2 * MULTI_RMAX + 1>(sc, PEND_X(PB, g), 1);
            scr_load(inv, sc, PEND_ZI(PB, g));
            if (labels_backward(inv, k, labels, g, sc, LB, f_at, out)) hit = true;
          }
        }
        if (hit) hits |= 1u << j;
      }
      stream_emit(ctrl, dev, wn, count, lane, hits);
    } else if (K == 1) {
#pragma unroll 1
      for (int j = 0; j < count; j++) {
        gej P;
        fe zi;
        pend_load(P, sc, PB, np + j);
        scr_load(zi, sc, PEND_ZI(PB, np + j));
        uint32_t sx[8], t[8];
        const uint32_t y_odd = row_shared_secret_affine(sx, P, zi);
        bip352_shared_secret_hash(t, k.mid, sx, y_odd);
        gej F;
        row_match_point<FBB>(F, t, fb, k);
        pend_store(sc, PB, j, F);  // slot np + j' (j' < j) is consumed already
      }
    } else {
      // every S first (the F slots of row j overlap later rows' S slots)
#pragma unroll 1
      for (int j = 0; j < count; j++) {
        gej P;
        fe zi;
        pend_load(P, sc, PB, np + j);
        scr_load(zi, sc, PEND_ZI(PB, np + j));
        uint32_t sx[8];
        const uint32_t y_odd = row_shared_secret_affine(sx, P, zi);
#pragma unroll
        for (int q = 0; q < 8; q++) scr_store_w(sc, SXA + 9 * j + q, sx[q]);
        scr_store_w(sc, SXA + 9 * j + 8, y_odd);
      }
#pragma unroll 1
      for (int u = 0; u < count * K; u++) {
        const int j = u / K, kk = u - j * K;
        uint32_t sx[8], t[8];
#pragma unroll
        for (int q = 0; q < 8; q++) sx[q] = scr_load_w(sc, SXA + 9 * j + q);
        const uint32_t y_odd = scr_load_w(sc, SXA + 9 * j + 8);
        bip352_shared_secret_hash(t, k.mid, sx, y_odd, (uint32_t)kk);
        gej F;
        row_match_point<FBB>(F, t, fb, k);
        pend_store(sc, PB, u, F);
      }
    }
    if constexpr (!wide) {  // the new piece becomes P
      const int t = pp;
      pp = pn;
      pn = t;
      count_p = count;
      if (lane == 0 && count) me.t_p = t_it;
    }
    if (lane == 0) {
      me.busy = me.busy + (wall_clock64() - t_it);
      ST_EV(ST_ITER_END, st_wave, 0ull, 0u, 0u);
    }
  }
  if (lane == 0) {
    ST_EV(ST_EXIT, st_wave, 0ull, me.polls, me.rows);
    // this wave's counters, summed over the query's launches (a wave slot
    // runs one wave per launch); the host adds them up (cudasp_stream_counters)
    unsigned long long* o = wstat + (size_t)(slot / 64u) * STREAM_WSTAT;
    const unsigned long long v[STREAM_WSTAT] = {me.pieces, me.rows, me.polls, me.drains, 0ull, 1ull, me.busy,
                                                wall_clock64() - me.t_start};
#pragma unroll
    for (int i = 0; i < (int)STREAM_WSTAT; i++) o[i] += v[i];
  }
}

// The fixed-base table of `windows` windows of `entries` odd multiples each
// (the width's FbWidth), built in runs: a thread takes run_len (FB_RUN, or
// the window's entries if fewer) consecutive odd multiples (2j+1) Q,
// j = j0 .. j0 + run_len - 1, of one
// window's base Q -- the first by double-and-add, each next one by adding
// D = 2Q with a co-Z addition (ZADDU, D kept at the running Z) -- keeps them
// Jacobian in its scratch with the running product of their Z, inverts that
// product once, and walks back writing each entry's normalized affine words
// (Montgomery's batch inversion).  Per entry: one co-Z addition, three
// multiplications and the affine conversion, against ~25 doublings, ~12
// additions and one inversion for an entry computed on its own
// (fb_build_entry; 0.55 s for the 26-bit table that way) -- and the same
// words, since an entry is the unique normalized affine point (k_fb_check).
// The run's first entry (a double-and-add) and its inversion are shared by
// the run's 128 entries (32 before round 6's last change).  Scratch: run_len x
// 4 field elements (X, Y, Z, prefix product) of raw limbs per thread,
// limb-major over the grid's threads (coalesced).
constexpr uint32_t FB_RUN = 128;
constexpr uint32_t fb_run_len(uint32_t entries) { return entries < FB_RUN ? entries : FB_RUN; }
constexpr uint32_t fb_run_words(uint32_t run_len) { return run_len * 4 * FE_LIMBS; }  // scratch words per thread

__device__ __forceinline__ void fb_run_store(uint32_t* __restrict__ scr, uint32_t G, uint32_t elem, const fe& a) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) scr[(size_t)(elem * FE_LIMBS + i) * G] = a.n[i];
}
__device__ __forceinline__ void fb_run_load(fe& a, const uint32_t* __restrict__ scr, uint32_t G, uint32_t elem) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) a.n[i] = scr[(size_t)(elem * FE_LIMBS + i) * G];
}

__global__ __launch_bounds__(BLOCK) void k_fb_build_runs(const uint32_t* __restrict__ bases2, uint32_t windows,
                                                         uint32_t entries, uint32_t run_len,
                                                         uint32_t* __restrict__ table,
                                                         uint32_t* __restrict__ scratch) {
  const uint32_t G = gridDim.x * blockDim.x;
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t* scr = scratch + tid;
  const uint32_t runs_per_window = entries / run_len;
  const uint32_t runs = windows * runs_per_window;
  for (uint32_t run = tid; run < runs; run += G) {
    const uint32_t window = run / runs_per_window;
    const uint32_t j0 = (run % runs_per_window) * run_len;
    ge Q, D;
    ge_from_words(Q, bases2 + (size_t)window * 32);
    ge_from_words(D, bases2 + (size_t)window * 32 + 16);
    // (2 j0 + 1) Q, double-and-add from the top bit (as fb_build_entry)
    const uint32_t m = 2 * j0 + 1;
    const int top = 31 - __builtin_clz(m);
    gej P;
    gej_set_ge(P, Q);
    for (int b = top - 1; b >= 0; b--) {
      gej_double(P, P);
      if ((m >> b) & 1u) gej_add_ge(P, P, Q);
    }
    // D = 2Q at P's Z, then each next entry by co-Z addition (ZADDU, 5M + 2S
    // instead of a mixed addition's 8M + 3S), which moves D to the new Z
    gej Dz;
    {
      fe z2, z3;
      fe_sqr(z2, P.z);
      fe_mul(z3, z2, P.z);
      fe_mul(Dz.x, D.x, z2);
      fe_mul(Dz.y, D.y, z3);
      Dz.z = P.z;
    }
    fe acc;
    for (uint32_t k = 0; k < run_len; k++) {
      if (k) {  // (2 (j0 + k) + 1) Q; never +-D or infinity for j < 2^26
        gej nxt;
        gej_zaddu(nxt, Dz, P);
        P = nxt;
      }
      fb_run_store(scr, G, 4 * k + 0, P.x);
      fb_run_store(scr, G, 4 * k + 1, P.y);
      fb_run_store(scr, G, 4 * k + 2, P.z);
      if (k)
        fe_mul(acc, acc, P.z);
      else
        acc = P.z;
      fb_run_store(scr, G, 4 * k + 3, acc);
    }
    fe inv;
    fe_inv(inv, acc);  // 1 / (Z_0 ... Z_{R-1})
    for (int k = (int)run_len - 1; k >= 0; k--) {
      gej Pk;
      fb_run_load(Pk.x, scr, G, 4 * k + 0);
      fb_run_load(Pk.y, scr, G, 4 * k + 1);
      fb_run_load(Pk.z, scr, G, 4 * k + 2);
      fe zi;
      if (k) {
        fe prev;
        fb_run_load(prev, scr, G, 4 * (k - 1) + 3);
        fe_mul(zi, inv, prev);    // 1 / Z_k
        fe_mul(inv, inv, Pk.z);   // 1 / (Z_0 ... Z_{k-1})
      } else {
        zi = inv;
      }
      ge A;
      gej_to_ge_zinv(A, Pk, zi);
      uint32_t out[16];
      fe_to_u32x8(out, A.x);
      fe_to_u32x8(out + 8, A.y);
      uint4* dst = reinterpret_cast<uint4*>(table + ((size_t)window * entries + j0 + (uint32_t)k) * FB_WORDS);
#pragma unroll
      for (int q = 0; q < 4; q++) dst[q] = make_uint4(out[4 * q], out[4 * q + 1], out[4 * q + 2], out[4 * q + 3]);
    }
  }
}

// Test support: entries idx = 0, stride, 2 stride, ... of a built table
// recomputed one by one (fb_build_entry) and compared;
// *bad counts the entries that differ.
__global__ __launch_bounds__(BLOCK) void k_fb_check(const uint32_t* __restrict__ bases, uint32_t windows,
                                                    uint32_t entries, const uint32_t* __restrict__ table,
                                                    uint32_t stride, uint32_t* __restrict__ bad) {
  const uint64_t total = (uint64_t)windows * entries;
  const uint64_t n = (total + stride - 1) / stride;
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t idx = t * stride;
    ge Q;
    ge_from_words(Q, bases + (idx / entries) * 16);
    uint32_t out[16];
    fb_build_entry(out, Q, (uint32_t)(idx % entries));
    const uint32_t* e = table + idx * FB_WORDS;
    bool same = true;
#pragma unroll
    for (int q = 0; q < 16; q++) same &= out[q] == e[q];
    if (!same) atomicAdd(bad, 1u);
  }
}

// The fixed-base table's top window with the spend key B folded in
// (ScanConsts::fb_top): entry j of window W - 1 plus B, then minus B.  A
// thread takes FOLD_RUN consecutive entries and one inversion for all of
// them (Montgomery's trick over the denominators x(B) - x(P_j), which the two
// sums of an entry share): the prefix products wait in the entries' own +B
// output words until the walk back overwrites them (0.96 -> ~0.2 ms for the
// 2^21 entries of 26-bit windows against one inversion per entry).  *bad is
// set if any sum is exceptional (x equal), and the scanner then keeps adding
// B on its own.
struct SpendWords {
  uint32_t w[16];
};
constexpr uint32_t FOLD_RUN = 16;

__device__ __forceinline__ bool fold_den(fe& den, const ge& P, const ge& B) {
  fe_sub<1>(den, B.x, P.x);
  fe_normalize(den);
  if (!fe_is_zero_norm(den)) return true;
  fe_set_int(den, 1);  // exceptional: the table is discarded, the run stays finite
  return false;
}

template <int BITS>
__global__ __launch_bounds__(BLOCK) void k_fb_fold(const uint32_t* __restrict__ fb, SpendWords spend,
                                                   uint32_t* __restrict__ out, uint32_t* __restrict__ bad) {
  constexpr uint32_t TOP = FbWidth<BITS>::TOP_ENTRIES;
  constexpr uint32_t RUN = FOLD_RUN < TOP ? FOLD_RUN : TOP;
  static_assert(TOP % RUN == 0, "runs tile the top window");
  const uint32_t j0 = (blockIdx.x * blockDim.x + threadIdx.x) * RUN;
  if (j0 >= TOP) return;
  const uint32_t* top = fb + (size_t)(FbWidth<BITS>::WINDOWS - 1) * FbWidth<BITS>::ENTRIES * FB_WORDS;
  ge B, nB;
  ge_from_words(B, spend.w);
  nB.x = B.x;
  fe_negate<1>(nB.y, B.y);
  fe_normalize(nB.y);
  fe acc;
  fe_set_int(acc, 1);
  bool ok = true;
  for (uint32_t k = 0; k < RUN; k++) {
    ge P;
    ge_from_words(P, top + (size_t)(j0 + k) * FB_WORDS);
    fe den;
    ok = fold_den(den, P, B) && ok;
    uint32_t* pre = out + (size_t)(j0 + k) * FB_WORDS;
#pragma unroll
    for (int l = 0; l < FE_LIMBS; l++) pre[l] = acc.n[l];
    fe_mul(acc, acc, den);
  }
  if (!ok) atomicOr(bad, 1u);
  fe inv;
  fe_inv(inv, acc);  // 1 / (den_0 ... den_(RUN-1))
  for (int k = (int)RUN - 1; k >= 0; k--) {
    const uint32_t j = j0 + (uint32_t)k;
    ge P;
    ge_from_words(P, top + (size_t)j * FB_WORDS);
    fe den, pre, di;
    (void)fold_den(den, P, B);
    const uint32_t* pw = out + (size_t)j * FB_WORDS;
#pragma unroll
    for (int l = 0; l < FE_LIMBS; l++) pre.n[l] = pw[l];
    fe_mul(di, inv, pre);   // 1 / den_j
    fe_mul(inv, inv, den);  // 1 / (den_0 ... den_(j-1))
    uint32_t a[16], b[16];
    affine_add_inv(a, P, B, di);
    affine_add_inv(b, P, nB, di);
    uint4* pa = reinterpret_cast<uint4*>(out + (size_t)j * FB_WORDS);
    uint4* pb = reinterpret_cast<uint4*>(out + ((size_t)TOP + j) * FB_WORDS);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      pa[q] = make_uint4(a[4 * q], a[4 * q + 1], a[4 * q + 2], a[4 * q + 3]);
      pb[q] = make_uint4(b[4 * q], b[4 * q + 1], b[4 * q + 2], b[4 * q + 3]);
    }
  }
}

// Test support: entries j = 0, stride, 2 stride, ... of a fold table
// recomputed one by one (fb_fold_entry: one inversion per entry) and compared.
template <int BITS>
__global__ __launch_bounds__(BLOCK) void k_fold_check(const uint32_t* __restrict__ fb, SpendWords spend,
                                                      const uint32_t* __restrict__ fold, uint32_t stride,
                                                      uint32_t* __restrict__ bad) {
  constexpr uint32_t TOP = FbWidth<BITS>::TOP_ENTRIES;
  ge B;
  ge_from_words(B, spend.w);
  for (uint64_t j = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * stride; j < TOP;
       j += (uint64_t)gridDim.x * blockDim.x * stride) {
    ge P;
    ge_from_words(P, fb + ((size_t)(FbWidth<BITS>::WINDOWS - 1) * FbWidth<BITS>::ENTRIES + j) * FB_WORDS);
    uint32_t a[16], b[16];
    bool same = fb_fold_entry(a, b, P, B);
    for (int q = 0; q < 16 && same; q++)
      same = a[q] == fold[j * FB_WORDS + q] && b[q] == fold[((size_t)TOP + j) * FB_WORDS + q];
    if (!same) atomicAdd(bad, 1u);
  }
}

__global__ __launch_bounds__(BLOCK) void k_rows_to_cols(const uint8_t* __restrict__ rows, uint32_t n,
                                                        uint32_t* __restrict__ x, uint32_t* __restrict__ y) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t row = blockIdx.x * blockDim.x + threadIdx.x; row < n; row += stride) {
    const uint4* src = reinterpret_cast<const uint4*>(rows + (size_t)row * 64);
    uint32_t w[16];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      uint4 v = src[q];
      w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
      x[(size_t)j * n + row] = w[j];
      y[(size_t)j * n + row] = w[8 + j];
    }
  }
}

// Layout probe (measurement only; never part of a scan): moves exactly the
// algorithmic bytes of a row (tweak x and y columns 64 B,
// offset + length 8 B, outputs 8k B, flag 1 B) with stage A's thread-to-row
// mapping (ROWS_A rows per thread: g, g + G, ...), so its time and HBM
// counters show what the column-major layout costs when the arithmetic is
// free.  The flag is a function of every byte read (nothing is dead code).
__global__ __launch_bounds__(BLOCK) void k_layout_probe(const uint32_t* __restrict__ tx,
                                                        const uint32_t* __restrict__ ty, uint32_t n,
                                                        const int64_t* __restrict__ outputs,
                                                        const uint32_t* __restrict__ offs,
                                                        const uint32_t* __restrict__ lens,
                                                        uint8_t* __restrict__ flags) {
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t G = (n + ROWS_A - 1) / ROWS_A;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < G; g += stride) {
#pragma unroll
    for (int j = 0; j < ROWS_A; j++) {
      const uint32_t row = g + (uint32_t)j * G;
      if (row >= n) break;
      uint32_t h = 0;
#pragma unroll
      for (int w = 0; w < 8; w++) h = (h ^ tx[(size_t)w * n + row]) + ty[(size_t)w * n + row];
      const uint32_t off = offs[row], len = lens[row];
      bool hit = false;
      for (uint32_t k = 0; k < len; k++) hit |= (uint32_t)outputs[(size_t)off + k] == h;
      flags[row] = hit ? 1 : 0;
    }
  }
}

// ------------------------------------------------------ synthetic tables
// Deterministic benchmark/test inputs: tweak T_i = (s0 + i) G
// and splitmix64 outputs.  Generation only; never part of a scan.
struct SynthConsts {
  uint32_t s0[8];  // < n
};

__device__ __forceinline__ void add_index_mod_n(uint32_t s[8], const uint32_t s0[8], uint64_t idx) {
  const uint32_t nn[8] = {0xD0364141u, 0xBFD25E8Cu, 0xAF48A03Bu, 0xBAAEDCE6u,
                          0xFFFFFFFEu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t add = i == 0 ? (idx & 0xFFFFFFFFu) : (i == 1 ? (idx >> 32) : 0);
    c += (uint64_t)s0[i] + add;
    s[i] = (uint32_t)c;
    c >>= 32;
  }
  // s >= n ?  (s < 2^256 + n, so compare including the carry word)
  bool ge = c != 0;
  if (!ge) {
    ge = true;
    for (int i = 7; i >= 0; i--) {
      if (s[i] != nn[i]) {
        ge = s[i] > nn[i];
        break;
      }
    }
  }
  if (ge) {
    int64_t b = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      b += (int64_t)s[i] - nn[i];
      s[i] = (uint32_t)b;
      b >>= 32;
    }
  }
}

template <int FBB>
__global__ __launch_bounds__(BLOCK) void k_synth_tweaks(SynthConsts c, uint64_t first, uint32_t n,
                                                        const uint32_t* __restrict__ fb, uint32_t* __restrict__ x,
                                                        uint32_t* __restrict__ y) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t row = blockIdx.x * blockDim.x + threadIdx.x; row < n; row += stride) {
    uint32_t s[8];
    add_index_mod_n(s, c.s0, first + row);
    gej R;
    fixed_base_mul<FBB>(R, s, fb);
    fe zi;
    fe_inv(zi, R.z);
    ge A;
    gej_to_ge_zinv(A, R, zi);
    uint32_t wx[8], wy[8];
    fe_to_u32x8(wx, A.x);
    fe_to_u32x8(wy, A.y);
#pragma unroll
    for (int j = 0; j < 8; j++) {
      x[(size_t)j * n + row] = wx[j];
      y[(size_t)j * n + row] = wy[j];
    }
  }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(BLOCK) void k_synth_outputs(uint64_t seed, uint64_t first, uint32_t n, uint32_t k,
                                                         int64_t* __restrict__ outs, uint32_t* __restrict__ offs,
                                                         uint32_t* __restrict__ lens) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t row = blockIdx.x * blockDim.x + threadIdx.x; row < n; row += stride) {
    uint64_t g = first + row;
    offs[row] = row * k;
    lens[row] = k;
    for (uint32_t j = 0; j < k; j++) outs[(size_t)row * k + j] = (int64_t)splitmix64(seed ^ (g * k + j));
  }
}

// Variable-length outputs lists: pass 1 writes lengths uniform in [1, kmax]
// (mean (kmax+1)/2), the caller scans them into offsets, pass 2 fills values.
__global__ __launch_bounds__(BLOCK) void k_synth_output_lengths(uint64_t seed, uint64_t first, uint32_t n,
                                                                uint32_t kmax, uint32_t* __restrict__ lens) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t row = blockIdx.x * blockDim.x + threadIdx.x; row < n; row += stride)
    lens[row] = 1u + (uint32_t)(splitmix64(~seed ^ (first + row)) % kmax);
}

__global__ __launch_bounds__(BLOCK) void k_synth_output_values(uint64_t seed, uint64_t first, uint32_t n,
                                                               const uint32_t* __restrict__ offs,
                                                               const uint32_t* __restrict__ lens,
                                                               int64_t* __restrict__ outs) {
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t row = blockIdx.x * blockDim.x + threadIdx.x; row < n; row += stride) {
    uint64_t g = first + row;
    for (uint32_t j = 0; j < lens[row]; j++)
      outs[(size_t)offs[row] + j] = (int64_t)splitmix64(seed ^ ((g << 4) + j));
  }
}

__global__ __launch_bounds__(BLOCK) void k_debug_field_ops(int op, const uint32_t* __restrict__ a,
                                                           const uint32_t* __restrict__ b,
                                                           uint32_t* __restrict__ out, uint32_t n) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe x, y, r;
#pragma unroll
  for (int k = 0; k < FE_LIMBS; k++) {
    x.n[k] = a[(size_t)i * FE_LIMBS + k];
    y.n[k] = b[(size_t)i * FE_LIMBS + k];
  }
  if (op == 0) {
    fe_mul(r, x, y);
  } else if (op == 1) {
    fe_sqr(r, x);
  } else if (op == 7) {
    fe_inv(r, x);
  } else {
#if CUDASP_FE_LIMBS == 9
    fe c, e;
#pragma unroll
    for (int k = 0; k < FE_LIMBS; k++) {
      c.n[k] = b[((size_t)n + i) * FE_LIMBS + k];
      e.n[k] = b[((size_t)2 * n + i) * FE_LIMBS + k];
    }
    if (op == 2)
      fe_mul2(r, x, y, c, e);
    else if (op == 3)
      fe_mulsqr(r, x, y, c);
    else if (op == 4)
      fe_mul_add(r, x, y, c);
    else if (op == 5)
      fe_sqr_add(r, x, c);
    else
      fe_sqr3(r, x);
#endif
  }
#pragma unroll
  for (int k = 0; k < FE_LIMBS; k++) out[(size_t)i * FE_LIMBS + k] = r.n[k];
}

// ------------------------------------------------------------- host helpers
namespace {

// ------------------------------------------------ per-device fixed-base table
// One table per (device, window width), built on first use and kept for the
// process.  Each table has its own once-guard, so the first scanners of
// several devices (one DuckDB executor thread per GPU) build their tables in
// parallel; the map itself is only locked for the lookup.
struct DeviceTable {
  std::mutex mu;  // held while building
  uint32_t* table = nullptr;
};
std::mutex g_table_map_mutex;
std::map<std::pair<int, int>, DeviceTable> g_tables;

// Prebuilt widths (k_match / k_synth_tweaks instances): 22 and 26 (HBM), 7
// (LDS-staged, stage B only).
bool fb_bits_supported(int bits) { return bits == 22 || bits == 26 || bits == LDS_FB_BITS; }

// Devices with at least this much memory take the 26-bit table by default
// (21.5 GB: 7.5% of an MI355X's 288 GB); smaller ones the 22-bit table.
constexpr uint64_t FB26_MIN_DEVICE_BYTES = 128ull << 30;

// The default width of a device (-1: the current one): CUDASP_FB_BITS (22 or
// 26) from the environment; else 26 bits when that device has >= 128 GiB
// (every MI355X), else the build's FB_BITS.  Decided once per device, so a
// host with GPUs of different sizes gives each its own.
int default_fb_bits(int device = -1) {
  static const int env_bits = [] {
    const char* e = getenv("CUDASP_FB_BITS");
    const int b = e ? atoi(e) : 0;
    return b == 22 || b == 26 ? b : 0;
  }();
  if (env_bits) return env_bits;
  if (device < 0 && hipGetDevice(&device) != hipSuccess) return FB_BITS;
  static std::mutex mu;
  static std::map<int, int> bits_of;
  std::lock_guard<std::mutex> lk(mu);
  auto it = bits_of.find(device);
  if (it != bits_of.end()) return it->second;
  size_t total = 0;
  const int b = hipDeviceTotalMem(&total, device) == hipSuccess && (uint64_t)total >= FB26_MIN_DEVICE_BYTES ? 26 : FB_BITS;
  bits_of[device] = b;
  return b;
}

size_t fb_table_bytes(int bits) {
  const size_t windows = (256 + bits - 1) / bits;
  return windows * ((size_t)1 << (bits - 1)) * FB_WORDS * 4;
}

// The library's one-off builds (the fixed-base tables, the spend-key folds)
// run on the stream of the scanner that needs them, or on a temporary stream
// when there is none (cudasp_fixed_base_prepare, the synthetic tables).  Not
// on a stream kept for the purpose: every stream a process keeps takes one of
// the GPU_MAX_HW_QUEUES hardware queues, and the host's per-slot launch feeds
// size their streams to the queues left (a kept build stream made two of
// their three streams share a queue: 167 -> 107 M tx/s end to end).  A
// temporary stream costs ~3 ms to create and ~1.5 ms to destroy, which a new
// key's fold paid inside the query before it took the scanner's stream.
struct BuildStream {
  hipStream_t st = nullptr;
  bool owned = false;
  explicit BuildStream(hipStream_t given) : st(given) {
    if (!st) {
      if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        st = nullptr;
      } else {
        owned = true;
      }
    }
  }
  ~BuildStream() {
    if (owned) (void)hipStreamDestroy(st);
  }
};

int ensure_device_table(int device, int bits, const uint32_t** out, bool* built = nullptr,
                        hipStream_t stream = nullptr) {
  if (!fb_bits_supported(bits))
    return set_error(CUDASP_ERR_INVALID_ARG, "fixed-base window width %d not supported (22, 26, or 7 = LDS)", bits);
  DeviceTable* dt;
  {
    std::lock_guard<std::mutex> lock(g_table_map_mutex);
    dt = &g_tables[std::make_pair(device, bits)];  // std::map: stable address
  }
  std::lock_guard<std::mutex> lock(dt->mu);
  if (dt->table) {
    *out = dt->table;
    return CUDASP_OK;
  }
  const uint32_t windows = (256 + bits - 1) / bits, entries = 1u << (bits - 1);
  const std::vector<uint32_t> bases2 = fb_window_bases_doubled(bits);
  const size_t table_bytes = fb_table_bytes(bits);
  uint32_t* d_table = nullptr;
  if (hipMalloc(&d_table, table_bytes) != hipSuccess) {
    (void)hipGetLastError();
    return set_error(CUDASP_ERR_HIP,
                     "device %d: cannot allocate the %.1f GB fixed-base table (%d-bit windows); free device memory "
                     "or choose 22-bit windows (1.5 GiB; CUDASP_FB_BITS=22)",
                     device, table_bytes / 1e9, bits);
  }
  // k_fb_build_runs: run_len entries per thread in runs, a grid of 2 blocks
  // per CU (its scratch, fb_run_words(run_len) per thread, is freed after the build)
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
  const uint32_t run_len = fb_run_len(entries);
  const uint32_t runs = windows * (entries / run_len);
  uint32_t blocks = (uint32_t)cus * 2;
  if ((uint64_t)blocks * BLOCK > runs) blocks = (runs + BLOCK - 1) / BLOCK;
  uint32_t* d_bases = nullptr;
  uint32_t* d_scratch = nullptr;
  hipStream_t st = nullptr;
  auto cleanup = [&](bool keep_table) {
    if (d_bases) (void)hipFree(d_bases);
    if (d_scratch) (void)hipFree(d_scratch);
    if (!keep_table) (void)hipFree(d_table);
  };
  // The build runs on the caller's (or a temporary) stream, so other threads'
  // work on the device is not serialized behind it (no device-wide synchronize).
  BuildStream bst(stream);
  if (hipMalloc(&d_bases, bases2.size() * 4) != hipSuccess ||
      hipMalloc(&d_scratch, (size_t)fb_run_words(run_len) * blocks * BLOCK * 4) != hipSuccess ||
      (st = bst.st) == nullptr ||
      hipMemcpyAsync(d_bases, bases2.data(), bases2.size() * 4, hipMemcpyHostToDevice, st) != hipSuccess) {
    (void)hipGetLastError();
    cleanup(false);
    return set_error(CUDASP_ERR_HIP, "device %d: fixed-base table build: allocation failed", device);
  }
  hipLaunchKernelGGL(k_fb_build_runs, dim3(blocks), dim3(BLOCK), 0, st, d_bases, windows, entries, run_len, d_table,
                     d_scratch);
  const hipError_t e1 = hipGetLastError();
  const hipError_t e2 = e1 == hipSuccess ? hipStreamSynchronize(st) : e1;
  if (e2 != hipSuccess) {
    cleanup(false);
    return set_error(CUDASP_ERR_HIP, "device %d: fixed-base table build failed: %s", device, hipGetErrorString(e2));
  }
  cleanup(true);
  if (built) *built = true;
  dt->table = d_table;
  *out = d_table;
  return CUDASP_OK;
}

// The calling thread's current device switched for a scope.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// --- spend key folded into the top window (ScanConsts::fb_top) -------------
// One table per (device, width, spend key), shared by every scanner with that
// key (a query's feeds, a wallet's pooled scanners) and refcounted: 2 x 2^21
// entries (268 MB) at 26 bits, 2 x 2^13 (1 MB) at 22.  A few unreferenced
// tables stay cached per device for the next query; beyond that the oldest is
// freed.  CUDASP_FB_FOLD=0 turns the fold off (A/B; the separate addition).
struct FoldKey {
  int device, bits;
  uint32_t spend[16];
  bool operator<(const FoldKey& o) const {
    if (device != o.device) return device < o.device;
    if (bits != o.bits) return bits < o.bits;
    return memcmp(spend, o.spend, sizeof(spend)) < 0;
  }
};
struct FoldTable {
  uint32_t* table = nullptr;  // nullptr: exceptional (or failed) -- no fold for this key
  int refs = 0;
  uint64_t last_release = 0;
  bool building = false;  // fold_acquire is building it (outside g_fold_mu)
};
std::mutex g_fold_mu;
std::condition_variable g_fold_cv;
std::map<FoldKey, FoldTable> g_folds;
uint64_t g_fold_clock = 0;
constexpr int FOLD_CACHED_PER_DEVICE = 4;

bool fold_enabled() {
  static const bool on = [] {
    const char* e = getenv("CUDASP_FB_FOLD");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

size_t fold_table_bytes(int bits) {
  const size_t top = bits == 26 ? FbWidth<26>::TOP_ENTRIES : FbWidth<22>::TOP_ENTRIES;
  return 2 * top * FB_WORDS * 4;
}

// Caller holds g_fold_mu: free unreferenced tables of `device` beyond the cap,
// oldest first.
void fold_trim_locked(int device) {
  for (;;) {
    int unref = 0;
    auto oldest = g_folds.end();
    for (auto it = g_folds.begin(); it != g_folds.end(); ++it)
      if (it->first.device == device && it->second.refs == 0) {
        unref++;
        if (oldest == g_folds.end() || it->second.last_release < oldest->second.last_release) oldest = it;
      }
    if (unref <= FOLD_CACHED_PER_DEVICE) return;
    if (oldest->second.table) {
      DeviceGuard g(device);
      (void)hipFree(oldest->second.table);
    }
    g_folds.erase(oldest);
  }
}

// The fold table of `key` built on `stream` (or a temporary one): the table, or nullptr
// when the key cannot be folded (exceptional sums) or anything failed (the
// scanner then adds B on its own; every partial allocation is freed).
uint32_t* fold_build(const FoldKey& key, const uint32_t* d_fb, hipStream_t stream) {
  DeviceGuard g(key.device);
  BuildStream bst(stream);
  uint32_t* d = nullptr;
  uint32_t* d_bad = nullptr;
  hipStream_t st = nullptr;
  uint32_t bad = 1;
  bool ok = hipMalloc(&d, fold_table_bytes(key.bits)) == hipSuccess && hipMalloc(&d_bad, 4) == hipSuccess &&
            (st = bst.st) != nullptr && hipMemsetAsync(d_bad, 0, 4, st) == hipSuccess;
  if (ok) {
    SpendWords sw;
    memcpy(sw.w, key.spend, sizeof(sw.w));
    const uint32_t top = key.bits == 26 ? FbWidth<26>::TOP_ENTRIES : FbWidth<22>::TOP_ENTRIES;
    auto kf = key.bits == 26 ? k_fb_fold<26> : k_fb_fold<22>;
    const uint32_t threads = (top + FOLD_RUN - 1) / FOLD_RUN;
    hipLaunchKernelGGL(kf, dim3((threads + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, st, d_fb, sw, d, d_bad);
    ok = hipGetLastError() == hipSuccess && hipMemcpyAsync(&bad, d_bad, 4, hipMemcpyDeviceToHost, st) == hipSuccess &&
         hipStreamSynchronize(st) == hipSuccess;
  }
  (void)hipGetLastError();
  if (d_bad) (void)hipFree(d_bad);
  if (!ok || bad) {
    if (d) (void)hipFree(d);
    d = nullptr;
  }
  return d;
}

// A reference to the fold table of (device, bits, spend), built on first use.
// The build runs outside g_fold_mu (an entry marked `building` holds its
// place; other scanners of the same key wait for it, other keys and devices
// go ahead).  *table = nullptr when the key cannot be folded.
int fold_acquire(const FoldKey& key, const uint32_t* d_fb, const uint32_t** table, hipStream_t stream) {
  std::unique_lock<std::mutex> lk(g_fold_mu);
  auto it = g_folds.find(key);
  if (it != g_folds.end()) {
    it->second.refs++;  // a referenced entry is never trimmed: `it` stays valid
    g_fold_cv.wait(lk, [&] { return !it->second.building; });
    *table = it->second.table;
    return CUDASP_OK;
  }
  it = g_folds.emplace(key, FoldTable()).first;
  it->second.refs = 1;
  it->second.building = true;
  lk.unlock();
  uint32_t* d = fold_build(key, d_fb, stream);
  lk.lock();
  it->second.table = d;
  it->second.building = false;
  g_fold_cv.notify_all();
  *table = d;
  return CUDASP_OK;
}

void fold_release(const FoldKey& key) {
  std::lock_guard<std::mutex> lk(g_fold_mu);
  auto it = g_folds.find(key);
  if (it == g_folds.end()) return;
  if (--it->second.refs == 0) {
    it->second.last_release = ++g_fold_clock;
    fold_trim_locked(key.device);
  }
}

}  // namespace

// ------------------------------------------------------------------ scanner
struct cudasp_scanner {
  int device = 0;
  hipStream_t stream = nullptr;
  ScanConsts consts{};
  const uint32_t* d_fb = nullptr;
  int fb_bits = 0;  // window width of d_fb (22 or 26)
  int8_t* d_naf = nullptr;
  uint32_t* d_labels = nullptr;
  uint32_t label_count = 0;  // label keys in d_labels (x2 with label_negation)
  uint32_t label_cap = 0;  // label keys the label buffers are sized for
  uint32_t capacity = 0;
  cudasp_scan_options opt{1, 0, 0};
  bool fold_allowed = true;        // cudasp_scanner_set_spend_fold (and CUDASP_FB_FOLD)
  bool fold_held = false;          // holds a reference to g_folds[fold_key]
  FoldKey fold_key{};
  const uint32_t* fold_table = nullptr;  // its table (nullptr: not foldable)
  uint32_t t_cap_k = 1;            // output indices d_t / d_vflags are sized for
  std::vector<uint8_t> keys;       // scan key || spend key || label keys (set_options re-prepares)
  bool prepared = false;           // consts / d_naf / d_labels hold `keys` under prepared_opt (set_keys)
  cudasp_scan_options prepared_opt{1, 0, 0};
  uint32_t raw_label_count = 0;
  // Stage-kernel buffers (k_shared_secret / k_match: the stage entry points,
  // the values path, the protocol variants, the LDS width).  Allocated on
  // first use (ensure_stage_buffers): a scanner that only runs the fused
  // k_scan_multi path -- every default-option batch -- never holds them.
  uint32_t* d_t = nullptr;         // 8 x (t_cap_k capacity)
  uint8_t* d_vflags = nullptr;     // t_cap_k x capacity (K > 1: per output index)
  uint32_t* d_vscratch = nullptr;  // VSCRATCH_WORDS x slots_a
  uint32_t* d_lscratch = nullptr;  // lscratch_words(label_cap) x slots_b
  uint32_t slots_a = 0, slots_b = 0;
  uint32_t fill_threads = 0;    // stage-A threads per launch that fill the device (rows_a_for)
  uint32_t fill_threads_b = 0;  // the same for stage B (rows_b_for)
  int rows_a_force = 0;         // CUDASP_ROWS_A_FORCE (tests): fixed rows per stage-A thread
  int rows_b_force = 0;         // CUDASP_ROWS_B_FORCE (tests): fixed rows per stage-B thread
  // host-path staging
  uint8_t* d_rows = nullptr;   // capacity x 64
  uint32_t* d_tx = nullptr;    // 8 x capacity
  uint32_t* d_ty = nullptr;
  uint8_t* d_flags = nullptr;  // capacity
  uint32_t* d_offs = nullptr;
  uint32_t* d_lens = nullptr;
  int64_t* d_outputs = nullptr;
  size_t outputs_cap = 0;
  // multi-batch persistent path (cudasp_scan_device_batches)
  MultiBatch* d_multi = nullptr;   // batch descriptors on the device
  // pinned staging of the descriptors: a ring of MULTI_STAGING areas of
  // multi_cap descriptors each, so queued launches do not make the host wait
  // for an earlier upload before it can stage the next one
  MultiBatch* h_multi = nullptr;
  uint32_t multi_cap = 0;                       // descriptors per area (and in d_multi)
  hipEvent_t multi_copied[8] = {};              // area i's upload has been read
  bool multi_pending[8] = {};
  uint32_t multi_next = 0;
  uint32_t* d_counter = nullptr;   // the persistent kernel's work counter
  uint32_t* d_mscratch = nullptr;  // mscratch_words u32
  uint64_t mscratch_words = 0;
  int cus = 0;
  // cudasp_scan_device / cudasp_scan_host through one k_scan_multi launch
  // (both stages fused, t kept in the thread) instead of the two stage kernels;
  // CUDASP_FUSED_SINGLE=0 selects the two kernels (A/B; the stage entry points,
  // the values path, forced launch shapes and the variants always use them)
  bool fused_single = true;
  // k_scan_multi with the pipelined schedule (one Z inversion per piece);
  // CUDASP_MULTI_PIPE=0 selects the two-inversion schedule (A/B)
  bool multi_pipe = true;
  // k_scan_multi pieces sized by each wave's share of the work done
  // (multi_piece_rows_adaptive); CUDASP_MULTI_ADAPT=0 selects the plain rule
  bool multi_adaptive = true;
  // k_scan_multi's drain: youngest waves first once the counter has run out
  // (MultiTick); CUDASP_MULTI_ENDGAME=0 turns it off (A/B)
  bool multi_endgame = true;
  // k_scan_multi: the SIMDs' youngest waves take no piece they would finish
  // last (multi_piece_rows_adaptive); CUDASP_MULTI_YOUNG=0 turns it off (A/B)
  bool multi_young = true;
};

namespace {

uint32_t grid_for(uint32_t n) {
  uint32_t blocks = (n + BLOCK - 1) / BLOCK;
  if (blocks > MAX_BLOCKS) blocks = MAX_BLOCKS;
  if (blocks == 0) blocks = 1;
  return blocks;
}

// Blocks for a batch of n rows in stage A / B (one thread per group of
// ROWS_A / ROWS_B rows), within the scratch slots the scanner allocated.
uint32_t grid_a(const cudasp_scanner* s, uint32_t n, int rows = ROWS_A) {
  uint32_t b = grid_for((n + rows - 1) / rows);
  // the scratch holds slots_a slots of VSCRATCH_WORDS; fewer rows per thread
  // take fewer words per slot
  const uint64_t cap = (uint64_t)s->slots_a * VSCRATCH_WORDS / ((uint64_t)vscratch_words(rows) * BLOCK);
  return b > cap ? (uint32_t)(cap ? cap : 1) : b;
}

// Rows per stage-A thread for a launch of n rows.  ROWS_A rows share one
// inversion, but a thread scans them in sequence, so a launch lasts at least
// ROWS_A row-times however few rows it has.  The HIP runtime runs a process's
// launches on 4 hardware queues (GPU_MAX_HW_QUEUES), so a launch with fewer
// threads than a quarter of the device's wave slots leaves the GPU part idle:
// such launches take 2 or 1 rows per thread instead.
int rows_a_for(const cudasp_scanner* s, uint32_t n) {
  if (s->rows_a_force) return s->rows_a_force;
  int r = ROWS_A;
  while (r > 1 && (n + r - 1) / (uint32_t)r < s->fill_threads) r = r > 2 ? 2 : 1;
  return r;
}

void launch_a(const cudasp_scanner* s, const uint32_t* tx, const uint32_t* ty, uint32_t n, uint32_t* t,
              hipStream_t st) {
  const int r = rows_a_for(s, n);
  const dim3 grid(grid_a(s, n, r)), block(BLOCK);
  if (r == 1)
    hipLaunchKernelGGL(k_shared_secret<1>, grid, block, 0, st, tx, ty, n, s->d_naf, s->consts, s->d_vscratch, t);
  else if (r == 2)
    hipLaunchKernelGGL(k_shared_secret<2>, grid, block, 0, st, tx, ty, n, s->d_naf, s->consts, s->d_vscratch, t);
  else
    hipLaunchKernelGGL(k_shared_secret<ROWS_A>, grid, block, 0, st, tx, ty, n, s->d_naf, s->consts,
                       s->d_vscratch, t);
}
uint32_t grid_b(const cudasp_scanner* s, uint32_t n, int rows = ROWS_B) {
  uint32_t b = grid_for((n + rows - 1) / rows);
  // the label scratch holds slots_b slots sized for label_cap labels
  const uint64_t cap = (uint64_t)s->slots_b * lscratch_words(s->label_cap) /
                       ((uint64_t)lscratch_words(s->label_count, rows) * BLOCK);
  return b > cap ? (uint32_t)(cap ? cap : 1) : b;
}

// Rows per stage-B thread: ROWS_B, or 2 for launches with fewer threads than
// a quarter of the device's wave slots (as rows_a_for).
int rows_b_for(const cudasp_scanner* s, uint32_t n) {
  if (s->rows_b_force) return s->rows_b_force;
  return (n + ROWS_B - 1) / ROWS_B >= s->fill_threads_b ? ROWS_B : 2;
}

// Stream arguments (include/cudasp_abi.h): NULL = the scanner's own stream
// (the stateless entry points: the null stream), CUDASP_STREAM_DEFAULT = the
// device's null stream -- torch's default stream, whose handle is 0 and so
// cannot be passed as itself.
hipStream_t plain_stream(void* stream) {
  return stream == CUDASP_STREAM_DEFAULT ? nullptr : (hipStream_t)stream;
}
hipStream_t scanner_stream(const cudasp_scanner* s, void* stream) {
  return stream == nullptr ? s->stream : plain_stream(stream);
}

// The scanner's fold of its spend key into the top window (ScanConsts::fb_top)
// after its keys or fixed-base width changed: an on-curve key at an HBM width
// takes (or shares) a fold table; anything else adds B on its own.  Caller:
// no work of the scanner in flight.
int scanner_update_fold(cudasp_scanner* s) {
  FoldKey key{};
  const bool want = s->fold_allowed && fold_enabled() && (s->fb_bits == 22 || s->fb_bits == 26) &&
                    s->d_fb != nullptr && on_curve_words(s->consts.spend);
  if (want) {
    key.device = s->device;
    key.bits = s->fb_bits;
    memcpy(key.spend, s->consts.spend, sizeof(key.spend));
    if (s->fold_held && !(key < s->fold_key) && !(s->fold_key < key)) {
      s->consts.fb_top = s->fold_table;
      return CUDASP_OK;
    }
  }
  if (s->fold_held) {
    fold_release(s->fold_key);
    s->fold_held = false;
    s->fold_table = nullptr;
  }
  s->consts.fb_top = nullptr;
  if (!want) return CUDASP_OK;
  const uint32_t* t = nullptr;
  const int rc = fold_acquire(key, s->d_fb, &t, s->stream);  // no work of the scanner in flight
  if (rc != CUDASP_OK) return rc;
  s->fold_held = true;
  s->fold_key = key;
  s->fold_table = t;
  s->consts.fb_top = t;
  return CUDASP_OK;
}

void free_scanner(cudasp_scanner* s) {
  if (!s) return;
  if (s->fold_held) {
    fold_release(s->fold_key);
    s->fold_held = false;
  }
  DeviceGuard g(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  void* ptrs[] = {s->d_naf,  s->d_labels, s->d_t,       s->d_vscratch, s->d_lscratch, s->d_rows,
                  s->d_tx,   s->d_ty,     s->d_flags,   s->d_offs,     s->d_lens,     s->d_outputs,
                  s->d_vflags, s->d_multi, s->d_counter, s->d_mscratch};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (s->h_multi) (void)hipHostFree(s->h_multi);
  for (hipEvent_t e : s->multi_copied)
    if (e) (void)hipEventDestroy(e);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  if (!s->keys.empty()) wipe_bytes(s->keys.data(), s->keys.size());  // the scan private key
  delete s;
}

// The stage kernels' buffers, allocated on a scanner's first stage-kernel
// launch (sized for its capacity, output indices and label capacity).
int ensure_stage_buffers(cudasp_scanner* s) {
  if (s->d_t) return CUDASP_OK;
  DeviceGuard g(s->device);
  uint32_t* d_t = nullptr;
  uint8_t* d_vflags = nullptr;
  uint32_t* d_vscratch = nullptr;
  uint32_t* d_lscratch = nullptr;
  const size_t sizes[4] = {(size_t)8 * s->t_cap_k * s->capacity * 4, (size_t)s->t_cap_k * s->capacity,
                           (size_t)VSCRATCH_WORDS * s->slots_a * 4,
                           (size_t)lscratch_words(s->label_cap) * s->slots_b * 4};
  void** ptrs[4] = {(void**)&d_t, (void**)&d_vflags, (void**)&d_vscratch, (void**)&d_lscratch};
  for (int i = 0; i < 4; i++) {
    if (i == 1 && s->t_cap_k <= 1) continue;  // per-index flags only with output_count > 1
    hipError_t e = hipMalloc(ptrs[i], sizes[i] ? sizes[i] : 4);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      for (int j = 0; j < i; j++)
        if (*ptrs[j]) (void)hipFree(*ptrs[j]);
      return set_error(CUDASP_ERR_HIP, "hipMalloc(%zu) for the stage kernels failed: %s", sizes[i],
                       hipGetErrorString(e));
    }
  }
  s->d_t = d_t;
  s->d_vflags = d_vflags;
  s->d_vscratch = d_vscratch;
  s->d_lscratch = d_lscratch;
  return CUDASP_OK;
}

// Stage B with the LDS-staged 7-bit table (k_match_lds): 768-thread
// workgroups, 2 rows per thread (6 for launches large enough to fill the
// device at 6), within the label scratch's slots: every launched thread
// needs a slot, so the grid is capped at slots / LDS_BLOCK workgroups.  A
// small scanner (slots_b < LDS_BLOCK at 6 rows) takes 2 rows per thread,
// whose slots are smaller; if even one 2-row workgroup does not fit, the
// launch fails with CUDASP_ERR_CAPACITY instead of writing past the scratch.
int launch_match_lds(cudasp_scanner* s, const uint32_t* t, uint32_t n, const int64_t* outputs, const uint32_t* offs,
                     const uint32_t* lens, uint8_t* flags, uint32_t* match_rows, uint32_t* match_count,
                     int64_t* values, hipStream_t st) {
  const uint32_t K = s->consts.output_count;
  const uint32_t N = K * n;
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device);
  int r = s->rows_b_force ? s->rows_b_force
                          : ((N + ROWS_B - 1) / ROWS_B >= (uint32_t)cus * LDS_BLOCK ? ROWS_B : 2);
  auto cap_for = [s](int rows) {
    return (uint64_t)s->slots_b * lscratch_words(s->label_cap) /
           ((uint64_t)lscratch_words(s->label_count, rows) * LDS_BLOCK);
  };
  uint64_t cap = cap_for(r);
  if (cap == 0 && r != 2) {
    r = 2;
    cap = cap_for(r);
  }
  if (cap == 0)
    return set_error(CUDASP_ERR_CAPACITY,
                     "scanner too small for the LDS fixed-base width: %u scratch slots, a %d-thread workgroup "
                     "needs more; create it with more max_rows or use a 22/26-bit width",
                     s->slots_b, LDS_BLOCK);
  uint64_t blocks = ((N + r - 1) / (uint32_t)r + LDS_BLOCK - 1) / LDS_BLOCK;
  if (blocks > cap) blocks = cap;
  if (blocks > MAX_BLOCKS) blocks = MAX_BLOCKS;
  if (blocks == 0) blocks = 1;
  auto kv = r == ROWS_B ? k_match_lds<true, ROWS_B> : k_match_lds<true, 2>;
  auto kf = r == ROWS_B ? k_match_lds<false, ROWS_B> : k_match_lds<false, 2>;
  if (values) {
    hipLaunchKernelGGL(kv, dim3((uint32_t)blocks), dim3(LDS_BLOCK), 0, st, t, N, n, s->d_fb, s->consts, s->d_labels,
                       nullptr, nullptr, nullptr, s->d_lscratch, nullptr, nullptr, nullptr, values);
  } else if (K == 1) {
    hipLaunchKernelGGL(kf, dim3((uint32_t)blocks), dim3(LDS_BLOCK), 0, st, t, N, n, s->d_fb, s->consts, s->d_labels,
                       outputs, offs, lens, s->d_lscratch, flags, match_rows, match_count, nullptr);
  } else {
    hipLaunchKernelGGL(kf, dim3((uint32_t)blocks), dim3(LDS_BLOCK), 0, st, t, N, n, s->d_fb, s->consts, s->d_labels,
                       outputs, offs, lens, s->d_lscratch, s->d_vflags, nullptr, nullptr, nullptr);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_or_flags, dim3(grid_for(n)), dim3(BLOCK), 0, st, s->d_vflags, n, K, flags, match_rows,
                       match_count);
  }
  HIP_TRY(hipGetLastError());
  return CUDASP_OK;
}

// Stage B over the K n virtual rows of n input rows (t: 8 x (K n)); with
// K > 1 the per-index flags are ORed per input row before the compaction.
int launch_match(cudasp_scanner* s, const uint32_t* t, uint32_t n, const int64_t* outputs, const uint32_t* offs,
                 const uint32_t* lens, uint8_t* flags, uint32_t* match_rows, uint32_t* match_count, int64_t* values,
                 hipStream_t st) {
  const uint32_t K = s->consts.output_count;
  const uint32_t N = K * n;
  const int r = rows_b_for(s, N);
  const uint32_t blocks_b = grid_b(s, N, r);
  if (s->fb_bits == LDS_FB_BITS) return launch_match_lds(s, t, n, outputs, offs, lens, flags, match_rows, match_count,
                                                         values, st);
  const bool w26 = s->fb_bits == 26;
  auto kv = r == ROWS_B ? (w26 ? k_match<true, ROWS_B, 26> : k_match<true, ROWS_B, 22>)
                        : (w26 ? k_match<true, 2, 26> : k_match<true, 2, 22>);
  auto kf = r == ROWS_B ? (w26 ? k_match<false, ROWS_B, 26> : k_match<false, ROWS_B, 22>)
                        : (w26 ? k_match<false, 2, 26> : k_match<false, 2, 22>);
  if (values) {
    hipLaunchKernelGGL(kv, dim3(blocks_b), dim3(BLOCK), 0, st, t, N, n, s->d_fb, s->consts, s->d_labels, nullptr,
                       nullptr, nullptr, s->d_lscratch, nullptr, nullptr, nullptr, values);
  } else if (K == 1) {
    hipLaunchKernelGGL(kf, dim3(blocks_b), dim3(BLOCK), 0, st, t, N, n, s->d_fb, s->consts, s->d_labels, outputs,
                       offs, lens, s->d_lscratch, flags, match_rows, match_count, nullptr);
  } else {
    hipLaunchKernelGGL(kf, dim3(blocks_b), dim3(BLOCK), 0, st, t, N, n, s->d_fb, s->consts, s->d_labels, outputs,
                       offs, lens, s->d_lscratch, s->d_vflags, nullptr, nullptr, nullptr);
    HIP_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_or_flags, dim3(grid_for(n)), dim3(BLOCK), 0, st, s->d_vflags, n, K, flags, match_rows,
                       match_count);
  }
  HIP_TRY(hipGetLastError());
  return CUDASP_OK;
}

// Whether k_scan_multi can run this scanner's launches: output index 0 only
// (the reference's), an HBM fixed-base width, and scratch for at least one
// 256-thread block within 4 GiB (thousands of labels would not fit; those
// scanners use the two stage kernels).
static bool multi_ok(const cudasp_scanner* s) {
  return s->consts.output_count == 1 && (s->fb_bits == 22 || s->fb_bits == 26) &&
         (uint64_t)multi_scratch_words(s->consts.label_count, s->multi_pipe) * 4 * BLOCK <= (1ull << 32) - 1;
}

// Guided-scheduling parameters of k_scan_multi in hundredths of the grid's
// waves (multi_piece_rows): a piece is rem / (G1 x waves) rows; rmax rows
// while more than G2 x waves remain (0: no such phase).  CUDASP_MULTI_G1 /
// CUDASP_MULTI_G2 override the defaults (100 / 0) for tuning.
static uint32_t multi_threshold_x100(const char* env, uint32_t dflt_x100) {
  if (const char* e = getenv(env)) {
    const long v = atol(e);
    if (v >= 0 && v <= 100000) return (uint32_t)v;
  }
  return dflt_x100;
}

static MultiBatch multi_desc(const uint32_t* tx, const uint32_t* ty, const int64_t* outputs, const uint32_t* offs,
                             const uint32_t* lens, uint32_t n, uint8_t* flags, uint32_t* match_rows,
                             uint32_t* match_count, uint64_t first_wr) {
  MultiBatch m;
  m.tx = tx;
  m.ty = ty;
  m.outputs = outputs;
  m.offs = offs;
  m.lens = lens;
  m.flags = flags;
  const bool compact = match_rows && match_count;
  m.match_rows = compact ? match_rows : nullptr;
  m.match_count = compact ? match_count : nullptr;
  m.n = n;
  m.first_wr = (uint32_t)first_wr;
  return m;
}

// Blocks of a persistent k_scan_multi / k_scan_stream grid: at most
// CUDASP_WAVES_A waves per SIMD (one 256-thread block = one wave per SIMD of a
// CU), blocks_req if smaller (0 = the whole device), within 4 GiB of scratch
// (`words` per thread).
static uint64_t grid_blocks_for(cudasp_scanner* s, uint64_t blocks_req, uint64_t words) {
  if (!s->cus) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device) != hipSuccess || cus <= 0)
      cus = 256;
    s->cus = cus;
  }
  const uint64_t full_blocks = (uint64_t)s->cus * CUDASP_WAVES_A;
  const uint64_t cap_blocks = ((1ull << 32) - 1) / 4 / (words * BLOCK);
  uint64_t blocks = blocks_req ? blocks_req : full_blocks;
  if (blocks > full_blocks) blocks = full_blocks;
  if (blocks > cap_blocks) blocks = cap_blocks;
  if (blocks > MAX_BLOCKS) blocks = MAX_BLOCKS;
  return blocks;
}

static uint64_t multi_grid_blocks(cudasp_scanner* s, uint64_t blocks_req, bool pipe) {
  return grid_blocks_for(s, blocks_req, multi_scratch_words(s->consts.label_count, pipe));
}

static uint64_t stream_grid_blocks(cudasp_scanner* s, uint64_t blocks_req) {
  return grid_blocks_for(s, blocks_req, stream_scratch_words(s->consts.label_count));
}

// The streaming scan's options: any output_count (K x rows per piece <=
// MULTI_RMAX in the pipelined schedule, one row per piece and groups of
// MULTI_RMAX indices above that), an HBM fixed-base width, the pipelined
// schedule.
static_assert(CUDASP_STREAM_MAX_OUTPUT_COUNT == CUDASP_MAX_OUTPUT_COUNT, "every output_count streams");
static bool stream_ok(const cudasp_scanner* s) {
  return s->consts.output_count >= 1 && s->consts.output_count <= (uint32_t)CUDASP_STREAM_MAX_OUTPUT_COUNT &&
         (s->fb_bits == 22 || s->fb_bits == 26) && s->multi_pipe &&
         (uint64_t)stream_scratch_words(s->consts.label_count) * 4 * BLOCK <= (1ull << 32) - 1;
}

// k_scan_multi / k_scan_stream scratch for `blocks` blocks of `words` per
// thread.  Sized for the blocks a launch runs (a 300k-row fused batch: ~293
// of the 768 persistent blocks), grown when a later launch runs more.  An
// allocation failure is reported as CUDASP_ERR_CAPACITY before anything is
// queued, so launch_pipeline can fall back to the stage kernels.
static int ensure_scratch_words(cudasp_scanner* s, uint64_t blocks, uint64_t words, hipStream_t st) {
  const uint64_t need_words = blocks * BLOCK * words;
  if (need_words <= s->mscratch_words) return CUDASP_OK;
  HIP_TRY(hipStreamSynchronize(st));  // no kernel of this scanner still uses the old scratch
  if (s->d_mscratch) HIP_TRY(hipFree(s->d_mscratch));
  s->d_mscratch = nullptr;
  s->mscratch_words = 0;
  if (hipMalloc(&s->d_mscratch, (size_t)need_words * 4) != hipSuccess) {
    (void)hipGetLastError();
    s->d_mscratch = nullptr;
    return set_error(CUDASP_ERR_CAPACITY, "cannot allocate %.1f MB of k_scan_multi scratch", need_words * 4 / 1e6);
  }
  s->mscratch_words = need_words;
  return CUDASP_OK;
}

static int ensure_multi_scratch(cudasp_scanner* s, uint64_t blocks, bool pipe, hipStream_t st) {
  return ensure_scratch_words(s, blocks, multi_scratch_words(s->consts.label_count, pipe), st);
}

static int ensure_stream_scratch(cudasp_scanner* s, uint64_t blocks, hipStream_t st) {
  return ensure_scratch_words(s, blocks, stream_scratch_words(s->consts.label_count), st);
}

// One k_scan_multi launch over the described batches (total_wr wave-rows):
// uploads the descriptors, resets the work counter, launches on `st`.  rmax:
// rows per thread of the bulk; g1/g2: guided-scheduling parameters (hundredths of the
// grid's waves); blocks: 0 = the persistent grid (every wave slot), else a
// grid of that many blocks.
static int launch_multi(cudasp_scanner* s, const std::vector<MultiBatch>& md, uint64_t total_wr, hipStream_t st,
                        uint32_t rmax, uint32_t g1_x100, uint32_t g2_x100, uint64_t blocks_req) {
  if (total_wr >= (1ull << 31)) return set_error(CUDASP_ERR_CAPACITY, "too many rows in one multi-batch call");
  if (rmax < 1 || rmax > (uint32_t)MULTI_RMAX)  // the kernel's pending slots hold MULTI_RMAX rows per thread
    return set_error(CUDASP_ERR_INVALID_ARG, "multi-batch rows per thread %u outside 1..%d", rmax, MULTI_RMAX);
  const uint32_t nb = (uint32_t)md.size();
  constexpr uint32_t RING = sizeof(s->multi_pending) / sizeof(s->multi_pending[0]);
  if (nb > s->multi_cap) {
    for (uint32_t i = 0; i < RING; i++)  // every staged upload has been read before the areas move
      if (s->multi_pending[i]) {
        HIP_TRY(hipEventSynchronize(s->multi_copied[i]));
        s->multi_pending[i] = false;
      }
    if (s->d_multi) HIP_TRY(hipFree(s->d_multi));
    if (s->h_multi) HIP_TRY(hipHostFree(s->h_multi));
    s->d_multi = nullptr;
    s->h_multi = nullptr;
    s->multi_cap = 0;
    const uint32_t cap = nb < 256 ? 256 : nb;
    HIP_TRY(hipMalloc(&s->d_multi, (size_t)cap * sizeof(MultiBatch)));
    HIP_TRY(hipHostMalloc((void**)&s->h_multi, (size_t)cap * RING * sizeof(MultiBatch), hipHostMallocDefault));
    s->multi_cap = cap;
  }
  const uint32_t area = s->multi_next;
  s->multi_next = (area + 1) % RING;
  if (s->multi_pending[area]) {  // this area's previous upload must have been read before it is reused
    HIP_TRY(hipEventSynchronize(s->multi_copied[area]));
    s->multi_pending[area] = false;
  }
  if (!s->multi_copied[area]) HIP_TRY(hipEventCreateWithFlags(&s->multi_copied[area], hipEventDisableTiming));
  if (!s->d_counter) HIP_TRY(hipMalloc(&s->d_counter, sizeof(uint32_t)));
  uint64_t blocks = multi_grid_blocks(s, blocks_req, s->multi_pipe);
  const uint64_t need_blocks = (total_wr + 3) / 4;
  if (blocks > need_blocks) blocks = need_blocks;
  if (blocks == 0) return set_error(CUDASP_ERR_INVALID_ARG, "too many label keys for the multi-batch path");
  {
    const int rc = ensure_multi_scratch(s, blocks, s->multi_pipe, st);
    if (rc != CUDASP_OK) return rc;
  }
  // d_multi itself is reused in stream order: launches of one scanner run on
  // one stream (include/cudasp_abi.h), so this upload lands after the
  // previous kernel has read it
  MultiBatch* stage = s->h_multi + (size_t)area * s->multi_cap;
  memcpy(stage, md.data(), (size_t)nb * sizeof(MultiBatch));
  HIP_TRY(hipMemcpyAsync(s->d_multi, stage, (size_t)nb * sizeof(MultiBatch), hipMemcpyHostToDevice, st));
  HIP_TRY(hipEventRecord(s->multi_copied[area], st));
  s->multi_pending[area] = true;
  HIP_TRY(hipMemsetAsync(s->d_counter, 0, sizeof(uint32_t), st));
  const uint64_t waves = blocks * (BLOCK / 64);
  const uint32_t g1 = (uint32_t)(waves * g1_x100 / 100), g2 = (uint32_t)(waves * g2_x100 / 100);
  // the SIMDs' wave tiers by age on a grid of every wave slot (3 blocks per
  // CU, dispatched a CU-count at a time): the youngest third's claim rule
  // (multi_piece_rows_adaptive) and the drain priority (MultiTick)
  const bool tiers = CUDASP_WAVES_A == 3 && blocks == (uint64_t)s->cus * 3;
  const uint32_t young_from = tiers && s->multi_young ? (uint32_t)(2 * s->cus) : 0xFFFFFFFFu;
  const uint32_t tier_blocks = tiers && s->multi_endgame ? (uint32_t)s->cus : 0u;
  auto kf = s->multi_pipe ? (s->fb_bits == 26 ? k_scan_multi<26, true> : k_scan_multi<22, true>)
                          : (s->fb_bits == 26 ? k_scan_multi<26, false> : k_scan_multi<22, false>);
  hipLaunchKernelGGL(kf, dim3((uint32_t)blocks), dim3(BLOCK), 0, st, s->d_multi, nb, (uint32_t)total_wr, s->d_naf,
                     s->consts, s->d_fb, s->d_labels, s->d_mscratch, s->d_counter, g1, g2, rmax,
                     s->multi_adaptive ? 1u : 0u, young_from, tier_blocks);
  HIP_TRY(hipGetLastError());
  return CUDASP_OK;
}

int launch_pipeline(cudasp_scanner* s, const uint32_t* tx, const uint32_t* ty, const int64_t* outputs,
                    const uint32_t* offs, const uint32_t* lens, uint32_t n, uint8_t* flags, uint32_t* match_rows,
                    uint32_t* match_count, int64_t* values, uint32_t* t_out, hipStream_t st) {
  if (n == 0) return CUDASP_OK;
  if (n > s->capacity) return set_error(CUDASP_ERR_CAPACITY, "batch of %u rows exceeds scanner capacity %u", n, s->capacity);
  if (s->fused_single && !values && !t_out && flags && multi_ok(s) && !s->rows_a_force && !s->rows_b_force) {
    // both stages in one k_scan_multi launch over this batch: ROWS_A rows per
    // thread throughout, one wave per chunk
    // (R = rows_a_for: 4, or 2 / 1 for a launch too small to fill a quarter
    // of the device at 4, so the tail batch of a query runs 2-4x shorter)
    std::vector<MultiBatch> md(1, multi_desc(tx, ty, outputs, offs, lens, n, flags, match_rows, match_count, 0));
    const uint64_t wr = (n + 63u) / 64u;
    const uint32_t R = (uint32_t)rows_a_for(s, n);
    const int rc = launch_multi(s, md, wr, st, R, 0, 0, (wr + R * 4 - 1) / (R * 4));
    // CUDASP_ERR_CAPACITY: no scratch for the fused launch and nothing queued;
    // the two stage kernels below give the same results
    if (rc != CUDASP_ERR_CAPACITY) return rc;
  }
  const int brc = ensure_stage_buffers(s);
  if (brc != CUDASP_OK) return brc;
  uint32_t* t = t_out ? t_out : s->d_t;
  launch_a(s, tx, ty, n, t, st);
  HIP_TRY(hipGetLastError());
  return launch_match(s, t, n, outputs, offs, lens, flags, match_rows, match_count, values, st);
}

}  // namespace

extern "C" {

const char* cudasp_last_error(void) { return g_last_error.c_str(); }

// Used by the table-function host (csrc/host) to report through the same
// thread-local message; not part of the public header.
void cudasp_internal_set_error(const char* msg) { g_last_error = msg ? msg : ""; }
// The table-function host's device feeds launch each batch's copies and
// kernels on the stream of the scanner that scans it; not public either.
void* cudasp_internal_scanner_stream(cudasp_scanner* s) { return s ? (void*)s->stream : nullptr; }
// A scanner parked in the table-function host's pool: its spend key's fold
// table is released (so parked scanners do not keep old wallets' 268 MB
// tables alive; at most FOLD_CACHED_PER_DEVICE unreferenced ones stay cached),
// and its next cudasp_scanner_set_keys prepares again, even for the same
// keys, taking the fold table back.  No work of the scanner may be in flight.
void cudasp_internal_scanner_park(cudasp_scanner* s) {
  if (!s) return;
  if (s->fold_held) {
    fold_release(s->fold_key);
    s->fold_held = false;
    s->fold_table = nullptr;
  }
  s->consts.fb_top = nullptr;
  s->prepared = false;
}
// Wipe the process-wide scan-key digit cache (cudasp_tf_release_pool).
void cudasp_internal_clear_key_cache(void) { scan_digits_cache_clear(); }

const char* cudasp_version(void) { return CUDASP_VERSION_STRING; }

int cudasp_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int cudasp_scanner_create(int device, const uint8_t scan_private_key[32], const uint8_t spend_public_key[64],
                          const uint8_t* label_keys, uint32_t label_count, uint32_t max_rows,
                          cudasp_scanner** out) {
  g_last_error.clear();
  if (!out || !scan_private_key || !spend_public_key || (label_count > 0 && !label_keys))
    return set_error(CUDASP_ERR_INVALID_ARG, "null argument");
  *out = nullptr;
  int ndev = cudasp_device_count();
  if (ndev <= 0) return set_error(CUDASP_ERR_NO_DEVICE, "no HIP device visible");
  if (device < 0 || device >= ndev) return set_error(CUDASP_ERR_INVALID_ARG, "device %d out of range (%d devices)", device, ndev);
  if (max_rows == 0) max_rows = 1;

  // --- host-side constants -------------------------------------------------
  cudasp_scanner* s = new cudasp_scanner();
  std::vector<int8_t> naf;
  std::vector<uint32_t> labels;
  std::string err;
  int prc = prepare_scan(scan_private_key, spend_public_key, label_keys, label_count, s->consts, naf, labels, err);
  if (prc != CUDASP_OK) {
    delete s;
    return set_error(prc, "%s", err.c_str());
  }
  s->device = device;
  s->capacity = max_rows;
  s->label_count = label_count;
  s->label_cap = label_count;
  s->keys.assign(scan_private_key, scan_private_key + 32);
  s->keys.insert(s->keys.end(), spend_public_key, spend_public_key + 64);
  if (label_count) s->keys.insert(s->keys.end(), label_keys, label_keys + 64 * (size_t)label_count);
  s->raw_label_count = label_count;

  // --- device state --------------------------------------------------------
  DeviceGuard g(device);
  s->fb_bits = default_fb_bits(device);
  // the scanner's stream first: a first scanner builds the device's
  // fixed-base table on it
  hipError_t e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    s->stream = nullptr;
    free_scanner(s);
    return set_error(CUDASP_ERR_HIP, "hipStreamCreate failed: %s", hipGetErrorString(e));
  }
  int rc = ensure_device_table(device, s->fb_bits, &s->d_fb, nullptr, s->stream);
  if (rc != CUDASP_OK) {
    free_scanner(s);
    return rc;
  }
  // One scratch slot per thread of the largest launch; each scratch buffer is
  // kept below 4 GiB (32-bit buffer offsets, make_scratch) by capping the grid,
  // the kernels' grid-stride loops take the remaining rows.
  auto slots_for = [](uint32_t groups, uint64_t words_per_slot) {
    uint64_t cap_blocks = ((1ull << 32) - 1) / (words_per_slot * 4 * BLOCK);
    uint64_t blocks = grid_for(groups);
    if (blocks > cap_blocks) blocks = cap_blocks ? cap_blocks : 1;
    return (uint32_t)blocks * BLOCK;
  };
  s->slots_a = slots_for((max_rows + ROWS_A - 1) / ROWS_A, VSCRATCH_WORDS);
  s->slots_b = slots_for((max_rows + ROWS_B - 1) / ROWS_B, lscratch_words(label_count));
  {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
      cus = 256;
    // a quarter of the wave slots (4 SIMDs per CU, CUDASP_WAVES_A waves each)
    s->fill_threads = (uint32_t)cus * 4 * CUDASP_WAVES_A * 64 / 4;
    s->fill_threads_b = (uint32_t)cus * 4 * CUDASP_WAVES_B * 64 / 4;
    if (const char* f = getenv("CUDASP_FUSED_SINGLE")) s->fused_single = atoi(f) != 0;
    if (const char* f = getenv("CUDASP_MULTI_PIPE")) s->multi_pipe = atoi(f) != 0;
    if (const char* f = getenv("CUDASP_MULTI_ADAPT")) s->multi_adaptive = atoi(f) != 0;
    if (const char* f = getenv("CUDASP_MULTI_ENDGAME")) s->multi_endgame = atoi(f) != 0;
    if (const char* f = getenv("CUDASP_MULTI_YOUNG")) s->multi_young = atoi(f) != 0;
    if (const char* f = getenv("CUDASP_ROWS_A_FORCE")) {
      const int r = atoi(f);
      if (r == 1 || r == 2 || r == ROWS_A) s->rows_a_force = r;
    }
    if (const char* f = getenv("CUDASP_ROWS_B_FORCE")) {
      const int r = atoi(f);
      if (r == 2 || r == ROWS_B) s->rows_b_force = r;
    }
  }
  if ((uint64_t)lscratch_words(label_count) * 4 * BLOCK > (1ull << 32) - 1) {
    delete s;
    return set_error(CUDASP_ERR_INVALID_ARG, "too many label keys (%u)", label_count);
  }
#define ALLOC(ptr, bytes)                                                                          \
  do {                                                                                             \
    hipError_t e_ = hipMalloc(&(ptr), (bytes) ? (bytes) : 4);                                      \
    if (e_ != hipSuccess) {                                                                        \
      free_scanner(s);                                                                             \
      return set_error(CUDASP_ERR_HIP, "hipMalloc(%zu) failed: %s", (size_t)(bytes), hipGetErrorString(e_)); \
    }                                                                                              \
  } while (0)
  ALLOC(s->d_naf, naf.size());
  ALLOC(s->d_labels, labels.size() * 4);
#undef ALLOC
  // d_t / d_vscratch / d_lscratch: on first stage-kernel use (ensure_stage_buffers)
  e = hipMemcpy(s->d_naf, naf.data(), naf.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(s->d_labels, labels.data(), labels.size() * 4, hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    free_scanner(s);
    return set_error(CUDASP_ERR_HIP, "hipMemcpy failed: %s", hipGetErrorString(e));
  }
  rc = scanner_update_fold(s);
  if (rc != CUDASP_OK) {
    free_scanner(s);
    return rc;
  }
  s->prepared = true;  // prepare_scan above used the default options (s->opt)
  *out = s;
  return CUDASP_OK;
}

void cudasp_scanner_destroy(cudasp_scanner* s) { free_scanner(s); }

int cudasp_scanner_set_keys(cudasp_scanner* s, const uint8_t scan_private_key[32],
                            const uint8_t spend_public_key[64], const uint8_t* label_keys, uint32_t label_count) {
  g_last_error.clear();
  if (!s || !scan_private_key || !spend_public_key || (label_count > 0 && !label_keys))
    return set_error(CUDASP_ERR_INVALID_ARG, "null argument");
  // the keys and options the scanner's constants were prepared for: nothing
  // to do (a pooled scanner rebound to the same wallet, query after query)
  if (s->prepared && label_count == s->raw_label_count && s->keys.size() == 96 + 64 * (size_t)label_count &&
      memcmp(s->keys.data(), scan_private_key, 32) == 0 && memcmp(s->keys.data() + 32, spend_public_key, 64) == 0 &&
      (label_count == 0 || memcmp(s->keys.data() + 96, label_keys, 64 * (size_t)label_count) == 0) &&
      memcmp(&s->prepared_opt, &s->opt, sizeof(s->opt)) == 0)
    return CUDASP_OK;
  ScanConsts consts;
  std::vector<int8_t> naf;
  std::vector<uint32_t> labels;
  std::string err;
  int prc = prepare_scan(scan_private_key, spend_public_key, label_keys, label_count, consts, naf, labels, err,
                         &s->opt);
  if (prc != CUDASP_OK) return set_error(prc, "%s", err.c_str());
  const uint32_t raw_label_count = label_count;
  label_count = consts.label_count;  // with the negated copies
  if ((uint64_t)lscratch_words(label_count) * 4 * BLOCK > (1ull << 32) - 1)
    return set_error(CUDASP_ERR_INVALID_ARG, "too many label keys (%u)", label_count);
  DeviceGuard g(s->device);
  HIP_TRY(hipStreamSynchronize(s->stream));
  if (label_count > s->label_cap) {
    // grow the label keys and the label scratch (same slot count when it fits;
    // the scratch only if the stage buffers exist yet)
    uint32_t* d_labels = nullptr;
    uint32_t* d_lscratch = nullptr;
    uint64_t words = lscratch_words(label_count);
    uint64_t cap_slots = ((1ull << 32) - 1) / (words * 4 * BLOCK) * BLOCK;
    uint32_t slots_b = (uint32_t)(s->slots_b < cap_slots ? s->slots_b : cap_slots);
    HIP_TRY(hipMalloc(&d_labels, labels.size() * 4));
    hipError_t e = s->d_lscratch ? hipMalloc(&d_lscratch, (size_t)words * slots_b * 4) : hipSuccess;
    if (e != hipSuccess) {
      (void)hipFree(d_labels);
      return set_error(CUDASP_ERR_HIP, "hipMalloc failed: %s", hipGetErrorString(e));
    }
    (void)hipFree(s->d_labels);
    if (s->d_lscratch) (void)hipFree(s->d_lscratch);
    s->d_labels = d_labels;
    s->d_lscratch = d_lscratch;
    s->slots_b = slots_b;
    s->label_cap = label_count;
  }
  HIP_TRY(hipMemcpy(s->d_naf, naf.data(), naf.size(), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(s->d_labels, labels.data(), labels.size() * 4, hipMemcpyHostToDevice));
  s->consts = consts;
  s->label_count = label_count;
  {
    const int rc = scanner_update_fold(s);
    if (rc != CUDASP_OK) return rc;
  }
  s->prepared = true;
  s->prepared_opt = s->opt;
  if (s->keys.data() != scan_private_key) {
    std::vector<uint8_t> keys(scan_private_key, scan_private_key + 32);
    keys.insert(keys.end(), spend_public_key, spend_public_key + 64);
    if (raw_label_count) keys.insert(keys.end(), label_keys, label_keys + 64 * (size_t)raw_label_count);
    s->keys.swap(keys);
    if (!keys.empty()) wipe_bytes(keys.data(), keys.size());  // the previous scan key
    s->raw_label_count = raw_label_count;
  }
  return CUDASP_OK;
}

int cudasp_scanner_set_options(cudasp_scanner* s, const cudasp_scan_options* options) {
  g_last_error.clear();
  if (!s || !options) return set_error(CUDASP_ERR_INVALID_ARG, "null argument");
  const uint32_t K = options->output_count;
  if (K < 1 || K > CUDASP_MAX_OUTPUT_COUNT)
    return set_error(CUDASP_ERR_INVALID_ARG, "output_count must be between 1 and %d", CUDASP_MAX_OUTPUT_COUNT);
  if ((uint64_t)K * s->capacity > 0xFFFFFFFFull)
    return set_error(CUDASP_ERR_CAPACITY, "output_count %u x capacity %u exceeds 2^32 virtual rows", K, s->capacity);
  if (K == s->opt.output_count && (options->label_negation != 0) == (s->opt.label_negation != 0) &&
      (options->full_x != 0) == (s->opt.full_x != 0) && s->prepared &&
      memcmp(&s->prepared_opt, &s->opt, sizeof(s->opt)) == 0)
    return CUDASP_OK;  // unchanged
  DeviceGuard g(s->device);
  HIP_TRY(hipStreamSynchronize(s->stream));
  if (K > s->t_cap_k && !s->d_t) {
    s->t_cap_k = K;  // the stage buffers do not exist yet: sized at first use
  } else if (K > s->t_cap_k) {
    uint32_t* d_t = nullptr;
    uint8_t* d_vflags = nullptr;
    HIP_TRY(hipMalloc(&d_t, (size_t)8 * K * s->capacity * 4));
    hipError_t e = hipMalloc(&d_vflags, (size_t)K * s->capacity);
    if (e != hipSuccess) {
      (void)hipFree(d_t);
      return set_error(CUDASP_ERR_HIP, "hipMalloc failed: %s", hipGetErrorString(e));
    }
    (void)hipFree(s->d_t);
    (void)hipFree(s->d_vflags);
    s->d_t = d_t;
    s->d_vflags = d_vflags;
    s->t_cap_k = K;
  }
  const cudasp_scan_options old = s->opt;
  s->opt = *options;
  s->opt.label_negation = options->label_negation ? 1u : 0u;
  s->opt.full_x = options->full_x ? 1u : 0u;
  const uint8_t* k = s->keys.data();
  int rc = cudasp_scanner_set_keys(s, k, k + 32, s->raw_label_count ? k + 96 : nullptr, s->raw_label_count);
  if (rc != CUDASP_OK) s->opt = old;
  return rc;
}

int cudasp_default_fixed_base_bits(void) { return default_fb_bits(); }

uint64_t cudasp_fixed_base_table_bytes(int bits) { return fb_bits_supported(bits) ? (uint64_t)fb_table_bytes(bits) : 0; }

int cudasp_fixed_base_prepare(int device, int bits, double* build_seconds) {
  g_last_error.clear();
  if (build_seconds) *build_seconds = 0;
  const int ndev = cudasp_device_count();
  if (ndev <= 0) return set_error(CUDASP_ERR_NO_DEVICE, "no HIP device visible");
  if (device < 0 || device >= ndev) return set_error(CUDASP_ERR_INVALID_ARG, "device %d out of range", device);
  DeviceGuard g(device);
  if (bits == 0) bits = default_fb_bits(device);
  const auto t0 = std::chrono::steady_clock::now();
  bool built = false;
  const uint32_t* fb = nullptr;
  const int rc = ensure_device_table(device, bits, &fb, &built);
  if (rc == CUDASP_OK && built && build_seconds)
    *build_seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return rc;
}

int cudasp_debug_fb_check(int device, int bits, uint32_t stride, uint64_t* checked, uint64_t* mismatched) {
  g_last_error.clear();
  if (!checked || !mismatched || stride == 0) return set_error(CUDASP_ERR_INVALID_ARG, "bad argument");
  int rc = cudasp_fixed_base_prepare(device, bits, nullptr);
  if (rc != CUDASP_OK) return rc;
  DeviceGuard g(device);
  if (bits == 0) bits = default_fb_bits(device);
  const uint32_t* fb = nullptr;
  rc = ensure_device_table(device, bits, &fb);
  if (rc != CUDASP_OK) return rc;
  const uint32_t windows = (256 + bits - 1) / bits, entries = 1u << (bits - 1);
  const std::vector<uint32_t> bases = fb_window_bases(bits);
  uint32_t *d_bases = nullptr, *d_bad = nullptr;
  HIP_TRY(hipMalloc(&d_bases, bases.size() * 4));
  HIP_TRY(hipMalloc(&d_bad, 4));
  HIP_TRY(hipMemcpy(d_bases, bases.data(), bases.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(d_bad, 0, 4));
  hipLaunchKernelGGL(k_fb_check, dim3(1024), dim3(BLOCK), 0, 0, d_bases, windows, entries, fb, stride, d_bad);
  HIP_TRY(hipGetLastError());
  uint32_t bad = 0;
  HIP_TRY(hipMemcpy(&bad, d_bad, 4, hipMemcpyDeviceToHost));
  (void)hipFree(d_bases);
  (void)hipFree(d_bad);
  const uint64_t total = (uint64_t)windows * entries;
  *checked = (total + stride - 1) / stride;
  *mismatched = bad;
  return CUDASP_OK;
}

int cudasp_debug_fold_check(int device, int bits, const uint8_t spend_public_key[64], uint32_t stride,
                            uint64_t* checked, uint64_t* mismatched) {
  g_last_error.clear();
  if (!checked || !mismatched || !spend_public_key || stride == 0 || (bits != 22 && bits != 26))
    return set_error(CUDASP_ERR_INVALID_ARG, "bad argument");
  int rc = cudasp_fixed_base_prepare(device, bits, nullptr);
  if (rc != CUDASP_OK) return rc;
  DeviceGuard g(device);
  const uint32_t* fb = nullptr;
  rc = ensure_device_table(device, bits, &fb);
  if (rc != CUDASP_OK) return rc;
  FoldKey key{};
  key.device = device;
  key.bits = bits;
  hp_words(key.spend, hp_from_bytes(spend_public_key));
  uint32_t* fold = fold_build(key, fb, nullptr);
  if (!fold) return set_error(CUDASP_ERR_INVALID_ARG, "the spend key cannot be folded");
  SpendWords sw;
  memcpy(sw.w, key.spend, sizeof(sw.w));
  uint32_t* d_bad = nullptr;
  uint32_t bad = 0;
  hipError_t e2 = hipMalloc(&d_bad, 4);
  if (e2 == hipSuccess) e2 = hipMemset(d_bad, 0, 4);
  if (e2 == hipSuccess) {
    auto kf = bits == 26 ? k_fold_check<26> : k_fold_check<22>;
    hipLaunchKernelGGL(kf, dim3(1024), dim3(BLOCK), 0, 0, fb, sw, fold, stride, d_bad);
    e2 = hipGetLastError();
  }
  if (e2 == hipSuccess) e2 = hipMemcpy(&bad, d_bad, 4, hipMemcpyDeviceToHost);
  (void)hipGetLastError();
  if (d_bad) (void)hipFree(d_bad);
  (void)hipFree(fold);  // every path frees both
  if (e2 != hipSuccess) return set_error(CUDASP_ERR_HIP, "fold check failed: %s", hipGetErrorString(e2));
  const uint64_t top = bits == 26 ? FbWidth<26>::TOP_ENTRIES : FbWidth<22>::TOP_ENTRIES;
  *checked = (top + stride - 1) / stride;
  *mismatched = bad;
  return CUDASP_OK;
}

int cudasp_scanner_set_fixed_base_bits(cudasp_scanner* s, int bits) {
  g_last_error.clear();
  if (!s) return set_error(CUDASP_ERR_INVALID_ARG, "null scanner");
  if (bits == 0) bits = default_fb_bits(s->device);
  if (bits == s->fb_bits) return CUDASP_OK;
  DeviceGuard g(s->device);
  HIP_TRY(hipStreamSynchronize(s->stream));
  const uint32_t* fb = nullptr;
  int rc = ensure_device_table(s->device, bits, &fb, nullptr, s->stream);
  if (rc != CUDASP_OK) return rc;
  s->d_fb = fb;
  s->fb_bits = bits;
  return scanner_update_fold(s);
}

int cudasp_scanner_fixed_base_bits(const cudasp_scanner* s) { return s ? s->fb_bits : 0; }

int cudasp_scanner_set_spend_fold(cudasp_scanner* s, int on) {
  g_last_error.clear();
  if (!s) return set_error(CUDASP_ERR_INVALID_ARG, "null scanner");
  if (s->fold_allowed == (on != 0)) return CUDASP_OK;
  DeviceGuard g(s->device);
  HIP_TRY(hipStreamSynchronize(s->stream));
  s->fold_allowed = on != 0;
  return scanner_update_fold(s);
}

int cudasp_scanner_spend_folded(const cudasp_scanner* s) { return s && s->consts.fb_top ? 1 : 0; }

int cudasp_scanner_set_rows_per_thread(cudasp_scanner* s, int rows_a, int rows_b) {
  g_last_error.clear();
  if (!s) return set_error(CUDASP_ERR_INVALID_ARG, "null scanner");
  if (!(rows_a == 0 || rows_a == 1 || rows_a == 2 || rows_a == ROWS_A) || !(rows_b == 0 || rows_b == 2 || rows_b == ROWS_B))
    return set_error(CUDASP_ERR_INVALID_ARG, "rows per thread: stage A 0, 1, 2 or %d; stage B 0, 2 or %d", ROWS_A,
                     ROWS_B);
  s->rows_a_force = rows_a;
  s->rows_b_force = rows_b;
  return CUDASP_OK;
}

int cudasp_scanner_sync(cudasp_scanner* s) {
  if (!s) return set_error(CUDASP_ERR_INVALID_ARG, "null scanner");
  DeviceGuard g(s->device);
  HIP_TRY(hipStreamSynchronize(s->stream));
  return CUDASP_OK;
}

int cudasp_scan_device(cudasp_scanner* s, const uint32_t* d_tweak_x, const uint32_t* d_tweak_y,
                       const int64_t* d_outputs, const uint32_t* d_output_offsets,
                       const uint32_t* d_output_lengths, uint32_t n, uint8_t* d_match_flags,
                       uint32_t* d_match_rows, uint32_t* d_match_count, void* stream) {
  if (!s) return set_error(CUDASP_ERR_INVALID_ARG, "null scanner");
  if (n == 0) return CUDASP_OK;
  if (!d_tweak_x || !d_tweak_y || !d_output_offsets || !d_output_lengths || !d_match_flags)
    return set_error(CUDASP_ERR_INVALID_ARG, "null device buffer");
  DeviceGuard g(s->device);
  hipStream_t st = scanner_stream(s, stream);
  return launch_pipeline(s, d_tweak_x, d_tweak_y, d_outputs, d_output_offsets, d_output_lengths, n, d_match_flags,
                         (d_match_rows && d_match_count) ? d_match_rows : nullptr,
                         (d_match_rows && d_match_count) ? d_match_count : nullptr, nullptr, nullptr, st);
}

int cudasp_scan_device_batches(cudasp_scanner* s, const cudasp_device_batch* batches, uint32_t count, void* stream) {
  if (!s) return set_error(CUDASP_ERR_INVALID_ARG, "null scanner");
  if (count == 0) return CUDASP_OK;
  if (!batches) return set_error(CUDASP_ERR_INVALID_ARG, "null batch array");
  for (uint32_t i = 0; i < count; i++) {
    const cudasp_device_batch& b = batches[i];
    if (b.n && (!b.tweak_x || !b.tweak_y || !b.output_offsets || !b.output_lengths || !b.match_flags))
      return set_error(CUDASP_ERR_INVALID_ARG, "batch %u: null device buffer", i);
  }
  const bool persistent = multi_ok(s);
  if (!persistent) {  // the per-batch path (protocol variants, the LDS width, very many labels)
    for (uint32_t i = 0; i < count; i++) {
      const cudasp_device_batch& b = batches[i];
      int rc = cudasp_scan_device(s, b.tweak_x, b.tweak_y, b.outputs, b.output_offsets, b.output_lengths, b.n,
                                  b.match_flags, b.match_rows, b.match_count, stream);
      if (rc != CUDASP_OK) return rc;
    }
    return CUDASP_OK;
  }
  DeviceGuard g(s->device);
  hipStream_t st = scanner_stream(s, stream);
  // descriptors: batches with rows only, each starting at a fresh wave-row
  std::vector<MultiBatch> md;
  md.reserve(count);
  uint64_t total_wr = 0;
  for (uint32_t i = 0; i < count; i++) {
    const cudasp_device_batch& b = batches[i];
    if (b.n == 0) continue;
    md.push_back(multi_desc(b.tweak_x, b.tweak_y, b.outputs, b.output_offsets, b.output_lengths, b.n, b.match_flags,
                            b.match_rows, b.match_count, total_wr));
    total_wr += (b.n + 63u) / 64u;
  }
  if (md.empty()) return CUDASP_OK;
  // CUDASP_MULTI_ROWS = 2..MULTI_RMAX: rows per thread of the bulk (tuning)
  uint32_t rmax = MULTI_RMAX;
  if (const char* e = getenv("CUDASP_MULTI_ROWS")) {
    const long v = atol(e);
    if (v >= 2 && v <= MULTI_RMAX) rmax = (uint32_t)v;
  }
  // CUDASP_MULTI_BLOCKS = a grid of that many blocks instead of every wave slot (tuning)
  uint64_t blocks = 0;
  if (const char* e = getenv("CUDASP_MULTI_BLOCKS")) {
    const long v = atol(e);
    if (v >= 1 && v <= MAX_BLOCKS) blocks = (uint64_t)v;
  }
  return launch_multi(s, md, total_wr, st, rmax, multi_threshold_x100("CUDASP_MULTI_G1", 100),
                      multi_threshold_x100("CUDASP_MULTI_G2", 0), blocks);
}

int cudasp_debug_multi_clock(int device, double* mhz, double* seconds) {
  if (!mhz) return set_error(CUDASP_ERR_INVALID_ARG, "null argument");
  DeviceGuard g(device);
  uint64_t c[4] = {};
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(c, HIP_SYMBOL(g_multi_clock), sizeof(c)));
  int rate_khz = 0;
  HIP_TRY(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, device));
  if (c[3] <= c[1] || rate_khz <= 0) return set_error(CUDASP_ERR_INVALID_ARG, "no k_scan_multi launch recorded");
  const double secs = (double)(c[3] - c[1]) / (rate_khz * 1e3);
  *mhz = (double)(c[2] - c[0]) / secs / 1e6;
  if (seconds) *seconds = secs;
  return CUDASP_OK;
}

#if CUDASP_MULTI_TRACE
// Measurement builds only (not in include/cudasp_abi.h): copies up to
// max_waves records (8 words: start, end, pieces, wave-rows, placement,
// exhausted, shader ticks, last stage A) of the last k_scan_multi launch; returns the
// number of records and the realtime clock in *hz.
extern "C" int cudasp_debug_multi_trace(uint64_t* out, uint32_t max_waves, int* hz) {
  const uint32_t n = max_waves < MULTI_TRACE_WAVES ? max_waves : MULTI_TRACE_WAVES;
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_multi_trace), (size_t)n * MULTI_TRACE_WORDS * sizeof(uint64_t)));
  int dev = 0, rate_khz = 0;
  HIP_TRY(hipGetDevice(&dev));
  HIP_TRY(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, dev));
  *hz = rate_khz * 1000;
  return (int)n;
}
#endif

int cudasp_row_values_device(cudasp_scanner* s, const uint32_t* d_tweak_x, const uint32_t* d_tweak_y, uint32_t n,
                             uint32_t* d_t, int64_t* d_values, void* stream) {
  if (!s) return set_error(CUDASP_ERR_INVALID_ARG, "null scanner");
  if (n == 0) return CUDASP_OK;
  if (!d_tweak_x || !d_tweak_y || !d_values) return set_error(CUDASP_ERR_INVALID_ARG, "null device buffer");
  DeviceGuard g(s->device);
  hipStream_t st = scanner_stream(s, stream);
  return launch_pipeline(s, d_tweak_x, d_tweak_y, nullptr, nullptr, nullptr, n, nullptr, nullptr, nullptr, d_values,
                         d_t, st);
}

int cudasp_tweaks_to_columns(const uint8_t* d_tweak_rows, uint32_t n, uint32_t* d_tweak_x, uint32_t* d_tweak_y,
                             void* stream) {
  if (n == 0) return CUDASP_OK;
  if (!d_tweak_rows || !d_tweak_x || !d_tweak_y) return set_error(CUDASP_ERR_INVALID_ARG, "null device buffer");
  hipLaunchKernelGGL(k_rows_to_cols, dim3(grid_for(n)), dim3(BLOCK), 0, plain_stream(stream), d_tweak_rows, n,
                     d_tweak_x, d_tweak_y);
  HIP_TRY(hipGetLastError());
  return CUDASP_OK;
}

int cudasp_layout_probe(const uint32_t* d_tweak_x, const uint32_t* d_tweak_y, uint32_t n, const int64_t* d_outputs,
                        const uint32_t* d_output_offsets, const uint32_t* d_output_lengths, uint8_t* d_flags,
                        void* stream) {
  if (n == 0) return CUDASP_OK;
  if (!d_tweak_x || !d_tweak_y || !d_output_offsets || !d_output_lengths || !d_flags)
    return set_error(CUDASP_ERR_INVALID_ARG, "null device buffer");
  const uint32_t groups = (n + ROWS_A - 1) / ROWS_A;
  hipLaunchKernelGGL(k_layout_probe, dim3(grid_for(groups)), dim3(BLOCK), 0, plain_stream(stream), d_tweak_x,
                     d_tweak_y, n, d_outputs, d_output_offsets, d_output_lengths, d_flags);
  HIP_TRY(hipGetLastError());
  return CUDASP_OK;
}

int cudasp_scan_host(cudasp_scanner* s, const uint8_t* h_tweak_keys, const int64_t* h_outputs, size_t outputs_size,
                     const uint32_t* h_output_offsets, const uint32_t* h_output_lengths, uint32_t n,
                     uint8_t* h_match_flags) {
  if (!s) return set_error(CUDASP_ERR_INVALID_ARG, "null scanner");
  if (n == 0) return CUDASP_OK;
  if (!h_tweak_keys || !h_output_offsets || !h_output_lengths || !h_match_flags || (outputs_size && !h_outputs))
    return set_error(CUDASP_ERR_INVALID_ARG, "null host buffer");
  if (n > s->capacity) return set_error(CUDASP_ERR_CAPACITY, "batch of %u rows exceeds scanner capacity %u", n, s->capacity);
  for (uint32_t i = 0; i < n; i++)
    if ((size_t)h_output_offsets[i] + h_output_lengths[i] > outputs_size)
      return set_error(CUDASP_ERR_INVALID_ARG, "row %u: outputs range [%u, +%u) exceeds outputs_size %zu", i,
                       h_output_offsets[i], h_output_lengths[i], outputs_size);
  DeviceGuard g(s->device);
  if (!s->d_rows) {
    HIP_TRY(hipMalloc(&s->d_rows, (size_t)64 * s->capacity));
    HIP_TRY(hipMalloc(&s->d_tx, (size_t)32 * s->capacity));
    HIP_TRY(hipMalloc(&s->d_ty, (size_t)32 * s->capacity));
    HIP_TRY(hipMalloc(&s->d_flags, (size_t)s->capacity));
    HIP_TRY(hipMalloc(&s->d_offs, (size_t)4 * s->capacity));
    HIP_TRY(hipMalloc(&s->d_lens, (size_t)4 * s->capacity));
  }
  const size_t out_bytes = outputs_size * (s->consts.full_x ? 32 : 8);  // one int64 or one 32-byte x
  if (out_bytes > s->outputs_cap) {
    if (s->d_outputs) HIP_TRY(hipFree(s->d_outputs));
    s->d_outputs = nullptr;
    HIP_TRY(hipMalloc(&s->d_outputs, out_bytes));
    s->outputs_cap = out_bytes;
  }
  hipStream_t st = s->stream;
  HIP_TRY(hipMemcpyAsync(s->d_rows, h_tweak_keys, (size_t)64 * n, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(s->d_offs, h_output_offsets, (size_t)4 * n, hipMemcpyHostToDevice, st));
  HIP_TRY(hipMemcpyAsync(s->d_lens, h_output_lengths, (size_t)4 * n, hipMemcpyHostToDevice, st));
  if (outputs_size) HIP_TRY(hipMemcpyAsync(s->d_outputs, h_outputs, out_bytes, hipMemcpyHostToDevice, st));
  int rc = cudasp_tweaks_to_columns(s->d_rows, n, s->d_tx, s->d_ty, st);
  if (rc != CUDASP_OK) return rc;
  rc = launch_pipeline(s, s->d_tx, s->d_ty, s->d_outputs, s->d_offs, s->d_lens, n, s->d_flags, nullptr, nullptr,
                       nullptr, nullptr, st);
  if (rc != CUDASP_OK) return rc;
  HIP_TRY(hipMemcpyAsync(h_match_flags, s->d_flags, n, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  return CUDASP_OK;
}

int cudasp_stage_shared_secret_device(cudasp_scanner* s, const uint32_t* d_tweak_x, const uint32_t* d_tweak_y,
                                      uint32_t n, uint32_t* d_t, void* stream) {
  if (!s) return set_error(CUDASP_ERR_INVALID_ARG, "null scanner");
  if (n == 0) return CUDASP_OK;
  if (!d_tweak_x || !d_tweak_y || !d_t) return set_error(CUDASP_ERR_INVALID_ARG, "null device buffer");
  if (n > s->capacity) return set_error(CUDASP_ERR_CAPACITY, "batch of %u rows exceeds scanner capacity %u", n, s->capacity);
  DeviceGuard g(s->device);
  const int brc = ensure_stage_buffers(s);
  if (brc != CUDASP_OK) return brc;
  hipStream_t st = scanner_stream(s, stream);
  launch_a(s, d_tweak_x, d_tweak_y, n, d_t, st);
  HIP_TRY(hipGetLastError());
  return CUDASP_OK;
}

int cudasp_stage_match_device(cudasp_scanner* s, const uint32_t* d_t, const int64_t* d_outputs,
                              const uint32_t* d_output_offsets, const uint32_t* d_output_lengths, uint32_t n,
                              uint8_t* d_match_flags, uint32_t* d_match_rows, uint32_t* d_match_count, void* stream) {
  if (!s) return set_error(CUDASP_ERR_INVALID_ARG, "null scanner");
  if (n == 0) return CUDASP_OK;
  if (!d_t || !d_output_offsets || !d_output_lengths || !d_match_flags)
    return set_error(CUDASP_ERR_INVALID_ARG, "null device buffer");
  if (n > s->capacity) return set_error(CUDASP_ERR_CAPACITY, "batch of %u rows exceeds scanner capacity %u", n, s->capacity);
  DeviceGuard g(s->device);
  const int brc = ensure_stage_buffers(s);
  if (brc != CUDASP_OK) return brc;
  hipStream_t st = scanner_stream(s, stream);
  bool compact = d_match_rows && d_match_count;
  return launch_match(s, d_t, n, d_outputs, d_output_offsets, d_output_lengths, d_match_flags,
                      compact ? d_match_rows : nullptr, compact ? d_match_count : nullptr, nullptr, st);
}

int cudasp_synth_tweak_columns(int device, const uint8_t s0_le[32], uint64_t first_index, uint32_t n,
                               uint32_t* d_x, uint32_t* d_y, void* stream) {
  if (n == 0) return CUDASP_OK;
  if (!s0_le || !d_x || !d_y) return set_error(CUDASP_ERR_INVALID_ARG, "null argument");
  DeviceGuard g(device);
  const uint32_t* fb = nullptr;
  const int bits = default_fb_bits();
  int rc = ensure_device_table(device, bits, &fb);
  if (rc != CUDASP_OK) return rc;
  SynthConsts c;
  host::Big<8> s0 = host::big_zero<8>();
  for (int i = 0; i < 32; i++) s0.w[i / 4] |= (uint32_t)s0_le[i] << (8 * (i % 4));
  s0 = host::scalar_reduce(s0);
  for (int i = 0; i < 8; i++) c.s0[i] = s0.w[i];
  hipLaunchKernelGGL(bits == 26 ? k_synth_tweaks<26> : k_synth_tweaks<22>, dim3(grid_for(n)), dim3(BLOCK), 0,
                     plain_stream(stream), c, first_index, n, fb, d_x, d_y);
  HIP_TRY(hipGetLastError());
  return CUDASP_OK;
}

int cudasp_synth_outputs(uint64_t seed, uint64_t first_index, uint32_t n, uint32_t k, int64_t* d_outputs,
                         uint32_t* d_offsets, uint32_t* d_lengths, void* stream) {
  if (n == 0) return CUDASP_OK;
  if (!d_outputs || !d_offsets || !d_lengths) return set_error(CUDASP_ERR_INVALID_ARG, "null device buffer");
  hipLaunchKernelGGL(k_synth_outputs, dim3(grid_for(n)), dim3(BLOCK), 0, plain_stream(stream), seed, first_index, n,
                     k, d_outputs, d_offsets, d_lengths);
  HIP_TRY(hipGetLastError());
  return CUDASP_OK;
}

int cudasp_synth_output_lengths(uint64_t seed, uint64_t first_index, uint32_t n, uint32_t kmax, uint32_t* d_lengths,
                                void* stream) {
  if (n == 0) return CUDASP_OK;
  if (!d_lengths || kmax == 0) return set_error(CUDASP_ERR_INVALID_ARG, "invalid argument");
  hipLaunchKernelGGL(k_synth_output_lengths, dim3(grid_for(n)), dim3(BLOCK), 0, plain_stream(stream), seed,
                     first_index, n, kmax, d_lengths);
  HIP_TRY(hipGetLastError());
  return CUDASP_OK;
}

int cudasp_synth_output_values(uint64_t seed, uint64_t first_index, uint32_t n, const uint32_t* d_offsets,
                               const uint32_t* d_lengths, int64_t* d_outputs, void* stream) {
  if (n == 0) return CUDASP_OK;
  if (!d_offsets || !d_lengths || !d_outputs) return set_error(CUDASP_ERR_INVALID_ARG, "null device buffer");
  hipLaunchKernelGGL(k_synth_output_values, dim3(grid_for(n)), dim3(BLOCK), 0, plain_stream(stream), seed,
                     first_index, n, d_offsets, d_lengths, d_outputs);
  HIP_TRY(hipGetLastError());
  return CUDASP_OK;
}

int cudasp_field_layout(int* limbs, int* bits, int* mul_mag_max, int* sqr_mag_max, int* limb_mag_max) {
  if (!limbs || !bits || !mul_mag_max || !sqr_mag_max || !limb_mag_max)
    return set_error(CUDASP_ERR_INVALID_ARG, "null argument");
  *limbs = FE_LIMBS;
  *bits = FE_BITS;
  *mul_mag_max = (int)MUL_MAG_MAX;
  *sqr_mag_max = (int)SQR_MAG_MAX;
  *limb_mag_max = (int)LIMB_MAG_MAX;
  return CUDASP_OK;
}

int cudasp_debug_field_ops(int op, const uint32_t* d_a, const uint32_t* d_b, uint32_t* d_out, uint32_t n) {
  if (n == 0) return CUDASP_OK;
  if (op < 0 || op > 7 || (op >= 2 && op <= 6 && CUDASP_FE_LIMBS != 9))
    return set_error(CUDASP_ERR_INVALID_ARG,
                     "op must be 0 (mul), 1 (sqr), 7 (inverse), or 2..6 (fused, 9 x 29 layout)");
  if (!d_a || !d_b || !d_out) return set_error(CUDASP_ERR_INVALID_ARG, "null device buffer");
  hipLaunchKernelGGL(k_debug_field_ops, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, 0, op, d_a, d_b, d_out, n);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipDeviceSynchronize());
  return CUDASP_OK;
}

// ----------------------------------------------------------- streaming scan
// cudasp_stream_*: one persistent k_scan_stream kernel scans batches as the
// host publishes them (scan_stream.hpp).

// Coherent pinned allocations of cudasp_host_alloc, by start address: a
// published batch's host buffers must lie inside them.  The protocol needs
// it: the kernel reads the buffers with uncached (MTYPE UC) loads and writes
// its results with system-scope stores that the host sees without any cache
// maintenance, which holds for coherent host memory only (a non-coherent
// pinned buffer would let results sit in a device cache).
static std::mutex g_host_alloc_mu;
static std::map<uintptr_t, size_t> g_host_allocs;

static bool host_range_coherent(const void* p, size_t bytes) {
#ifdef CUDASP_AB_STREAM_ANY_MEMORY
  // measurement-only builds (tools/stream_probe.py --device-inputs): batch
  // buffers in device memory, to price the zero-copy PCIe reads
  return p != nullptr || bytes == 0;
#endif
  if (!p) return false;
  const uintptr_t a = (uintptr_t)p;
  std::lock_guard<std::mutex> lk(g_host_alloc_mu);
  auto it = g_host_allocs.upper_bound(a);
  if (it == g_host_allocs.begin()) return false;
  --it;
  return a >= it->first && a + bytes <= it->first + it->second;
}

constexpr uint32_t STREAM_MAX_WAVES = MAX_BLOCKS * (BLOCK / 64);

struct cudasp_stream {
  cudasp_scanner* s = nullptr;
  StreamCtrl* ctrl = nullptr;  // coherent pinned host memory (same address on the device)
  StreamDev* dev = nullptr;    // device memory
  unsigned long long* wstat = nullptr;    // device: STREAM_WSTAT counters per wave slot of the grid
  unsigned long long* h_counts = nullptr;  // pinned: StreamDev::stat, then the per-wave counters (finish copies)
  uint64_t blocks_req = 0;  // requested grid (0: the whole device)
  uint64_t blocks = 0;      // the current query's grid
  uint32_t rmax = MULTI_RMAX;
  uint64_t idle_ticks = 0;  // 100 MHz wall-clock ticks with nothing to do before the kernel leaves
  uint64_t prio_ticks = 0;  // wave priority step by piece age (stream_prio; 0: off)
  uint32_t pf_coal = 1;     // row blobs read lane-contiguously + LDS transpose (stream_prefetch)
  uint32_t timeout_ms = 0;  // waits fail after this long without progress (cudasp_stream_set_timeout)
  hipEvent_t exited = nullptr;
  bool running = false;     // a kernel was launched and `exited` recorded after it
  bool failed = false;      // a kernel of this query failed or a wait timed out (sticky until finish)
  bool abandoned = false;   // finish timed out with the kernel alive: nothing may be freed
  bool counts_pending = false;      // finish queued the counters' copy; counters() waits for it
  uint64_t counts_waves = 0;        // wave slots of the last finished query's grid
  uint32_t next = 0;        // batches published
  uint64_t published_wr = 0;
  uint64_t launches = 0;
  unsigned long long last_stat[16] = {};  // the kernel's counters of the last finished query
  std::mutex mu;            // publish / launch / finish
};

// Caller holds st->mu.  Whether the query's kernel is still running.  One
// that ended before the stream was closed left idle (or failed: sticky).
static bool stream_kernel_alive(cudasp_stream* st, int* err) {
  *err = CUDASP_OK;
  if (!st->running) return false;
  const hipError_t e = hipEventQuery(st->exited);
  if (e == hipErrorNotReady) return true;
  st->running = false;
  if (e != hipSuccess) {
    st->failed = true;
    *err = set_error(CUDASP_ERR_HIP, "streaming scan kernel failed: %s", hipGetErrorString(e));
  }
  return false;
}

// Before every launch (same stream; a relaunch follows the idle kernel's
// end): the claim counter back to the rows mirrored so far -- claims past
// them were never processed (the idle kernel's pub_wr was final) -- and
// `idle` cleared.  Each worker's first ticket is one wave-row, worker w's at
// first_wr + w, and the counter starts past them: the grid's ~3k first
// claims would otherwise be same-address atomics that the L2 serializes
// (~45 ns each, ~150 us before the last wave starts, profiles/r04_*).
__global__ void k_stream_start(StreamDev* dev, uint32_t workers) {
  if (threadIdx.x == 0) {
    const uint64_t w0 = dev->pub_wr;
    dev->first_wr = w0;
    dev->ticket = w0 + workers;
    dev->idle = 0;
  }
}

// Caller holds st->mu.  Launch a kernel for the query: at its first batch,
// or again after the previous one left idle (the device state -- claim
// counter, mirrored descriptors, per-batch counts -- carries over; only
// `idle` is cleared).  Uses the scanner's current keys and options (a host
// may rebind the scanner between queries: the grid and its scratch follow
// the label count).
static int stream_launch(cudasp_stream* st) {
  cudasp_scanner* s = st->s;
  DeviceGuard g(s->device);
  if (!stream_ok(s))
    return set_error(CUDASP_ERR_INVALID_ARG, "the scanner's options do not allow the streaming scan");
  st->blocks = stream_grid_blocks(s, st->blocks_req);
  if (st->blocks < 2) return set_error(CUDASP_ERR_INVALID_ARG, "too many label keys for the streaming scan");
  {
    const int rc = ensure_stream_scratch(s, st->blocks, s->stream);
    if (rc != CUDASP_OK) return rc;
  }
  const uint32_t K = s->consts.output_count;
  const uint32_t rmax = std::max(1u, std::min(st->rmax, (uint32_t)MULTI_RMAX / K));
  hipLaunchKernelGGL(k_stream_start, dim3(1), dim3(64), 0, s->stream, st->dev,
                     (uint32_t)st->blocks * (BLOCK / 64u) - 1u);  // every wave but the poller
  const bool wide = K > (uint32_t)MULTI_RMAX;
  auto kf = s->fb_bits == 26 ? (wide ? k_scan_stream<26, true> : k_scan_stream<26, false>)
                             : (wide ? k_scan_stream<22, true> : k_scan_stream<22, false>);
  hipLaunchKernelGGL(kf, dim3((uint32_t)st->blocks), dim3(BLOCK), 0, s->stream, st->ctrl, st->dev, s->d_naf,
                     s->consts, s->d_fb, s->d_labels, s->d_mscratch, rmax, st->idle_ticks, st->wstat, st->prio_ticks, st->pf_coal);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(st->exited, s->stream));
  ST_HOST(102, st->blocks, (uint32_t)st->launches);
  st->running = true;
  st->launches++;
  return CUDASP_OK;
}

// Caller holds st->mu.  A kernel runs for the published batches: relaunched
// if the last one left idle.
static int stream_ensure_running(cudasp_stream* st) {
  int err;
  if (stream_kernel_alive(st, &err)) return CUDASP_OK;
  if (err != CUDASP_OK) return err;
  if (st->failed) return set_error(CUDASP_ERR_HIP, "streaming scan kernel failed earlier in this query");
  return stream_launch(st);
}

static bool stream_seq_done(const cudasp_stream* st, uint64_t seq) {
  const uint32_t d = __atomic_load_n(&st->ctrl->done[seq % STREAM_RING], __ATOMIC_ACQUIRE);
  return (int32_t)(d - (uint32_t)(seq + 1)) >= 0;
}

// A fingerprint of the kernel's visible progress: the done words of the ring
// (a completed batch changes one) -- what a wait's no-progress deadline
// watches.
static uint64_t stream_progress(const cudasp_stream* st) {
  uint64_t h = 0;
  for (uint32_t e = 0; e < STREAM_RING; e++)
    h = h * 1000003ull + __atomic_load_n(&st->ctrl->done[e], __ATOMIC_ACQUIRE);
  return h;
}

int cudasp_host_alloc(void** p, size_t bytes) {
  if (!p) return set_error(CUDASP_ERR_INVALID_ARG, "null pointer");
  *p = nullptr;
  if (bytes == 0) return CUDASP_OK;
  void* q = nullptr;
  HIP_TRY(hipHostMalloc(&q, bytes, hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable));
  void* dq = nullptr;
  if (hipHostGetDevicePointer(&dq, q, 0) != hipSuccess || dq != q) {
    (void)hipHostFree(q);
    return set_error(CUDASP_ERR_HIP, "pinned host memory is not device-addressable at its host address");
  }
  {
    std::lock_guard<std::mutex> lk(g_host_alloc_mu);
    g_host_allocs[(uintptr_t)q] = bytes;
  }
  *p = q;
  return CUDASP_OK;
}

void cudasp_host_free(void* p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> lk(g_host_alloc_mu);
    g_host_allocs.erase((uintptr_t)p);
  }
  (void)hipHostFree(p);
}

int cudasp_stream_supported(const cudasp_scanner* s) {
  if (!s || !stream_ok(s)) return 0;
  return stream_grid_blocks(const_cast<cudasp_scanner*>(s), 0) >= 2 ? 1 : 0;
}

int cudasp_stream_create(cudasp_scanner* s, uint32_t blocks, cudasp_stream** out) {
  if (!s || !out) return set_error(CUDASP_ERR_INVALID_ARG, "null argument");
  *out = nullptr;
  if (!stream_ok(s))
    return set_error(CUDASP_ERR_INVALID_ARG,
                     "the streaming scan needs an HBM fixed-base width (22 or 26 bits), the pipelined schedule and "
                     "a label count whose scratch fits");
  DeviceGuard g(s->device);
  std::unique_ptr<cudasp_stream> st(new cudasp_stream());
  st->s = s;
  st->blocks_req = blocks;
  st->blocks = stream_grid_blocks(s, blocks);
  if (st->blocks < 2) return set_error(CUDASP_ERR_INVALID_ARG, "too many label keys for the streaming scan");
  uint32_t idle_ms = 20;
  if (const char* e = getenv("CUDASP_STREAM_IDLE_MS")) {
    const long v = atol(e);
    if (v >= 1 && v <= 600000) idle_ms = (uint32_t)v;
  }
  st->idle_ticks = (uint64_t)idle_ms * 100000ull;
  // wave priority by piece age, one level per 3 ms (round 4, config 3 end to
  // end: 148.7 / 150.7 M tx/s without, 158.2 / 162.5 with; config 4 172.4 vs
  // 173.9, config 2 even; profiles/r04_stream_prio_ab.txt); 0 turns it off
  uint32_t prio_us = 3000;
  if (const char* e = getenv("CUDASP_STREAM_PRIO_US")) {
    const long v = atol(e);
    if (v >= 0 && v <= 1000000) prio_us = (uint32_t)v;
  }
  st->prio_ticks = (uint64_t)prio_us * 100ull;
  if (const char* e = getenv("CUDASP_STREAM_PF_COAL")) st->pf_coal = atoi(e) != 0 ? 1u : 0u;
  st->timeout_ms = 60000;
  if (const char* e = getenv("CUDASP_STREAM_TIMEOUT_MS")) {
    const long v = atol(e);
    if (v >= 1 && v <= 86400000) st->timeout_ms = (uint32_t)v;
  }
  if (const char* e = getenv("CUDASP_MULTI_ROWS")) {
    const int v = atoi(e);
    if (v >= 1 && v <= MULTI_RMAX) st->rmax = (uint32_t)v;
  }
  int rc = ensure_stream_scratch(s, st->blocks, s->stream);
  if (rc != CUDASP_OK) return rc;
  void* c = nullptr;
  rc = cudasp_host_alloc(&c, sizeof(StreamCtrl));
  if (rc != CUDASP_OK) return rc;
  st->ctrl = static_cast<StreamCtrl*>(c);
  memset(st->ctrl, 0, sizeof(StreamCtrl));
  const size_t wbytes = (size_t)STREAM_MAX_WAVES * STREAM_WSTAT * sizeof(unsigned long long);
  if (hipMalloc(&st->dev, sizeof(StreamDev)) != hipSuccess || hipMalloc(&st->wstat, wbytes) != hipSuccess ||
      hipHostMalloc(&st->h_counts, 16 * sizeof(unsigned long long) + wbytes, hipHostMallocDefault) != hipSuccess ||
      hipEventCreateWithFlags(&st->exited, hipEventDisableTiming) != hipSuccess ||
      hipMemsetAsync(st->dev, 0, sizeof(StreamDev), s->stream) != hipSuccess ||
      hipMemsetAsync(st->wstat, 0, wbytes, s->stream) != hipSuccess || hipStreamSynchronize(s->stream) != hipSuccess) {
    cudasp_stream_destroy(st.release());
    return set_error(CUDASP_ERR_HIP, "streaming scan: device state allocation failed");
  }
  *out = st.release();
  return CUDASP_OK;
}

int cudasp_stream_publish_batch(cudasp_stream* st, const cudasp_stream_batch* bt, uint64_t* seq) {
  if (!st || !bt) return set_error(CUDASP_ERR_INVALID_ARG, "null argument");
  const uint32_t n = bt->n;
  if (n == 0 || !bt->tweak_keys || !bt->output_offsets || !bt->d_mirror)
    return set_error(CUDASP_ERR_INVALID_ARG, "empty batch or null buffer (the outputs mirror included)");
  // no lengths: the offsets are Arrow list offsets, n + 1 of them
  const size_t noffs = bt->output_lengths ? n : (size_t)n + 1;
  if (!bt->match_flags && !bt->match_rows)
    return set_error(CUDASP_ERR_INVALID_ARG, "a streamed batch needs match_flags and/or match_rows");
  // every host buffer the kernel touches must be coherent pinned memory
  // (cudasp_host_alloc), inputs and results; the outputs list is checked at
  // its start (its rows' offsets and lengths, like every CSR this library
  // takes, are the caller's)
  if ((bt->match_flags && !host_range_coherent(bt->match_flags, n)) ||
      (bt->match_rows && !host_range_coherent(bt->match_rows, (size_t)n * 4)) ||
      !host_range_coherent(bt->output_offsets, noffs * 4) ||
      (bt->output_lengths && !host_range_coherent(bt->output_lengths, (size_t)n * 4)) ||
      !host_range_coherent(bt->tweak_keys, (size_t)n * 64) || (bt->outputs && !host_range_coherent(bt->outputs, 8)))
    return set_error(CUDASP_ERR_INVALID_ARG, "streamed batch buffers must come from cudasp_host_alloc");
  std::lock_guard<std::mutex> lk(st->mu);
  if (st->ctrl->closed) return set_error(CUDASP_ERR_INVALID_ARG, "stream already closed");
  if (st->failed) return set_error(CUDASP_ERR_HIP, "streaming scan kernel failed earlier in this query");
  const uint32_t b = st->next;
  const uint32_t e = b % STREAM_RING;
  if (b >= STREAM_RING && !stream_seq_done(st, (uint64_t)b - STREAM_RING))
    return set_error(CUDASP_ERR_CAPACITY, "more than %u streamed batches in flight", STREAM_RING);
  StreamBatch& d = st->ctrl->desc[e];
  d.rows = bt->tweak_keys;
  d.outputs = bt->outputs;
  d.offs = bt->output_offsets;
  d.lens = bt->output_lengths;
  d.flags = bt->match_flags;
  d.matches = bt->match_rows;
  d.mirror = bt->d_mirror;
  d.n = n;
  d.nwr = (n + 63u) / 64u;
  d.reserved0 = 0;
  d.reserved1 = 0;
  d.first_wr = st->published_wr;
  d.seq = b;
  st->published_wr += d.nwr;
  __atomic_store_n(&st->ctrl->published_wr, st->published_wr, __ATOMIC_RELEASE);
  __atomic_store_n(&st->ctrl->published, b + 1, __ATOMIC_RELEASE);
  st->next = b + 1;
  if (seq) *seq = b;
  ST_HOST(101, n, b);
  // the query's kernel: launched at its first batch, relaunched if it left
  // idle (its poller picks the batch up from the control block either way)
  return stream_ensure_running(st);
}

int cudasp_stream_publish(cudasp_stream* st, const uint8_t* rows, const int64_t* outputs, const uint32_t* offs,
                          const uint32_t* lens, uint32_t n, uint8_t* flags, int64_t* d_mirror, uint64_t* seq) {
  cudasp_stream_batch b{};
  b.tweak_keys = rows;
  b.outputs = outputs;
  b.output_offsets = offs;
  b.output_lengths = lens;
  b.n = n;
  b.match_flags = flags;
  b.match_rows = nullptr;
  b.d_mirror = d_mirror;
  if (!flags) return set_error(CUDASP_ERR_INVALID_ARG, "null flags buffer");
  return cudasp_stream_publish_batch(st, &b, seq);
}

int cudasp_stream_close(cudasp_stream* st) {
  if (!st) return set_error(CUDASP_ERR_INVALID_ARG, "null stream");
  std::lock_guard<std::mutex> lk(st->mu);
  __atomic_store_n(&st->ctrl->closed, 1u, __ATOMIC_RELEASE);
  ST_HOST(103, 0, 0);
  return CUDASP_OK;
}

int cudasp_stream_query(cudasp_stream* st, uint64_t seq) {
  if (!st) return set_error(CUDASP_ERR_INVALID_ARG, "null stream");
  if (stream_seq_done(st, seq)) return 1;
  std::lock_guard<std::mutex> lk(st->mu);
  if (seq >= st->next) return set_error(CUDASP_ERR_INVALID_ARG, "batch %llu was not published", (unsigned long long)seq);
  if (stream_seq_done(st, seq)) return 1;
  // not done: a kernel must be running for it (one that left idle while
  // the batch was being published is relaunched here)
  const int rc = stream_ensure_running(st);
  if (rc != CUDASP_OK) return rc;
  return stream_seq_done(st, seq) ? 1 : 0;
}

// Spin (yield) for the first 2 ms, then sleep in short steps: a batch's
// completion is noticed within microseconds while it is close (the end of a
// query waits for its last batches), and a long wait costs no core.  Fails
// after timeout_ms without progress (no batch of the stream completed).
int cudasp_stream_wait(cudasp_stream* st, uint64_t seq) {
  if (!st) return set_error(CUDASP_ERR_INVALID_ARG, "null stream");
  const auto t0 = std::chrono::steady_clock::now();
  auto t_prog = t0, t_check = t0;
  uint64_t prog = stream_progress(st);
  for (;;) {
    const int q = cudasp_stream_query(st, seq);
    if (q != 0) return q < 0 ? q : CUDASP_OK;
    const auto now = std::chrono::steady_clock::now();
    if (now - t_check > std::chrono::microseconds(100)) {
      t_check = now;
      const uint64_t p = stream_progress(st);
      if (p != prog) {
        prog = p;
        t_prog = now;
      } else if (now - t_prog > std::chrono::milliseconds(st->timeout_ms)) {
        std::lock_guard<std::mutex> lk(st->mu);
        st->failed = true;
        return set_error(CUDASP_ERR_HIP,
                         "streaming scan: batch %llu not done after %u ms without progress (batches published %u, "
                         "kernel launches %llu, running %d)",
                         (unsigned long long)seq, st->timeout_ms, st->next, (unsigned long long)st->launches,
                         (int)st->running);
      }
    }
    if (now - t0 < std::chrono::milliseconds(2))
      std::this_thread::yield();
    else
      std::this_thread::sleep_for(std::chrono::microseconds(10));
  }
}

int cudasp_stream_set_timeout(cudasp_stream* st, uint32_t ms) {
  if (!st || ms == 0) return set_error(CUDASP_ERR_INVALID_ARG, "null stream or zero timeout");
  std::lock_guard<std::mutex> lk(st->mu);
  st->timeout_ms = ms;
  return CUDASP_OK;
}

int cudasp_stream_matches(cudasp_stream* st, uint64_t seq, uint32_t* count) {
  if (!st || !count) return set_error(CUDASP_ERR_INVALID_ARG, "null argument");
  if (seq >= st->next || st->next - seq > STREAM_RING || !stream_seq_done(st, seq))
    return set_error(CUDASP_ERR_INVALID_ARG, "batch %llu is not a done batch of the last %u", (unsigned long long)seq,
                     STREAM_RING);
  *count = __atomic_load_n(&st->ctrl->nmatch[seq % STREAM_RING], __ATOMIC_ACQUIRE);
  return CUDASP_OK;
}

#if CUDASP_STREAM_TRACE
// Caller holds st->mu, the query's kernels have ended: append the query's
// events to $CUDASP_STREAM_TRACE_FILE (u32 count, then the events) and reset.
static void stream_trace_dump(cudasp_stream* st) {
  uint32_t n = 0;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(g_st_n), sizeof(n)) != hipSuccess) return;
  if (n > STREAM_TRACE_CAP) n = STREAM_TRACE_CAP;
  std::vector<StreamTraceEv> ev(n);
  if (n && hipMemcpyFromSymbol(ev.data(), HIP_SYMBOL(g_st_ev), n * sizeof(StreamTraceEv)) != hipSuccess) return;
  const uint32_t zero = 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_st_n), &zero, sizeof(zero));
  {
    std::lock_guard<std::mutex> lk(g_st_host_mu);
    ev.insert(ev.end(), g_st_host.begin(), g_st_host.end());
    g_st_host.clear();
  }
  n = (uint32_t)ev.size();
  const char* path = getenv("CUDASP_STREAM_TRACE_FILE");
  if (!path || !n) return;
  if (FILE* f = fopen(path, "ab")) {
    fwrite(&n, sizeof(n), 1, f);
    fwrite(ev.data(), sizeof(StreamTraceEv), n, f);
    fclose(f);
  }
  (void)st;
}
#endif

int cudasp_stream_finish(cudasp_stream* st) {
  if (!st) return set_error(CUDASP_ERR_INVALID_ARG, "null stream");
  if (st->abandoned) return set_error(CUDASP_ERR_HIP, "streaming scan abandoned after a timeout");
  int rc = CUDASP_OK;
  {
    std::lock_guard<std::mutex> lk(st->mu);
    if (!st->ctrl->closed) {
      __atomic_store_n(&st->ctrl->closed, 1u, __ATOMIC_RELEASE);
      ST_HOST(103, 0, 0);
    }
  }
  const bool had_failed = st->failed;
  if (st->next > 0) rc = cudasp_stream_wait(st, (uint64_t)st->next - 1);
  for (uint64_t b = st->next > STREAM_RING ? st->next - STREAM_RING : 0; rc == CUDASP_OK && b < st->next; b++)
    rc = cudasp_stream_wait(st, b);
  if (had_failed && rc != CUDASP_OK) {
    // a wait of this query timed out: the batches may still complete (a
    // slow kernel), so give them the deadline once more from here
    st->failed = false;
    rc = CUDASP_OK;
    for (uint64_t b = st->next > STREAM_RING ? st->next - STREAM_RING : 0; rc == CUDASP_OK && b < st->next; b++)
      rc = cudasp_stream_wait(st, b);
  }
  ST_HOST(104, 0, 0);
  std::lock_guard<std::mutex> lk(st->mu);
  DeviceGuard g(st->s->device);
  if (st->running) {
    // its waves leave as soon as they see the closed stream drained (or
    // idle); bounded like the waits: a kernel that never ends is abandoned
    // (the caller must then leak everything it may still touch)
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e;
    while ((e = hipEventQuery(st->exited)) == hipErrorNotReady) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(st->timeout_ms)) {
        st->abandoned = true;
        return set_error(CUDASP_ERR_HIP, "streaming scan kernel still running %u ms after the stream was closed",
                         st->timeout_ms);
      }
      std::this_thread::sleep_for(std::chrono::microseconds(5));
    }
    st->running = false;
    if (e != hipSuccess && rc == CUDASP_OK)
      rc = set_error(CUDASP_ERR_HIP, "streaming scan kernel failed: %s", hipGetErrorString(e));
  }
  ST_HOST(105, 0, 0);
  if (rc != CUDASP_OK && !st->running && st->next > 0) {
    // the kernel has ended without finishing every batch (it failed): the
    // query's error stands; the stream is reset below for the next query
  }
  st->failed = false;
  // Ready for the next query: the control block here, the device state and
  // the counters' copy queued on the scanner's stream (ordered before its
  // next launch; cudasp_stream_counters waits for the copy).
  const bool ran = st->next > 0;
  memset(st->ctrl, 0, sizeof(StreamCtrl));
  st->next = 0;
  st->published_wr = 0;
  const uint64_t waves = st->blocks * (BLOCK / 64);
  const size_t wbytes = (size_t)waves * STREAM_WSTAT * sizeof(unsigned long long);
  if (ran) {
    if (hipMemcpyAsync(st->h_counts, st->dev->stat, 16 * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                       st->s->stream) != hipSuccess ||
        hipMemcpyAsync(st->h_counts + 16, st->wstat, wbytes, hipMemcpyDeviceToHost, st->s->stream) != hipSuccess ||
        hipMemsetAsync(st->wstat, 0, wbytes, st->s->stream) != hipSuccess) {
      if (rc == CUDASP_OK) rc = set_error(CUDASP_ERR_HIP, "streaming scan: counters copy failed");
    }
    st->counts_pending = true;
    st->counts_waves = waves;
  }
  if (hipMemsetAsync(st->dev, 0, sizeof(StreamDev), st->s->stream) != hipSuccess && rc == CUDASP_OK)
    rc = set_error(CUDASP_ERR_HIP, "streaming scan: state reset failed");
  ST_HOST(106, 0, 0);
#if CUDASP_STREAM_TRACE
  stream_trace_dump(st);
#endif
  return rc;
}

int cudasp_stream_stats(const cudasp_stream* st, uint64_t* launches, uint32_t* blocks) {
  if (!st) return set_error(CUDASP_ERR_INVALID_ARG, "null stream");
  if (launches) *launches = st->launches;
  if (blocks) *blocks = (uint32_t)st->blocks;
  return CUDASP_OK;
}

int cudasp_stream_counters(cudasp_stream* st, uint64_t* out, uint32_t count) {
  if (!st || !out) return set_error(CUDASP_ERR_INVALID_ARG, "null argument");
  std::lock_guard<std::mutex> lk(st->mu);
  if (st->counts_pending) {
    DeviceGuard g(st->s->device);
    HIP_TRY(hipStreamSynchronize(st->s->stream));
    for (int i = 0; i < 16; i++) st->last_stat[i] = st->h_counts[i];
    // per-wave counters: pieces, wave-rows, polls, drains, (0), exits, busy, life
    static const int map[STREAM_WSTAT] = {STREAM_STAT_PIECES,       STREAM_STAT_WAVE_ROWS, STREAM_STAT_WAIT_POLLS,
                                          STREAM_STAT_DRAINS,       STREAM_STAT_RESERVED,  STREAM_STAT_WORKER_EXITS,
                                          STREAM_STAT_BUSY_TICKS,   STREAM_STAT_LIFE_TICKS};
    const unsigned long long* w = st->h_counts + 16;
    for (uint64_t v = 0; v < st->counts_waves; v++)
      for (uint32_t i = 0; i < STREAM_WSTAT; i++) st->last_stat[map[i]] += w[v * STREAM_WSTAT + i];
    st->counts_pending = false;
  }
  for (uint32_t i = 0; i < count && i < 16; i++) out[i] = st->last_stat[i];
  return CUDASP_OK;
}

int cudasp_stream_abandoned(const cudasp_stream* st) { return st && st->abandoned ? 1 : 0; }

void cudasp_stream_destroy(cudasp_stream* st) {
  if (!st) return;
  if (st->ctrl && !st->abandoned) (void)cudasp_stream_finish(st);
  if (st->abandoned) {
    // a kernel may still read the control block and write the device state:
    // leak them (and the caller leaks the scanner and the batch buffers)
    fprintf(stderr, "cudasp: a streaming scan kernel did not end; its buffers are leaked\n");
    delete st;
    return;
  }
  if (st->ctrl) cudasp_host_free(st->ctrl);
  DeviceGuard g(st->s->device);
  if (st->s->stream) (void)hipStreamSynchronize(st->s->stream);
  if (st->dev) (void)hipFree(st->dev);
  if (st->wstat) (void)hipFree(st->wstat);
  if (st->h_counts) (void)hipHostFree(st->h_counts);
  if (st->exited) (void)hipEventDestroy(st->exited);
  delete st;
}

// ------------------------------------------------ reference three-phase ABI
struct LegacyBatch {
  cudasp_scanner* scanner = nullptr;
  int64_t* d_outputs = nullptr;
  uint32_t* d_offs = nullptr;
  uint32_t* d_lens = nullptr;
  uint32_t* d_tx = nullptr;
  uint32_t* d_ty = nullptr;
  uint8_t* d_flags = nullptr;
  uint32_t count = 0;
};

static void words_to_bytes(uint8_t* out, const uint32_t* w, int nwords) {
  for (int i = 0; i < nwords; i++) {
    out[4 * i] = (uint8_t)w[i];
    out[4 * i + 1] = (uint8_t)(w[i] >> 8);
    out[4 * i + 2] = (uint8_t)(w[i] >> 16);
    out[4 * i + 3] = (uint8_t)(w[i] >> 24);
  }
}

static void free_legacy(LegacyBatch* b) {
  if (!b) return;
  if (b->scanner) {
    DeviceGuard g(b->scanner->device);
    (void)hipStreamSynchronize(b->scanner->stream);
    void* ptrs[] = {b->d_outputs, b->d_offs, b->d_lens, b->d_tx, b->d_ty, b->d_flags};
    for (void* p : ptrs)
      if (p) (void)hipFree(p);
    free_scanner(b->scanner);
  }
  delete b;
}

void* LaunchBatchScan(uint32_t** managed_points_x, uint32_t** managed_points_y, const uint32_t* h_scalar,
                      const uint32_t* h_spend_pubkey_x, const uint32_t* h_spend_pubkey_y,
                      const uint32_t* h_label_keys_x, const uint32_t* h_label_keys_y, uint32_t label_count,
                      const int64_t* h_outputs, const uint32_t* h_output_offsets,
                      const uint32_t* h_output_lengths, uint8_t** managed_match_flags, uint32_t count,
                      size_t outputs_size) {
  if (!managed_points_x || !managed_points_y || !managed_match_flags || !h_scalar || !h_spend_pubkey_x ||
      !h_spend_pubkey_y || !h_output_offsets || !h_output_lengths || count == 0) {
    set_error(CUDASP_ERR_INVALID_ARG, "LaunchBatchScan: invalid argument");
    return nullptr;
  }
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess) {
    set_error(CUDASP_ERR_HIP, "hipGetDevice failed");
    return nullptr;
  }
  uint8_t scan[32], spend[64];
  words_to_bytes(scan, h_scalar, 8);
  words_to_bytes(spend, h_spend_pubkey_x, 8);
  words_to_bytes(spend + 32, h_spend_pubkey_y, 8);
  std::vector<uint8_t> labels(64 * (size_t)label_count);
  for (uint32_t j = 0; j < label_count; j++) {
    words_to_bytes(&labels[64 * j], h_label_keys_x + 8 * j, 8);
    words_to_bytes(&labels[64 * j + 32], h_label_keys_y + 8 * j, 8);
  }
  LegacyBatch* b = new LegacyBatch();
  b->count = count;
  if (cudasp_scanner_create(device, scan, spend, labels.data(), label_count, count, &b->scanner) != CUDASP_OK) {
    delete b;
    return nullptr;
  }
  hipStream_t st = b->scanner->stream;
  bool ok = hipMallocManaged((void**)managed_points_x, (size_t)32 * count) == hipSuccess &&
            hipMallocManaged((void**)managed_points_y, (size_t)32 * count) == hipSuccess &&
            hipMallocManaged((void**)managed_match_flags, count) == hipSuccess &&
            hipMalloc(&b->d_outputs, (outputs_size ? outputs_size : 1) * 8) == hipSuccess &&
            hipMalloc(&b->d_offs, (size_t)4 * count) == hipSuccess &&
            hipMalloc(&b->d_lens, (size_t)4 * count) == hipSuccess &&
            hipMalloc(&b->d_tx, (size_t)32 * count) == hipSuccess &&
            hipMalloc(&b->d_ty, (size_t)32 * count) == hipSuccess &&
            hipMalloc(&b->d_flags, count) == hipSuccess;
  if (ok) {
    memset(*managed_match_flags, 0, count);
    ok = (outputs_size == 0 ||
          hipMemcpyAsync(b->d_outputs, h_outputs, outputs_size * 8, hipMemcpyHostToDevice, st) == hipSuccess) &&
         hipMemcpyAsync(b->d_offs, h_output_offsets, (size_t)4 * count, hipMemcpyHostToDevice, st) == hipSuccess &&
         hipMemcpyAsync(b->d_lens, h_output_lengths, (size_t)4 * count, hipMemcpyHostToDevice, st) == hipSuccess &&
         hipStreamSynchronize(st) == hipSuccess;
  }
  if (!ok) {
    set_error(CUDASP_ERR_HIP, "LaunchBatchScan: allocation or copy failed");
    free_legacy(b);
    return nullptr;
  }
  return b;
}

int RunBatchScanKernels(void* state_handle, uint32_t* managed_points_x, uint32_t* managed_points_y,
                        const uint32_t* /*h_scalar*/, const uint32_t* /*h_spend_pubkey_x*/,
                        const uint32_t* /*h_spend_pubkey_y*/, const uint32_t* /*h_label_keys_x*/,
                        const uint32_t* /*h_label_keys_y*/, uint32_t /*label_count*/, uint8_t* managed_match_flags,
                        uint32_t count) {
  // Like the reference, the keys were bound in LaunchBatchScan; the repeated
  // host key arguments are accepted and ignored (src/cudasp_gpu.cu:677-682).
  LegacyBatch* b = static_cast<LegacyBatch*>(state_handle);
  if (!b || !b->scanner || !managed_points_x || !managed_points_y || !managed_match_flags || count != b->count) {
    set_error(CUDASP_ERR_INVALID_ARG, "RunBatchScanKernels: invalid state or arguments");
    return -1;
  }
  DeviceGuard g(b->scanner->device);
  hipStream_t st = b->scanner->stream;
  if (hipMemcpyAsync(b->d_tx, managed_points_x, (size_t)32 * count, hipMemcpyDefault, st) != hipSuccess ||
      hipMemcpyAsync(b->d_ty, managed_points_y, (size_t)32 * count, hipMemcpyDefault, st) != hipSuccess) {
    set_error(CUDASP_ERR_HIP, "RunBatchScanKernels: point copy failed");
    return -1;
  }
  if (launch_pipeline(b->scanner, b->d_tx, b->d_ty, b->d_outputs, b->d_offs, b->d_lens, count, b->d_flags, nullptr,
                      nullptr, nullptr, nullptr, st) != CUDASP_OK)
    return -1;
  if (hipMemcpyAsync(managed_match_flags, b->d_flags, count, hipMemcpyDefault, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    set_error(CUDASP_ERR_HIP, "RunBatchScanKernels: kernel or flag copy failed");
    return -1;
  }
  return 0;
}

void FreeBatchScanState(void* state_handle) { free_legacy(static_cast<LegacyBatch*>(state_handle)); }

void FreeBatchScanManaged(void* ptr) {
  if (ptr) (void)hipFree(ptr);
}

}  // extern "C"
