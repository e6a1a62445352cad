// Streaming scan: ONE persistent kernel per device feed scans batches while
// the host is still reading the table (cudasp_stream_*, include/cudasp_abi.h).
//
// The per-batch host path (cudasp_tf_* before this) copied each closed slot
// to the device, transposed it, and launched one k_scan_multi per slot on
// 3 streams: every 300k-row launch ends in its own drain, the GPU holds at
// most 3 launches, and a table smaller than a few batches never fills it
// (end to end 0.92 / 0.88 / 0.62 of the device-resident rate at 32.7M /
// 9.4M / 1M rows).  Here the host publishes each closed slot into a
// descriptor ring in coherent pinned host memory and the kernel's waves take
// 64-row wave-rows from it as they are published:
//   * inputs are read straight from the pinned slot (zero copy over PCIe):
//     when a wave takes a piece of R wave-rows it first fetches all of them
//     -- the 64-byte row blobs into its scratch, offsets and lengths, and the
//     rows' outputs into the batch's device mirror, one cooperative copy per
//     batch of the piece -- so a piece pays a few PCIe latencies, not several
//     per row, and nothing after the prefetch reads host memory;
//   * results go straight back into the pinned slot: the matching rows'
//     indices (ballot compaction, one atomic per wave-row with a match) and/or
//     one flag per row; the wave that completes a batch (one device counter
//     per ring entry) writes the batch's match count and then, behind a
//     system-scope release, its sequence number into the ring's done word,
//     which the host polls;
//   * one poller wave per kernel reads the host's control block over PCIe
//     (published count, descriptors, closed) and mirrors it into device
//     memory; each worker wave's first ticket is one wave-row given by its
//     index, the later ones R wave-rows from one device counter (one
//     atomicAdd while published rows are unclaimed: concurrent claims may
//     pass the published rows, and such a ticket waits for the next batch);
//     a wave looks each wave-row's batch up in the mirror once, at the
//     prefetch (the piece's pointers then live in LDS);
//   * output_count K > 1 (K <= MULTI_RMAX): K hashes and K fixed-base points
//     per row, K x R <= MULTI_RMAX per piece, the row's flag the OR;
//   * the kernel is elastic: every wave leaves once the stream is closed and
//     drained, or once the poller has seen nothing to do for idle_ticks
//     (CUDASP_STREAM_IDLE_MS, 100 MHz wall clock; every published row
//     claimed, no new batch).  Rows past the mirrored pub_wr were never
//     processed, so the host's next publish or wait relaunches the kernel
//     with the claim counter reset to pub_wr (k_stream_start).  A host
//     that stalls (a slow source, or executor threads busy elsewhere) never
//     holds the GPU, and a host that never closes leaves no kernel spinning.
// Pieces and the pipelined schedule are k_scan_multi's (one inversion per
// piece).  A ticket may span two batches: every wave-row is looked up on its
// own.  This header holds the data structures and the pure scheduling rules
// (host + device; tests/test_stream_rules_cpu.py replays them and the ring
// lookup); the kernel is in scan_kernels.hip.
#pragma once
#include <stddef.h>
#include <stdint.h>

// The kernel's host/device ordering (the poller's write-through descriptor
// stores ordered by vmcnt waits, the done word behind a system-scope release)
// rests on gfx950's memory model and cache-policy bits, and
// tests/test_stream_isa_cpu.py checks the generated code for exactly that
// target: any other one must be re-verified before it is built.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "the streaming scan's ordering protocol is verified for gfx950 only (tests/test_stream_isa_cpu.py)"
#endif

#include "secp256k1_fe.hpp"  // CUDASP_HD

namespace cudasp {

// Batches published and not yet harvested, at most (the host's slot ring is
// far smaller: a streaming feed has 16 slots).
constexpr uint32_t STREAM_RING = 64;

// One published batch, written by the host before it bumps `published`.
// Pointers into coherent pinned host memory except `mirror` (device memory,
// outputs-sized; only read with labels).
struct StreamBatch {
  const uint8_t* rows;      // n x 64-byte tweak blobs (x then y, little-endian u32 words)
  const int64_t* outputs;   // outputs CSR values (words: 1 per output, 4 with full_x)
  const uint32_t* offs;     // n, in outputs
  const uint32_t* lens;     // n
  uint8_t* flags;           // n, written by the kernel (or null)
  uint32_t* matches;        // up to n matching row indices, written by the kernel (or null)
  int64_t* mirror;          // device copy of the outputs the compares read
  uint32_t n;
  uint32_t nwr;             // wave-rows: ceil(n / 64)
  uint32_t reserved0;
  uint32_t reserved1;
  uint64_t first_wr;        // wave-rows published before this batch
  uint64_t seq;             // the batch's sequence number (tells a reused ring entry)
};

// Host <-> kernel control block (coherent pinned host memory).
struct StreamCtrl {
  uint32_t published;               // batches published (host; release)
  uint32_t closed;                  // 1: no batch follows (host)
  uint64_t published_wr;            // wave-rows published (host)
  uint32_t reserved;
  uint32_t done[STREAM_RING];       // ring entry e: 1 + sequence number of the last batch completed there (kernel)
  uint32_t nmatch[STREAM_RING];     // matching rows of that batch (kernel; written before `done`)
  StreamBatch desc[STREAM_RING];    // batch b at entry b % STREAM_RING
};

// Device-side state (device memory), zeroed between queries.  The kernel's
// poller wave (one per kernel) mirrors the host's control block here --
// published batches, their descriptors, closed -- so the worker waves'
// claims and polls touch device memory only, never PCIe.
struct StreamDev {
  uint64_t ticket;                  // wave-rows handed out to the workers
  uint64_t first_wr;                // this launch's first wave-row: worker w's first ticket is
                                    // [first_wr + w, +1), handed out without an atomic (k_stream_start)
  uint64_t pub_wr;                  // mirror of StreamCtrl::published_wr
  uint32_t pub;                     // mirror of StreamCtrl::published
  uint32_t closed;                  // mirror of StreamCtrl::closed (set after the last pub)
  uint32_t idle;                    // the poller left idle: the workers leave as they drain
                                    // (reset by the host before it relaunches the kernel)
  uint32_t wr_done[STREAM_RING];    // wave-rows finished of the batch at each entry
  uint32_t nmatch[STREAM_RING];     // matching rows found so far of the batch at each entry
  StreamBatch desc[STREAM_RING];    // mirror of StreamCtrl::desc
  // the poller's counters (cudasp_stream_counters: STREAM_STAT_* below; the
  // workers' go to a per-wave array, summed on the host: a same-address
  // atomic per wave and counter serialized ~20k atomics at the kernel's exit)
  unsigned long long stat[16];
};

// StreamDev::stat indices (summed over the query's kernel launches): pieces
// and wave-rows claimed, polls of a wave with nothing to claim, pipeline
// drains, (unused), worker exits, idle exits of the
// poller (each one a kernel that left before the stream was closed), poller
// polls, and the workers' summed busy and lifetime in wall-clock ticks.
enum {
  STREAM_STAT_PIECES = 0,
  STREAM_STAT_WAVE_ROWS,
  STREAM_STAT_WAIT_POLLS,
  STREAM_STAT_DRAINS,
  STREAM_STAT_RESERVED,
  STREAM_STAT_WORKER_EXITS,
  STREAM_STAT_IDLE_EXITS,
  STREAM_STAT_POLLER_POLLS,
  STREAM_STAT_BUSY_TICKS,
  STREAM_STAT_LIFE_TICKS,
  STREAM_STAT_COUNT
};

// Wave-rows of the next claim (never past the published rows, rem > 0):
// k_scan_multi's adaptive rule, rem x mine / claimed
// (the wave's share of the work done so far: the three waves of a SIMD
// progress at ~1 : 0.3 : 0.05, so equal pieces would leave the slowest
// wave's piece as the tail), at least 1 and at most rmax; a wave's first
// claim is one wave-row.  A backlog of published batches gives rmax rows per
// thread (one inversion for rmax rows); a host slower than the GPU leaves
// small pieces, which cost only the GPU's slack.
CUDASP_HD uint32_t stream_piece_rows(uint64_t rem, uint64_t claimed, uint32_t mine, uint32_t rmax) {
  if (mine == 0 || claimed == 0) return 1u;
  const uint64_t r = rem * mine / claimed;
  return r < 1 ? 1u : (r > rmax ? rmax : (uint32_t)r);
}

// A worker wave's bookkeeping, kept by its lane 0 in LDS (k_scan_stream):
// its ticket, wave-rows claimed in this launch and the counters flushed to
// StreamDev::stat when it leaves.
struct StreamWave {
  uint64_t tk, t_start, busy;  // tk: the ticket, wave-rows [tk, tk + tr)
  uint64_t t_p, t_q, t_old;    // when pieces P and Q were taken; the oldest piece the wave holds
  uint32_t tr, have, mine, pieces, rows, polls, drains;
};

// Issue priority (s_setprio 0..3) of a wave whose oldest unfinished piece
// was taken `age` ticks ago: one level per `step` ticks.  A SIMD's resident
// waves issue by priority, then by wave age; without this the oldest wave
// of a SIMD takes most issue slots and the youngest one's piece waits until
// the others run dry (~1 : 0.3 : 0.05), so a batch completes only when its
// last, starved wave-row does -- 20+ ms after it was published, which
// stalls a host that reuses the batch's slot.  By piece age the SIMD works
// its pieces roughly in the order they were taken.  step 0: off.
CUDASP_HD uint32_t stream_prio(uint64_t age, uint64_t step) {
  if (step == 0) return 0;
  const uint64_t p = age / step;
  return p > 3 ? 3u : (uint32_t)p;
}

// Where a wave-row of a piece lives, looked up once at the piece's prefetch
// and kept in LDS by the wave (wave-uniform): its batch's device mirror and
// result buffers, its first row in the batch, the batch's rows, wave-rows
// and sequence number.  Valid while the wave holds the wave-row: the batch
// cannot complete (nor its ring entry or slot be reused) before it is done.
struct StreamWr {
  int64_t* mirror;
  uint8_t* flags;
  uint32_t* matches;
  uint32_t r0, n, nwr, b;
};

// Worker counters per wave (StreamDev::stat indices), flushed once at exit
// into the stream's per-wave array: STREAM_WSTAT words per wave.
constexpr uint32_t STREAM_WSTAT = 8;

}  // namespace cudasp
