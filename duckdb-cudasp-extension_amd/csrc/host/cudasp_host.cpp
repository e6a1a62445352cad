// cudasp_scan table-function host, DuckDB-independent (include/cudasp_host.h).
//
// Same state machine as the reference host (src/cudasp_extension.cu:87-659):
// bind validation with the same messages, per-thread chunks with the same
// NULL rules, round-robin GPU per thread, mutex-guarded global match list,
// last-thread-emits in 2048-row chunks.  What differs, by design:
//
//   * Rows do not wait in per-thread batches.  Each GPU has one *device feed*
//     per query: a ring of pinned batch slots that every executor thread fills
//     at once (a thread reserves room for its chunk under the feed's lock and
//     copies outside it), and a few streams, each with its own scanner, that
//     run the closed slots.  A slot closes at >= batch_size rows -- the
//     reference's trigger (:416-418), applied to the device's rows instead of
//     one thread's -- and the last thread still copying into it launches it:
//     H2D of the row blobs and the outputs CSR, the on-device transpose, both
//     stages fused in one k_scan_multi launch, D2H of the flags.  So
//       - the first launch starts after batch_size rows of the whole table,
//         not of one thread (the reference waits for one thread's batch);
//       - a table smaller than threads x batch_size still runs as full
//         batches while the threads are reading, instead of every thread's
//         partial batch in in_out_function_final (1M rows over 8 threads:
//         the reference runs 8 batches of 125k rows at the end);
//       - the end of the query drains one partial slot per device, not one
//         per thread;
//       - executor threads and GPUs are independent: a thread's chunks go to
//         the devices round-robin (chunk c of thread t to logical GPU
//         (t + c) mod num_gpus), so any thread count feeds any GPU count; a
//         thread's "assigned GPU" (:523-529) is where its chunks start;
//       - the streams in flight per device are the feed's (2 to 4, within
//         the hardware queues HIP gives the process: 3 at the default
//         GPU_MAX_HW_QUEUES = 4), not one per thread.
//     Batch composition therefore differs from the reference; the emitted
//     rows (a multiset -- the reference's order is unspecified) do not.
//   * Flat columns instead of two heap strings per row (:202-204), no host
//     transpose (:249-341) and no u64[n][64] staging (src/cudasp_gpu.cu:705-761).
//   * Scanners, streams and slots are created once and kept in a process-wide
//     pool across queries (src/cudasp_gpu.cu:487-666 allocates per batch).
//   * A failed batch is reported (cudasp_tf_function/final return an error)
//     instead of being dropped silently (:325, :378); a tweak_key BLOB that is
//     not 64 bytes is an error instead of an out-of-bounds read (:59-75).
#include "../../../include/cudasp_host.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/cudasp_abi.h"
#include "bind_data.hpp"
#include "slot_copy.hpp"

namespace {

constexpr uint64_t TWEAK_KEY_SIZE = 64;  // CudaspScanBindData::TWEAK_KEY_SIZE
constexpr uint64_t SCALAR_SIZE = 32;     // CudaspScanBindData::SCALAR_SIZE
constexpr uint32_t XONLY_SIZE = 32;      // full_x outputs: x-only keys
constexpr int FEED_MAX_STREAMS = 4;
// A streaming feed (one persistent kernel, cudasp_stream_*) keeps more slots
// in flight: the kernel's waves hold up to ~1.2M rows at once in 6-row
// pieces, and published work must stay ahead of them while the executor
// threads fill the next slots (paced probe at 9.4M rows, 1 label: 148.7 M
// tx/s with 8 slots in flight, 164.0 with 16, 166.6 with all published;
// profiles/r03_stream_iter2.txt).
constexpr int FEED_STREAM_SLOTS = 16;
// CUDASP_TF_STREAM_SLOTS overrides it, up to 48, inside the stream's
// descriptor ring: at most STREAM_RING batches may be published and not yet
// harvested (include/cudasp_abi.h, cudasp_stream_publish_batch and
// cudasp_stream_matches), which ring_overdue_locked enforces even when slots
// are reused out of order.
constexpr int FEED_MAX_STREAM_SLOTS = 48;
constexpr uint64_t STREAM_RING = 64;
constexpr int FEED_MAX_SLOTS = FEED_MAX_STREAM_SLOTS;
static_assert(FEED_MAX_SLOTS >= FEED_MAX_STREAMS + 2, "per-slot launch feeds");

int feed_stream_slots() {
  if (const char* e = getenv("CUDASP_TF_STREAM_SLOTS")) {
    const int v = atoi(e);
    if (v >= 4 && v <= FEED_MAX_STREAM_SLOTS) return v;
  }
  return FEED_STREAM_SLOTS;
}
// Rows resident on the GPU at once in k_scan_multi launches of 4 rows per
// thread: 256 CUs x 4 SIMDs x 3 waves x 64 lanes x 4 rows.
constexpr uint64_t GPU_FILL_ROWS = 786432;

void write_err(char* err, size_t cap, const char* fmt, ...) {
  if (!err || cap == 0) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(err, cap, fmt, ap);
  va_end(ap);
}

// Non-temporal stores for the copies into the slots (slot_copy.hpp);
// CUDASP_TF_NT=0 selects plain memcpy (A/B).
bool slot_nt() {
  static const bool on = [] {
    const char* e = getenv("CUDASP_TF_NT");
    return !(e && atoi(e) == 0);
  }();
  return on;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

extern "C" void cudasp_internal_scanner_park(cudasp_scanner* s);
extern "C" void cudasp_internal_set_error(const char* msg);
extern "C" void* cudasp_internal_scanner_stream(cudasp_scanner* s);
extern "C" void cudasp_internal_clear_key_cache(void);
#if CUDASP_STREAM_TRACE
extern "C" void cudasp_internal_trace_host(uint32_t kind, uint64_t a, uint32_t b);
#define ST_HOST(...) cudasp_internal_trace_host(__VA_ARGS__)
#else
#define ST_HOST(...) ((void)0)
#endif

namespace {

inline size_t out_words(const cudasp_tf_bind_data& b) { return b.opt.full_x ? XONLY_SIZE / 8 : 1; }

// Errors go to the library-wide thread-local message of cudasp_last_error().
int host_fail(int code, const char* fmt, ...) {
  char buf[768];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  cudasp_internal_set_error(buf);
  return code;
}

inline bool valid(const uint8_t* v, uint64_t i) { return v == nullptr || v[i] != 0; }
inline bool bit(const uint8_t* bm, uint64_t i) { return bm == nullptr || ((bm[i >> 3] >> (i & 7)) & 1u); }

#define HOST_HIP(expr)                                                                          \
  do {                                                                                          \
    hipError_t e_ = (expr);                                                                     \
    if (e_ != hipSuccess) return host_fail(CUDASP_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

struct DeviceSet {
  int prev = -1;
  explicit DeviceSet(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    (void)hipSetDevice(dev);
  }
  ~DeviceSet() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// Streams (= scanners) of a device feed: enough 4-row-per-thread launches of
// batch_size rows in flight to cover the GPU's wave slots (plus one for a
// slot being refilled), 2 to 4 -- but no more than the hardware queues the
// HIP runtime gives the feed: a process's streams on a device share
// GPU_MAX_HW_QUEUES queues (4 by default), one of them taken by the null
// stream, and kernels of streams that share a queue run one after another
// (measured: 4 streams at 4 queues map onto 3 queues, 132 M tx/s end to end;
// 3 streams, 158 M).  feeds_on_device: feeds of this query on the same HIP
// device (CUDASP_TF_DEVICE_MAP).  CUDASP_TF_STREAMS = 1..4 overrides.
int feed_streams_for(uint64_t batch_size, int hw_queues, int feeds_on_device) {
  if (const char* e = getenv("CUDASP_TF_STREAMS")) {
    const int v = atoi(e);
    if (v >= 1 && v <= FEED_MAX_STREAMS) return v;
  }
  const uint64_t k = (GPU_FILL_ROWS + batch_size - 1) / (batch_size ? batch_size : 1) + 1;
  int want = k < 2 ? 2 : (k > (uint64_t)FEED_MAX_STREAMS ? FEED_MAX_STREAMS : (int)k);
  const int budget = (hw_queues - 1) / (feeds_on_device > 0 ? feeds_on_device : 1);
  if (want > budget) want = budget;
  return want < 1 ? 1 : want;
}

enum SlotState { SLOT_FREE, SLOT_FILLING, SLOT_CLOSED, SLOT_BUSY, SLOT_LAUNCHED };

// One batch slot of a device feed.
struct FeedSlot {
  // pinned host buffers (H2D / D2H)
  uint8_t* h_tweaks = nullptr;  // cap_rows x 64, the row blobs as DuckDB holds them
  uint32_t* h_offs = nullptr;   // cap_rows, in outputs
  uint32_t* h_lens = nullptr;
  uint8_t* h_flags = nullptr;
  int64_t* h_outputs = nullptr;  // outputs_cap int64 words
  size_t outputs_cap = 0;
  uint32_t* h_matches = nullptr;  // streaming feed: the kernel's matching row indices (cap_rows)
  bool coherent = false;          // host buffers from cudasp_host_alloc (streaming feed)
  bool host_mem = false;          // host buffers from aligned_alloc (null-device measurement feed)
  // emit data of the rows (pageable; only read for matches)
  std::vector<uint8_t> txid_bytes;  // size() is the capacity
  std::vector<uint64_t> txid_off;   // cap_rows
  std::vector<uint32_t> txid_size;  // cap_rows
  // runs of rows whose txids are all 32 bytes, back to back from tx0 (a
  // chunk's rows; txid_off / txid_size are not written for them): r0, n, tx0
  struct TxRun {
    uint32_t r0, n;
    uint64_t tx0;
  };
  std::vector<TxRun> tx_runs;  // by r0 (reservations of a slot come in row order)
  std::vector<int32_t> heights;     // cap_rows
  // device buffers
  uint8_t* d_rows = nullptr;
  uint32_t* d_tx = nullptr;
  uint32_t* d_ty = nullptr;
  uint32_t* d_offs = nullptr;
  uint32_t* d_lens = nullptr;
  uint8_t* d_flags = nullptr;
  int64_t* d_outputs = nullptr;
  size_t d_outputs_cap = 0;  // words
  hipEvent_t done = nullptr;    // the batch's flags are on the host
  hipEvent_t copied = nullptr;  // the batch's H2D upload is done
  bool allocated = false;
  // fill state, guarded by Feed::mu
  SlotState state = SLOT_FREE;
  uint32_t rows = 0;     // rows reserved
  size_t words = 0;      // output words reserved
  size_t txid_used = 0;  // txid bytes reserved
  int writers = 0;       // reservations still copying
  int stream = 0;        // stream (scanner) of its launch
  uint64_t seq = 0;      // streaming feed: the batch's sequence number in the stream
  bool in_ring = false;  // streaming feed: published and not yet harvested (its seq holds a ring entry)
  double t_pub = 0;      // when it was published (the late-batch test hook)
};

// The GPU resources of a device feed, kept in a process-wide pool between
// queries (a later query only rebinds the scanners' keys).
struct FeedRes {
  int device = -1;
  uint32_t cap_rows = 0;
  int nstreams = 0;
  cudasp_scanner* scanners[FEED_MAX_STREAMS] = {};
  FeedSlot slots[FEED_MAX_SLOTS];
  // Streaming feed: one scanner, one persistent kernel (cudasp_stream_*)
  // reading the slots' coherent pinned buffers in place.  Buffers it
  // outgrows are freed only after the stream's kernel has ended (freeing
  // device or pinned memory waits for the device, hence for that kernel).
  cudasp_stream* stream = nullptr;
  uint32_t stream_blocks = 0;
  int stream_slots = FEED_STREAM_SLOTS;  // slots of a streaming feed (feed_stream_slots at creation)
  // null-device measurement feed (CUDASP_TF_NULL_DEVICE): no scanner, no
  // stream, no device call at all -- the slots are plain host memory -- so
  // the host's own ceiling can be measured anywhere, a GPU-less box included
  bool host_only = false;
  std::vector<void*> stale_host, stale_dev;
  int nslots() const { return stream || host_only ? stream_slots : nstreams + 2; }
};

void free_stale(FeedRes& r) {
  for (void* p : r.stale_host) cudasp_host_free(p);
  for (void* p : r.stale_dev) (void)hipFree(p);
  r.stale_host.clear();
  r.stale_dev.clear();
}

void free_slot(FeedSlot& s) {
  void* host[] = {s.h_tweaks, s.h_offs, s.h_lens, s.h_flags, s.h_outputs, s.h_matches};
  for (void* p : host)
    if (p) {
      if (s.host_mem)
        free(p);
      else if (s.coherent)
        cudasp_host_free(p);
      else
        (void)hipHostFree(p);
    }
  void* dev[] = {s.d_rows, s.d_tx, s.d_ty, s.d_offs, s.d_lens, s.d_flags, s.d_outputs};
  for (void* p : dev)
    if (p) (void)hipFree(p);
  if (s.done) (void)hipEventDestroy(s.done);
  if (s.copied) (void)hipEventDestroy(s.copied);
  s = FeedSlot();
}

void release_res(FeedRes* r) {
  if (!r) return;
  if (r->stream) {
    (void)cudasp_stream_finish(r->stream);  // closes it and waits for its kernel (bounded)
    if (cudasp_stream_abandoned(r->stream)) {
      // its kernel may still read the slots and use the scanner: leak them all
      fprintf(stderr, "cudasp_scan: device %d feed leaked (its streaming kernel did not end)\n", r->device);
      cudasp_stream_destroy(r->stream);
      return;
    }
    cudasp_stream_destroy(r->stream);
    r->stream = nullptr;
  }
  {
    DeviceSet dg(r->device);
    free_stale(*r);
    for (int k = 0; k < r->nstreams; k++)
      if (r->scanners[k]) (void)cudasp_scanner_sync(r->scanners[k]);
    for (FeedSlot& s : r->slots) free_slot(s);
  }
  for (int k = 0; k < r->nstreams; k++)
    if (r->scanners[k]) cudasp_scanner_destroy(r->scanners[k]);
  delete r;
}

constexpr size_t POOL_MAX = 64;
std::mutex g_pool_mu;
std::vector<FeedRes*> g_pool;

FeedRes* pool_take(int device, uint32_t cap_rows, int nstreams, uint32_t stream_blocks, bool host_only = false) {
  std::lock_guard<std::mutex> lock(g_pool_mu);
  for (size_t i = 0; i < g_pool.size(); i++) {
    FeedRes* r = g_pool[i];
    if (r->device == device && r->cap_rows == cap_rows && r->nstreams == nstreams &&
        (r->stream ? r->stream_blocks : 0u) == stream_blocks && r->host_only == host_only) {
      g_pool[i] = g_pool.back();
      g_pool.pop_back();
      return r;
    }
  }
  return nullptr;
}

void pool_put(FeedRes* r) {
  // parked scanners hold no spend-key fold table (cudasp_internal_scanner_park)
  for (int k = 0; k < r->nstreams; k++)
    if (r->scanners[k]) cudasp_internal_scanner_park(r->scanners[k]);
  {
    std::lock_guard<std::mutex> lock(g_pool_mu);
    if (g_pool.size() < POOL_MAX) {
      g_pool.push_back(r);
      return;
    }
  }
  release_res(r);
}

// Flags of the batch slots' pinned host buffers: the HIP default, or
// CUDASP_TF_PINNED = noncoherent / coherent / portable (measurement knob).
unsigned pinned_flags() {
  static const unsigned flags = [] {
    const char* e = getenv("CUDASP_TF_PINNED");
    if (!e) return (unsigned)hipHostMallocDefault;
    if (!strcmp(e, "noncoherent")) return (unsigned)hipHostMallocNonCoherent;
    if (!strcmp(e, "coherent")) return (unsigned)hipHostMallocCoherent;
    if (!strcmp(e, "portable")) return (unsigned)hipHostMallocPortable;
    return (unsigned)hipHostMallocDefault;
  }();
  return flags;
}

// Pinned/device buffers of a slot for cap_rows rows, at least `words` output
// words and `txid` txid bytes.  Called with the slot owned by the caller
// (state BUSY): no reservation, copy or launch touches it.
int prepare_slot_streaming(FeedRes& r, FeedSlot& s, size_t words, size_t txid);

int prepare_slot(FeedSlot& s, int device, uint32_t cap_rows, size_t words, size_t txid) {
  DeviceSet dg(device);
  if (!s.allocated) {
    const size_t n = cap_rows;
    HOST_HIP(hipHostMalloc((void**)&s.h_tweaks, n * 64, pinned_flags()));
    HOST_HIP(hipHostMalloc((void**)&s.h_offs, n * 4, pinned_flags()));
    HOST_HIP(hipHostMalloc((void**)&s.h_lens, n * 4, pinned_flags()));
    HOST_HIP(hipHostMalloc((void**)&s.h_flags, n, hipHostMallocDefault));
    HOST_HIP(hipMalloc((void**)&s.d_rows, n * 64));
    HOST_HIP(hipMalloc((void**)&s.d_tx, n * 32));
    HOST_HIP(hipMalloc((void**)&s.d_ty, n * 32));
    HOST_HIP(hipMalloc((void**)&s.d_offs, n * 4));
    HOST_HIP(hipMalloc((void**)&s.d_lens, n * 4));
    HOST_HIP(hipMalloc((void**)&s.d_flags, n));
    HOST_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    HOST_HIP(hipEventCreateWithFlags(&s.copied, hipEventDisableTiming));
    s.txid_off.resize(n);
    s.txid_size.resize(n);
    s.heights.resize(n);
    s.allocated = true;
  }
  if (words > s.outputs_cap) {
    size_t cap = s.outputs_cap ? s.outputs_cap : 4096;
    while (cap < words) cap *= 2;
    if (s.h_outputs) (void)hipHostFree(s.h_outputs);
    s.h_outputs = nullptr;
    s.outputs_cap = 0;
    HOST_HIP(hipHostMalloc((void**)&s.h_outputs, cap * sizeof(int64_t), pinned_flags()));
    s.outputs_cap = cap;
  }
  if (txid > s.txid_bytes.size()) s.txid_bytes.resize(txid);
  return CUDASP_OK;
}

// A null-device feed's slot (measurement): the same host buffers as a
// streaming slot, from aligned_alloc, and no device mirror.
int prepare_slot_host(FeedRes& r, FeedSlot& s, size_t words, size_t txid) {
  const size_t n = r.cap_rows;
  auto host = [&](void** p, size_t bytes) -> int {
    *p = aligned_alloc(4096, (bytes + 4095) / 4096 * 4096);
    return *p ? CUDASP_OK : host_fail(CUDASP_ERR_CAPACITY, "host slot allocation of %zu bytes failed", bytes);
  };
  if (!s.allocated) {
    s.host_mem = true;
    int rc = host((void**)&s.h_tweaks, n * 64);
    if (rc == CUDASP_OK) rc = host((void**)&s.h_offs, n * 4);
    if (rc == CUDASP_OK) rc = host((void**)&s.h_lens, n * 4);
    if (rc == CUDASP_OK) rc = host((void**)&s.h_matches, n * 4);
    if (rc != CUDASP_OK) return rc;
    s.txid_off.resize(n);
    s.txid_size.resize(n);
    s.heights.resize(n);
    s.allocated = true;
  }
  if (words > s.outputs_cap) {
    size_t cap = s.outputs_cap ? s.outputs_cap : 4096;
    while (cap < words) cap *= 2;
    free(s.h_outputs);
    s.h_outputs = nullptr;
    s.outputs_cap = 0;
    const int rc = host((void**)&s.h_outputs, cap * sizeof(int64_t));
    if (rc != CUDASP_OK) return rc;
    s.outputs_cap = cap;
  }
  if (txid > s.txid_bytes.size()) s.txid_bytes.resize(txid);
  return CUDASP_OK;
}

// A streaming feed's slot: coherent pinned buffers the kernel reads in place
// (cudasp_host_alloc) and, with labels, the device mirror of the outputs.
// Nothing is freed while the feed's kernel may run: outgrown buffers wait in
// the feed's stale lists.
int prepare_slot_streaming(FeedRes& r, FeedSlot& s, size_t words, size_t txid) {
  DeviceSet dg(r.device);
  const size_t n = r.cap_rows;
  auto host = [&](void** p, size_t bytes) -> int {
    const int rc = cudasp_host_alloc(p, bytes);
    return rc == CUDASP_OK ? rc : host_fail(rc, "pinned slot allocation failed: %s", cudasp_last_error());
  };
  if (!s.allocated) {
    s.coherent = true;
    int rc = host((void**)&s.h_tweaks, n * 64);
    if (rc == CUDASP_OK) rc = host((void**)&s.h_offs, n * 4);
    if (rc == CUDASP_OK) rc = host((void**)&s.h_lens, n * 4);
    if (rc == CUDASP_OK) rc = host((void**)&s.h_matches, n * 4);
    if (rc != CUDASP_OK) return rc;
    s.txid_off.resize(n);
    s.txid_size.resize(n);
    s.heights.resize(n);
    s.allocated = true;
  }
  if (words > s.outputs_cap) {
    size_t cap = s.outputs_cap ? s.outputs_cap : 4096;
    while (cap < words) cap *= 2;
    if (s.h_outputs) r.stale_host.push_back(s.h_outputs);
    s.h_outputs = nullptr;
    s.outputs_cap = 0;
    const int rc = host((void**)&s.h_outputs, cap * sizeof(int64_t));
    if (rc != CUDASP_OK) return rc;
    s.outputs_cap = cap;
  }
  // the device mirror of the outputs, which the kernel's compares read (at
  // least one word: a batch whose rows have no outputs still needs one)
  if (!s.d_outputs || s.d_outputs_cap < s.outputs_cap) {
    if (s.d_outputs) r.stale_dev.push_back(s.d_outputs);
    s.d_outputs = nullptr;
    s.d_outputs_cap = 0;
    const size_t cap = std::max<size_t>(s.outputs_cap, 1);
    if (hipMalloc((void**)&s.d_outputs, cap * sizeof(int64_t)) != hipSuccess) {
      (void)hipGetLastError();
      return host_fail(CUDASP_ERR_HIP, "outputs mirror of %zu words on device %d: allocation failed", cap, r.device);
    }
    s.d_outputs_cap = cap;
  }
  if (txid > s.txid_bytes.size()) s.txid_bytes.resize(txid);
  return CUDASP_OK;
}

}  // namespace

// One device feed of a query (see the header comment).
struct Feed {
  FeedRes* res = nullptr;
  cudasp_tf_global* g = nullptr;
  uint64_t batch_size = 0;
  size_t ow = 1;  // int64 words per output
  std::mutex mu;
  std::condition_variable cv;
  int open = 0;             // the slot being filled
  uint32_t launch_seq = 0;  // round-robin over the streams
  // capacity a slot opens with, per row (grown when slots close on output or
  // txid space before batch_size rows: long output lists, long txids)
  double words_per_row = 2.0;
  double txid_per_row = 32.0;
  int ramp = 3;          // ramp slots (close_at); CUDASP_TF_RAMP=N sets them, 0 turns the ramp off
  bool upload_null = true;  // H2D on the null stream; CUDASP_TF_UPLOAD=stream: on the scan stream (A/B)
  uint32_t closed = 0;   // slots closed so far
  uint64_t pub_next = 0;  // streaming feed: one past the highest sequence number published
  // test hook (CUDASP_TF_TEST_LATE_SEQ / _MS): batch late_seq reads as not
  // done to the non-blocking checks for late_s after its publish, so the ring
  // moves on without it (a starved batch; a blocking harvest still takes it)
  int64_t late_seq = -1;
  double late_s = 0;
  // measurement only (CUDASP_TF_NULL_DEVICE=1): slots are marked done by
  // the host at launch, with no publish, copy or kernel -- reservation,
  // copies into the slots and harvest unchanged, nothing emitted -- so a
  // query runs at the executor threads' own ceiling (the host's capacity
  // for N GPUs; tools/host_e2e --null-device)
  bool null_device = false;
  int error = CUDASP_OK;
  std::string error_msg;
  std::mutex stream_mu[FEED_MAX_STREAMS];  // a scanner's host state is not re-entrant
  // statistics (under mu)
  uint64_t launches = 0, rows = 0;
  double harvest_wait_s = 0;
  double reserve_s = 0, copy_s = 0, launch_s = 0;
};

struct cudasp_tf_global {
  std::atomic<uint64_t> currently_adding{0};
  std::mutex finalize_lock;
  std::mutex output_lock;
  std::vector<std::string> output_txids;
  std::vector<int32_t> output_heights;
  std::vector<std::string> output_tweak_keys;
  size_t output_position = 0;
  std::atomic<bool> output_thread_claimed{false};
  int num_gpus = 0;
  std::atomic<int> next_gpu_assignment{0};
  // logical GPU -> HIP device; the identity unless CUDASP_TF_DEVICE_MAP is set
  std::vector<int> device_map;
  // device feeds, one per logical GPU, created on its first chunk
  const cudasp_tf_bind_data* bind = nullptr;
  int feed_streams = 0;
  int launch_streams = 0;  // streams of a per-slot-launch feed (a streaming feed that falls back)
  // feeds[lg] is written once, under feed_create_mu[lg]; threads look a feed
  // up through feed_ptr[lg] (published after the feed is complete)
  std::vector<std::unique_ptr<Feed>> feeds;
  std::unique_ptr<std::atomic<Feed*>[]> feed_ptr;
  std::unique_ptr<std::mutex[]> feed_create_mu;
  int hw_queues = 0;  // GPU_MAX_HW_QUEUES at init (HIP's default 4 when unset)
  int max_streams_per_device = 0;
  // Streaming feeds (one persistent kernel per feed, cudasp_stream_*): the
  // default with the default options and one feed per device (measured
  // faster end to end); CUDASP_TF_MODE=launch selects the
  // per-slot launches.
  bool streaming = false;
  bool null_device = false;  // CUDASP_TF_NULL_DEVICE: measurement-only feeds (Feed::null_device)
  std::atomic<bool> streaming_fallback{false};  // this query's keys/options rule the streaming scan out (feed_for)
};

struct cudasp_tf_local {
  bool finalized = false;
  bool is_output_thread = false;
  int assigned_gpu = -1;  // logical GPU of the thread's first chunk (round-robin over num_gpus)
  int device = -1;        // the HIP device it maps to
  uint64_t chunks = 0;    // chunks fed so far (chunk c goes to logical GPU assigned_gpu + c)
};

namespace {

int feed_fail(Feed& f, int rc) {
  // first error of the feed wins; later callers report it too
  if (f.error == CUDASP_OK) {
    f.error = rc;
    f.error_msg = cudasp_last_error();
  }
  return rc;
}

int feed_error(const Feed& f) { return host_fail(f.error, "%s", f.error_msg.c_str()); }

// Launch a closed slot (writers done).  Caller holds `lk` on f.mu; it is
// released around the HIP calls (the slot is BUSY meanwhile).
int launch_locked(Feed& f, FeedSlot& s, std::unique_lock<std::mutex>& lk) {
  FeedRes& r = *f.res;
  s.state = SLOT_BUSY;
  s.stream = r.nstreams ? (int)(f.launch_seq++ % (uint32_t)r.nstreams) : 0;
  const uint32_t n = s.rows;
  const size_t words = s.words;
  lk.unlock();
  const double t0 = now_s();
  int rc = CUDASP_OK;
  if (f.null_device) {
    // measurement only: no device work
  } else if (r.stream) {
    // Streaming feed: publish the slot to the feed's kernel, which reads it
    // in place (no copies, no launch), copies each row's outputs to the
    // slot's device mirror (sized with the slot, prepare_slot_streaming) and
    // writes the matching rows' indices back into the slot.
    DeviceSet dg(r.device);
    if (words > s.d_outputs_cap) {
      rc = host_fail(CUDASP_ERR_INVALID_ARG, "batch of %zu output words exceeds its mirror (%zu)", words,
                     s.d_outputs_cap);
    } else {
      cudasp_stream_batch b{};
      b.tweak_keys = s.h_tweaks;
      b.outputs = s.h_outputs;
      b.output_offsets = s.h_offs;
      b.output_lengths = s.h_lens;
      b.n = n;
      b.match_flags = nullptr;
      b.match_rows = s.h_matches;
      b.d_mirror = s.d_outputs;
      rc = cudasp_stream_publish_batch(r.stream, &b, &s.seq);
      if (rc != CUDASP_OK)
        rc = host_fail(rc, "cudasp_scan batch of %u rows on device %d failed: %s", n, r.device, cudasp_last_error());
    }
  } else {
    std::lock_guard<std::mutex> sl(f.stream_mu[s.stream]);
    cudasp_scanner* sc = r.scanners[s.stream];
    hipStream_t st = (hipStream_t)cudasp_internal_scanner_stream(sc);
    DeviceSet dg(r.device);
    auto run = [&]() -> int {
      if (words > s.d_outputs_cap) {  // the slot's previous launch has been harvested: no kernel reads it
        if (s.d_outputs) HOST_HIP(hipFree(s.d_outputs));
        s.d_outputs = nullptr;
        s.d_outputs_cap = 0;
        HOST_HIP(hipMalloc((void**)&s.d_outputs, s.outputs_cap * sizeof(int64_t)));
        s.d_outputs_cap = s.outputs_cap;
      }
      // The upload goes on the device's null stream (its hardware queue is
      // otherwise idle) and the scan stream waits for it: on the scan stream
      // itself a batch's H2D would queue behind that stream's running kernel,
      // and each stream would spend ~0.8 ms of every ~6 ms launch cycle with
      // no kernel in flight (kernel + copy trace, profiles/r03_e2e_trace.txt).
      // The slot's device buffers are free: its previous batch was harvested.
      hipStream_t up = f.upload_null ? (hipStream_t)0 : st;
      HOST_HIP(hipMemcpyAsync(s.d_rows, s.h_tweaks, (size_t)n * 64, hipMemcpyHostToDevice, up));
      HOST_HIP(hipMemcpyAsync(s.d_offs, s.h_offs, (size_t)n * 4, hipMemcpyHostToDevice, up));
      HOST_HIP(hipMemcpyAsync(s.d_lens, s.h_lens, (size_t)n * 4, hipMemcpyHostToDevice, up));
      if (words)
        HOST_HIP(hipMemcpyAsync(s.d_outputs, s.h_outputs, words * sizeof(int64_t), hipMemcpyHostToDevice, up));
      if (up != st) {
        HOST_HIP(hipEventRecord(s.copied, up));
        HOST_HIP(hipStreamWaitEvent(st, s.copied, 0));
      }
      int rc2 = cudasp_tweaks_to_columns(s.d_rows, n, s.d_tx, s.d_ty, st);
      if (rc2 == CUDASP_OK)
        rc2 = cudasp_scan_device(sc, s.d_tx, s.d_ty, s.d_outputs, s.d_offs, s.d_lens, n, s.d_flags, nullptr, nullptr,
                                 st);
      if (rc2 != CUDASP_OK)
        return host_fail(rc2, "cudasp_scan batch of %u rows on device %d failed: %s", n, r.device,
                         cudasp_last_error());
      HOST_HIP(hipMemcpyAsync(s.h_flags, s.d_flags, n, hipMemcpyDeviceToHost, st));
      HOST_HIP(hipEventRecord(s.done, st));
      return CUDASP_OK;
    };
    rc = run();
  }
  const double spent = now_s() - t0;
  lk.lock();
  f.launch_s += spent;
  if (rc != CUDASP_OK) {
    s.state = SLOT_FREE;  // its rows are lost; the query fails with rc
    feed_fail(f, rc);
  } else {
    s.state = SLOT_LAUNCHED;
    f.launches++;
    f.rows += n;
    if (r.stream && !f.null_device) {
      s.in_ring = true;
      s.t_pub = now_s();
      f.pub_next = std::max(f.pub_next, s.seq + 1);
    }
  }
  f.cv.notify_all();
  return rc;
}

// Wait for a launched slot and move its matches to the global list
// (ProcessBatch :378-392).  Caller holds `lk`; released while waiting.
int harvest_locked(Feed& f, FeedSlot& s, std::unique_lock<std::mutex>& lk) {
  s.state = SLOT_BUSY;
  lk.unlock();
  const double t0 = now_s();
  hipError_t e;
  std::string stream_err;
  if (f.null_device) {
    e = hipSuccess;
  } else {
    DeviceSet dg(f.res->device);
    if (f.res->stream) {
      e = hipSuccess;
      if (cudasp_stream_wait(f.res->stream, s.seq) != CUDASP_OK) {
        e = hipErrorUnknown;
        stream_err = cudasp_last_error();
      }
    } else {
      e = hipEventSynchronize(s.done);
    }
  }
  const double waited = now_s() - t0;
  ST_HOST(112, (uint64_t)(waited * 1e9), (uint32_t)s.seq);
  if (e == hipSuccess && !f.null_device) {
    cudasp_tf_global& g = *f.g;
    const auto emit = [&](uint32_t i) {
      // a row of a 32-byte-txid run, else its own offset and size
      auto it = std::upper_bound(s.tx_runs.begin(), s.tx_runs.end(), i,
                                 [](uint32_t r, const FeedSlot::TxRun& t) { return r < t.r0; });
      if (it != s.tx_runs.begin() && i - (it - 1)->r0 < (it - 1)->n)
        g.output_txids.emplace_back((const char*)s.txid_bytes.data() + (it - 1)->tx0 + 32ull * (i - (it - 1)->r0),
                                    32);
      else
        g.output_txids.emplace_back((const char*)s.txid_bytes.data() + s.txid_off[i], s.txid_size[i]);
      g.output_heights.push_back(s.heights[i]);
      g.output_tweak_keys.emplace_back((const char*)s.h_tweaks + (size_t)i * TWEAK_KEY_SIZE, TWEAK_KEY_SIZE);
    };
    if (f.res->stream) {
      // the kernel's compacted matches (in no particular order: sorted, so a
      // batch emits in row order like the flags scan)
      uint32_t nm = 0;
      if (cudasp_stream_matches(f.res->stream, s.seq, &nm) != CUDASP_OK || nm > s.rows) {
        e = hipErrorUnknown;
        stream_err = cudasp_last_error();
      } else {
        std::sort(s.h_matches, s.h_matches + nm);
        std::lock_guard<std::mutex> lock(g.output_lock);
        for (uint32_t k = 0; k < nm; k++) emit(s.h_matches[k]);
      }
    } else {
      std::lock_guard<std::mutex> lock(g.output_lock);
      // eight flags at a time: matches are rare
      uint32_t i = 0;
      for (; i + 8 <= s.rows; i += 8) {
        uint64_t w;
        memcpy(&w, s.h_flags + i, 8);
        if (!w) continue;
        for (uint32_t k = i; k < i + 8; k++)
          if (s.h_flags[k]) emit(k);
      }
      for (; i < s.rows; i++)
        if (s.h_flags[i]) emit(i);
    }
  }
  lk.lock();
  f.harvest_wait_s += waited;
  s.in_ring = false;
  s.state = SLOT_FREE;
  f.cv.notify_all();
  if (e != hipSuccess)
    return feed_fail(f, host_fail(CUDASP_ERR_HIP, "batch on device %d failed: %s", f.res->device,
                                  stream_err.empty() ? hipGetErrorString(e) : stream_err.c_str()));
  return CUDASP_OK;
}

// Close the open slot (no more reservations) and move on to the next; the
// last writer launches it (launch_locked directly if there is none).
int close_open_locked(Feed& f, std::unique_lock<std::mutex>& lk) {
  FeedSlot& s = f.res->slots[f.open];
  s.state = SLOT_CLOSED;
  f.closed++;
  f.open = (f.open + 1) % f.res->nslots();
  if (s.writers == 0) return launch_locked(f, s, lk);
  return CUDASP_OK;
}

// Rows at which the open slot closes: batch_size, except that a feed's first
// `ramp` slots close at batch_size / 2^ramp, ..., / 4, / 2, so the GPU starts
// before a whole batch has been read.  Per-slot launches: 3 (/ 8, / 4, / 2:
// +6% end to end at 1M rows, +2% at 9.4M, within the spread at 32.7M,
// profiles/r03_e2e_ramp_ab.txt).  A streaming feed starts its kernel on the
// first slot and takes 5 (from / 32: ~9k rows, read in well under 0.1 ms).
// CUDASP_TF_RAMP=N sets N, 0 turns the ramp off.
uint64_t close_at(const Feed& f) {
  if (f.closed >= (uint32_t)f.ramp) return f.batch_size;
  const uint64_t r = f.batch_size >> (f.ramp - (int)f.closed);
  return r < CUDASP_TF_VECTOR_SIZE ? std::min<uint64_t>(f.batch_size, CUDASP_TF_VECTOR_SIZE) : r;
}

// The streaming feeds' wait timeout (cudasp_stream_set_timeout): a wait
// that sees no batch complete for this long fails the query instead of
// hanging it.  CUDASP_STREAM_TIMEOUT_MS, read per query; 60 s by default.
uint32_t stream_timeout_ms() {
  if (const char* e = getenv("CUDASP_STREAM_TIMEOUT_MS")) {
    const long v = atol(e);
    if (v >= 1 && v <= 86400000) return (uint32_t)v;
  }
  return 60000u;
}

// Whether a launched slot's batch is done (no waiting).
bool slot_done(Feed& f, FeedSlot& s) {
  if (f.null_device) return true;
  if (f.res->stream) {
    if (f.late_seq >= 0 && s.seq == (uint64_t)f.late_seq && now_s() - s.t_pub < f.late_s) return false;
    return cudasp_stream_query(f.res->stream, s.seq) == 1;
  }
  DeviceSet dg(f.res->device);
  return hipEventQuery(s.done) == hipSuccess;
}

// Another slot to open instead of the open one, whose batch is still in
// flight: the next slot in ring order that is free or whose batch is done
// (-1: none).  Slots are taken out of order, so a batch held up by a slow
// wave-row occupies its slot alone instead of stalling the whole ring (a
// streaming kernel's youngest waves get few issue slots: one batch of the
// 9.4M-row table finished 27 ms after it was published).  Out-of-order reuse
// is bounded by ring_overdue_locked, checked before every slot opens.
int ready_slot_locked(Feed& f) {
  const int n = f.res->nslots();
  for (int i = 1; i < n; i++) {
    const int k = (f.open + i) % n;
    FeedSlot& t = f.res->slots[k];
    if (t.state == SLOT_FREE || (t.state == SLOT_LAUNCHED && slot_done(f, t))) return k;
  }
  return -1;
}

// Streaming feed: the slot holding the oldest published, unharvested batch
// if opening another slot could let the stream run STREAM_RING batches past
// it (-1 otherwise).  Every batch published after this open comes from a
// slot opened by now or later, at most nslots of which are unpublished, so
// requiring pub_next + nslots - oldest < STREAM_RING at every open keeps
// each publish within STREAM_RING of the oldest batch not yet harvested:
// publish never finds its ring entry's previous batch undone
// (CUDASP_ERR_CAPACITY) and a late batch's match count is read before its
// entry is reused (cudasp_stream_matches).  The caller then harvests that
// slot first, however long its batch takes.
int ring_overdue_locked(Feed& f) {
  if (!f.res->stream) return -1;
  const int n = f.res->nslots();
  int k = -1;
  for (int i = 0; i < n; i++) {
    const FeedSlot& t = f.res->slots[i];
    if (t.in_ring && (k < 0 || t.seq < f.res->slots[k].seq)) k = i;
  }
  if (k < 0) return -1;
  return f.pub_next + (uint64_t)n - f.res->slots[k].seq >= STREAM_RING ? k : -1;
}

struct Reservation {
  FeedSlot* slot = nullptr;
  uint32_t row0 = 0;
  size_t word0 = 0;
  size_t tx0 = 0;
};

// Reservation flags: every txid of the chunk is 32 bytes (its rows become a
// TxRun; the writer skips txid_off / txid_size).
constexpr int RES_TXID32 = 1;

// Room for a chunk of nrows rows, nwords output words and ntx txid bytes in
// the feed's open slot.  Blocks while the ring is busy; harvests finished
// slots on the way (that wait is the executor threads' back-pressure).
int feed_reserve(Feed& f, uint32_t nrows, size_t nwords, size_t ntx, Reservation* out, int flags = 0) {
  FeedRes& r = *f.res;
  std::unique_lock<std::mutex> lk(f.mu);
  for (;;) {
    if (f.error != CUDASP_OK) return feed_error(f);
    FeedSlot& s = r.slots[f.open];
    switch (s.state) {
      case SLOT_FREE: {
        const int overdue = ring_overdue_locked(f);
        if (overdue >= 0) {
          FeedSlot& o = r.slots[overdue];
          if (o.state == SLOT_LAUNCHED) {
            const int rc = harvest_locked(f, o, lk);
            if (rc != CUDASP_OK) return rc;
          } else {
            f.cv.wait(lk);  // another thread is harvesting it
          }
          continue;
        }
        const size_t want_words = std::max(
            std::min((size_t)(f.words_per_row * r.cap_rows), (size_t)UINT32_MAX * f.ow), nwords);
        const size_t want_tx = std::max((size_t)(f.txid_per_row * r.cap_rows), ntx);
        if (!s.allocated || s.outputs_cap < want_words || s.txid_bytes.size() < want_tx) {
          s.state = SLOT_BUSY;
          lk.unlock();
          const int rc = r.host_only ? prepare_slot_host(r, s, want_words, want_tx)
                         : r.stream  ? prepare_slot_streaming(r, s, want_words, want_tx)
                                     : prepare_slot(s, r.device, r.cap_rows, want_words, want_tx);
          lk.lock();
          s.state = SLOT_FREE;
          f.cv.notify_all();
          if (rc != CUDASP_OK) return feed_fail(f, rc);
        }
        s.state = SLOT_FILLING;
        s.rows = 0;
        s.words = 0;
        s.txid_used = 0;
        s.writers = 0;
        s.tx_runs.clear();
        continue;
      }
      case SLOT_FILLING: {
        // output offsets are u32 (as the reference's h_output_offsets)
        const bool offs_fit = (s.words + nwords) / f.ow <= UINT32_MAX;
        if (!offs_fit && s.rows == 0)
          return feed_fail(f, host_fail(CUDASP_ERR_CAPACITY, "a chunk of %u rows holds %zu outputs: more than a "
                                        "batch's u32 output offsets address", nrows, nwords / f.ow));
        if (offs_fit && s.rows + nrows <= r.cap_rows && s.words + nwords <= s.outputs_cap &&
            s.txid_used + ntx <= s.txid_bytes.size()) {
          out->slot = &s;
          out->row0 = s.rows;
          out->word0 = s.words;
          out->tx0 = s.txid_used;
          if (flags & RES_TXID32) s.tx_runs.push_back(FeedSlot::TxRun{s.rows, nrows, s.txid_used});
          s.rows += nrows;
          s.words += nwords;
          s.txid_used += ntx;
          s.writers++;
          // >= batch_size (:416-418): closed now, launched by its last writer
          if (s.rows >= close_at(f)) {
            s.state = SLOT_CLOSED;
            f.closed++;
            f.open = (f.open + 1) % r.nslots();
          }
          return CUDASP_OK;
        }
        if (s.rows == 0) {  // an empty slot (no writers) too small for this chunk: grow it
          f.words_per_row = std::max(f.words_per_row, (double)nwords / r.cap_rows);
          f.txid_per_row = std::max(f.txid_per_row, (double)ntx / r.cap_rows);
          s.state = SLOT_BUSY;
          lk.unlock();
          const int rc = r.host_only ? prepare_slot_host(r, s, nwords, ntx)
                         : r.stream  ? prepare_slot_streaming(r, s, nwords, ntx)
                                     : prepare_slot(s, r.device, r.cap_rows, nwords, ntx);
          lk.lock();
          s.state = SLOT_FILLING;
          f.cv.notify_all();
          if (rc != CUDASP_OK) {
            s.state = SLOT_FREE;
            return feed_fail(f, rc);
          }
          continue;
        }
        // out of output or txid space before batch_size rows: close it, and
        // open later slots with room for this shape of row
        const double rows_after = (double)(s.rows + nrows);
        f.words_per_row = std::max(f.words_per_row, 1.25 * (s.words + nwords) / rows_after);
        f.txid_per_row = std::max(f.txid_per_row, 1.25 * (s.txid_used + ntx) / rows_after);
        const int rc = close_open_locked(f, lk);
        if (rc != CUDASP_OK) return rc;
        continue;
      }
      case SLOT_LAUNCHED: {
        // the open slot's batch may still be in flight: open a ready slot
        // (free, or its batch done) instead; with none, poll for one -- any
        // batch that completes frees a slot -- and block on this slot's
        // batch (under the stream's no-progress deadline) only after
        // nothing has become ready for that long.  Blocking on the open
        // slot at once stalled the ring behind one slow batch: 18 ms
        // without a publish at 9.4M rows (tools/stream_trace.py, round 4).
        if (!slot_done(f, s)) {
          const int open0 = f.open;
          const double t0 = now_s(), limit = 1e-3 * stream_timeout_ms();
          int k = ready_slot_locked(f);
          while (k < 0) {
            f.cv.wait_for(lk, std::chrono::microseconds(20));
            if (f.error != CUDASP_OK) return feed_error(f);
            if (f.open != open0 || s.state != SLOT_LAUNCHED || slot_done(f, s)) break;
            k = ready_slot_locked(f);
            if (now_s() - t0 > limit) break;
          }
          if (f.open != open0 || s.state != SLOT_LAUNCHED) continue;  // another thread moved on
          if (k >= 0) {
            f.open = k;
            continue;
          }
        }
        const int rc = harvest_locked(f, s, lk);
        if (rc != CUDASP_OK) return rc;
        continue;
      }
      default:  // CLOSED (writers still copying) or BUSY (allocating, launching, harvesting)
        f.cv.wait(lk);
    }
  }
}

// A reservation's copy is done; the last writer of a closed slot launches it.
int feed_commit(Feed& f, FeedSlot& s, double reserve_s, double copy_s) {
  std::unique_lock<std::mutex> lk(f.mu);
  f.reserve_s += reserve_s;
  f.copy_s += copy_s;
  s.writers--;
  if (s.state == SLOT_CLOSED && s.writers == 0) return launch_locked(f, s, lk);
  return CUDASP_OK;
}

// End of the query's input: launch every feed's partial slot (all feeds
// first, so the devices drain in parallel), then harvest everything.
int feeds_flush(cudasp_tf_global& g) {
  int rc = CUDASP_OK;
  ST_HOST(111, 0, 0);
  for (auto& fp : g.feeds) {
    if (!fp) continue;
    Feed& f = *fp;
    std::unique_lock<std::mutex> lk(f.mu);
    FeedSlot& s = f.res->slots[f.open];
    if (s.state == SLOT_FILLING) {
      if (s.rows > 0) {
        const int r2 = close_open_locked(f, lk);
        if (rc == CUDASP_OK) rc = r2;
      } else {
        s.state = SLOT_FREE;
      }
    }
    // a streaming feed's last batch is published: its kernel may end as
    // soon as the batches are done (finish below only waits and resets)
    if (f.res->stream) {
      lk.unlock();
      DeviceSet dg(f.res->device);
      (void)cudasp_stream_close(f.res->stream);
    }
  }
  for (auto& fp : g.feeds) {
    if (!fp) continue;
    Feed& f = *fp;
    std::unique_lock<std::mutex> lk(f.mu);
    for (int i = 0; i < f.res->nslots(); i++) {
      FeedSlot& s = f.res->slots[(f.open + i) % f.res->nslots()];
      while (s.state == SLOT_CLOSED || s.state == SLOT_BUSY) f.cv.wait(lk);
      if (s.state == SLOT_LAUNCHED) {
        const int r2 = harvest_locked(f, s, lk);
        if (rc == CUDASP_OK) rc = r2;
      }
    }
    if (rc == CUDASP_OK && f.error != CUDASP_OK) rc = feed_error(f);
  }
  ST_HOST(113, 0, 0);
  // streaming feeds: every batch is done; close the streams so their kernels
  // end (and the streams are ready for the next query)
  for (auto& fp : g.feeds) {
    if (!fp || !fp->res->stream) continue;
    DeviceSet dg(fp->res->device);
    const int r2 = cudasp_stream_finish(fp->res->stream);
    if (r2 != CUDASP_OK && rc == CUDASP_OK) rc = feed_fail(*fp, host_fail(r2, "%s", cudasp_last_error()));
    // an abandoned kernel may still read the outgrown buffers: feeds_release leaks them
    if (!cudasp_stream_abandoned(fp->res->stream)) free_stale(*fp->res);
  }
  return rc;
}

// The feed of logical GPU `lg`, created on first use: pooled resources for
// (device, capacity, streams), or new scanners, rebound to this query's keys.
// The query's logical GPUs: every device (cudaGetDeviceCount, falling back
// to 1, src/cudasp_extension.cu:129-132), or the test hook
// CUDASP_TF_DEVICE_MAP="0,0", which makes the host see 2 logical GPUs that
// both run on device 0, so the num_gpus > 1 round-robin can be exercised on a
// one-GPU box.
int tf_device_map(std::vector<int>& out) {
  int n = cudasp_device_count();
  if (n <= 0) n = 1;
  out.clear();
  for (int d = 0; d < n; d++) out.push_back(d);
  if (const char* m = getenv("CUDASP_TF_DEVICE_MAP")) {
    std::vector<int> map;
    const int ndev = cudasp_device_count();
    for (const char* p = m; *p;) {
      char* end = nullptr;
      const long d = strtol(p, &end, 10);
      if (end == p || d < 0 || (ndev > 0 && d >= ndev))
        return host_fail(CUDASP_ERR_INVALID_ARG, "CUDASP_TF_DEVICE_MAP: bad device list \"%s\"", m);
      map.push_back((int)d);
      p = *end == ',' ? end + 1 : end;
    }
    if (!map.empty()) out = map;
  }
  return CUDASP_OK;
}

// A streaming feed's wave slots on its device: the device's 3 waves per SIMD
// shared by the logical GPUs on it.
uint32_t stream_blocks_for(int device, const std::vector<int>& map) {
  int cus = 0, on_dev = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
  for (int d : map) on_dev += d == device;
  return (uint32_t)(cus * 3 / (on_dev > 0 ? on_dev : 1));
}

int feed_for(cudasp_tf_global& g, const cudasp_tf_bind_data& b, int lg, Feed** out) {
  if ((*out = g.feed_ptr[lg].load(std::memory_order_acquire)) != nullptr) return CUDASP_OK;
  std::lock_guard<std::mutex> lock(g.feed_create_mu[lg]);
  if ((*out = g.feed_ptr[lg].load(std::memory_order_acquire)) != nullptr) return CUDASP_OK;
  const int device = g.device_map[lg];
  const uint32_t cap_rows = (uint32_t)(b.batch_size + CUDASP_TF_VECTOR_SIZE);
  if (g.null_device) {  // (pooled apart from real feeds: pool_take matches host_only)
    FeedRes* r = pool_take(device, cap_rows, 0, 0, true);
    if (!r) {
      r = new FeedRes();
      r->device = device;
      r->cap_rows = cap_rows;
      r->host_only = true;
      r->stream_slots = feed_stream_slots();
    }
    auto f = std::make_unique<Feed>();
    f->res = r;
    f->g = &g;
    f->batch_size = b.batch_size;
    f->ow = out_words(b);
    f->words_per_row = 2.0 * f->ow;
    f->ramp = 5;
    f->null_device = true;
    *out = f.get();
    g.feeds[lg] = std::move(f);
    g.feed_ptr[lg].store(*out, std::memory_order_release);
    return CUDASP_OK;
  }
  const auto* scan = (const uint8_t*)b.scan_private_key_data.data();
  const auto* spend = (const uint8_t*)b.spend_public_key_data.data();
  const auto* labels = (const uint8_t*)b.label_keys_flat.data();
  const auto nlabels = (uint32_t)b.label_keys_data.size();
  // a streaming feed's grid: its share of the device's wave slots
  const uint32_t blocks = g.streaming ? stream_blocks_for(device, g.device_map) : 0u;
  FeedRes* r = pool_take(device, cap_rows, g.streaming ? 1 : g.feed_streams, blocks);
  if (r) {
    for (int k = 0; k < r->nstreams; k++) {
      int rc = cudasp_scanner_set_keys(r->scanners[k], scan, spend, labels, nlabels);
      if (rc == CUDASP_OK) rc = cudasp_scanner_set_options(r->scanners[k], &b.opt);
      if (rc != CUDASP_OK) {
        pool_put(r);
        return host_fail(rc, "Failed to bind scanner on GPU %d: %s", lg, cudasp_last_error());
      }
    }
    // a pooled streaming feed rebound to keys or options the streaming scan
    // cannot run (too many label keys): back to the pool, and this query
    // takes per-slot launches like a new feed would (cudasp_stream_create's
    // CUDASP_ERR_INVALID_ARG below)
    if (r->stream && !cudasp_stream_supported(r->scanners[0])) {
      pool_put(r);
      r = nullptr;
      g.streaming_fallback = true;
    }
  }
  if (!r && g.streaming_fallback) {
    r = pool_take(device, cap_rows, g.launch_streams, 0);
    if (r) {
      for (int k = 0; k < r->nstreams; k++) {
        int rc = cudasp_scanner_set_keys(r->scanners[k], scan, spend, labels, nlabels);
        if (rc == CUDASP_OK) rc = cudasp_scanner_set_options(r->scanners[k], &b.opt);
        if (rc != CUDASP_OK) {
          pool_put(r);
          return host_fail(rc, "Failed to bind scanner on GPU %d: %s", lg, cudasp_last_error());
        }
      }
    }
  }
  if (!r) {
    r = new FeedRes();
    r->device = device;
    r->cap_rows = cap_rows;
    r->nstreams = g.streaming && !g.streaming_fallback ? 1 : g.launch_streams;
    for (int k = 0; k < FEED_MAX_STREAMS; k++) {
      if (k >= r->nstreams) break;
      int rc = cudasp_scanner_create(device, scan, spend, labels, nlabels, cap_rows, &r->scanners[k]);
      if (rc == CUDASP_OK) rc = cudasp_scanner_set_options(r->scanners[k], &b.opt);
      if (rc == CUDASP_OK && k == 0 && g.streaming && !g.streaming_fallback) {
        rc = cudasp_stream_create(r->scanners[0], blocks, &r->stream);
        if (rc == CUDASP_OK) {
          r->stream_blocks = blocks;
          r->stream_slots = feed_stream_slots();
        } else if (rc == CUDASP_ERR_INVALID_ARG) {  // a width the streaming kernel lacks: per-slot launches
          r->stream = nullptr;
          r->nstreams = g.launch_streams;
          rc = CUDASP_OK;
        }
      }
      if (rc != CUDASP_OK) {
        std::string msg = cudasp_last_error();
        release_res(r);
        return host_fail(rc, "Failed to create scanner on GPU %d: %s", lg, msg.c_str());
      }
    }
  }
  if (r->stream) (void)cudasp_stream_set_timeout(r->stream, stream_timeout_ms());
  auto f = std::make_unique<Feed>();
  if (const char* e = getenv("CUDASP_TF_TEST_LATE_SEQ")) {
    f->late_seq = atoll(e);
    const char* ms = getenv("CUDASP_TF_TEST_LATE_MS");
    f->late_s = 1e-3 * (ms ? atof(ms) : 1000.0);
  }
  f->res = r;
  f->g = &g;
  f->batch_size = b.batch_size;
  f->ow = out_words(b);
  f->words_per_row = 2.0 * f->ow;
  f->ramp = r->stream ? 5 : 3;
  if (const char* e = getenv("CUDASP_TF_RAMP")) f->ramp = std::max(0, std::min(atoi(e), 10));
  if (const char* e = getenv("CUDASP_TF_UPLOAD")) f->upload_null = strcmp(e, "stream") != 0;
  *out = f.get();
  g.feeds[lg] = std::move(f);
  g.feed_ptr[lg].store(*out, std::memory_order_release);
  return CUDASP_OK;
}

// The logical GPU of a thread's next chunk: round-robin from its assigned GPU.
int next_feed_index(const cudasp_tf_global& g, cudasp_tf_local& l) {
  const uint64_t c = l.chunks++;
  return g.num_gpus > 1 ? (int)((l.assigned_gpu + c) % (uint64_t)g.num_gpus) : 0;
}

// Row access for the two per-chunk input forms.  ChunkRows: cudasp_tf_chunk,
// DuckDB's unified form unpacked by the caller into per-row pointers, sizes
// and byte validity.  VectorRows: cudasp_tf_vectors, DuckDB's vectors as they
// are (16-byte string_t, selection vectors, 64-bit validity words,
// list_entry_t), so the extension passes pointers and nothing is marshalled
// per row before the slot copy.  Element k of the outputs child is addressed
// by list_offset + position in both forms (the child's own selection vector,
// if any, applies on top).
struct ChunkRows {
  const cudasp_tf_chunk& c;
  uint32_t count() const { return c.count; }
  bool dense() const { return !c.txid_valid && !c.height_valid && !c.tweak_valid && !c.list_valid && !c.child_valid; }
  bool row_ok(uint32_t i) const {
    return valid(c.txid_valid, i) && valid(c.height_valid, i) && valid(c.tweak_valid, i);
  }
  uint32_t txid_size(uint32_t i) const { return c.txid_size[i]; }
  const uint8_t* txid(uint32_t i) const { return c.txid_data[i]; }
  uint32_t tweak_size(uint32_t i) const { return c.tweak_size[i]; }
  const uint8_t* tweak(uint32_t i) const { return c.tweak_data[i]; }
  int32_t height(uint32_t i) const { return c.height[i]; }
  const int32_t* heights() const { return c.height; }  // the chunk's heights back to back
  bool list_ok(uint32_t i) const { return valid(c.list_valid, i); }
  uint64_t list_offset(uint32_t i) const { return c.list_offset[i]; }
  uint64_t list_length(uint32_t i) const { return c.list_length[i]; }
  bool child_ok(uint64_t k) const { return valid(c.child_valid, k); }
  int64_t child_value(uint64_t k) const { return c.child_values[k]; }
  const int64_t* child_values() const { return c.child_values; }  // element k at [k]
  bool has_child_blobs() const { return c.child_blob_data && c.child_blob_size; }
  const uint8_t* child_blob(uint64_t k, uint32_t* size) const {
    *size = c.child_blob_size[k];
    return c.child_blob_data[k];
  }
};

struct VectorRows {
  const cudasp_tf_vectors& v;
  static uint64_t at(const cudasp_tf_vector& x, uint64_t i) { return x.sel ? x.sel[i] : i; }
  static bool ok(const cudasp_tf_vector& x, uint64_t i) {
    if (!x.validity) return true;
    const uint64_t j = at(x, i);
    return (x.validity[j >> 6] >> (j & 63)) & 1u;
  }
  static const cudasp_tf_string& str(const cudasp_tf_vector& x, uint64_t i) {
    return static_cast<const cudasp_tf_string*>(x.data)[at(x, i)];
  }
  static const uint8_t* bytes(const cudasp_tf_string& s) {
    return s.length <= CUDASP_TF_STRING_INLINE ? s.prefix : s.ptr;  // inline bytes start at prefix
  }
  uint32_t count() const { return v.count; }
  bool dense() const {
    return !v.txid.validity && !v.height.validity && !v.tweak.validity && !v.outputs.validity && !v.child.validity;
  }
  bool row_ok(uint32_t i) const { return ok(v.txid, i) && ok(v.height, i) && ok(v.tweak, i); }
  uint32_t txid_size(uint32_t i) const { return str(v.txid, i).length; }
  const uint8_t* txid(uint32_t i) const { return bytes(str(v.txid, i)); }
  uint32_t tweak_size(uint32_t i) const { return str(v.tweak, i).length; }
  const uint8_t* tweak(uint32_t i) const { return bytes(str(v.tweak, i)); }
  int32_t height(uint32_t i) const { return static_cast<const int32_t*>(v.height.data)[at(v.height, i)]; }
  const int32_t* heights() const { return v.height.sel ? nullptr : static_cast<const int32_t*>(v.height.data); }
  const cudasp_tf_list_entry& list(uint32_t i) const {
    return static_cast<const cudasp_tf_list_entry*>(v.outputs.data)[at(v.outputs, i)];
  }
  bool list_ok(uint32_t i) const { return ok(v.outputs, i); }
  uint64_t list_offset(uint32_t i) const { return list(i).offset; }
  uint64_t list_length(uint32_t i) const { return list(i).length; }
  bool child_ok(uint64_t k) const { return ok(v.child, k); }
  int64_t child_value(uint64_t k) const { return static_cast<const int64_t*>(v.child.data)[at(v.child, k)]; }
  const int64_t* child_values() const { return v.child.sel ? nullptr : static_cast<const int64_t*>(v.child.data); }
  bool has_child_blobs() const { return v.child.data != nullptr; }
  const uint8_t* child_blob(uint64_t k, uint32_t* size) const {
    const cudasp_tf_string& s = str(v.child, k);
    *size = s.length;
    return bytes(s);
  }
};

// AccumulateInput (src/cudasp_extension.cu:154-224) for one DuckDB chunk:
// count and validate the rows (NULL txid/height/tweak rows skipped, NULL list
// = no outputs, NULL elements dropped, :195-221), reserve, copy, commit.
// A chunk without NULLs (no validity) and with int64 outputs: one pass to
// validate and count, then bulk copies where DuckDB's vectors are contiguous
// (heights; the list children when the lists are back to back).
template <class Rows>
int feed_chunk_dense(const cudasp_tf_bind_data& b, cudasp_tf_global& g, cudasp_tf_local& l, const Rows& c) {
  const uint32_t n = c.count();
  size_t nouts = 0, ntx = 0;
  const int64_t* cv = c.child_values();  // nullptr: the child vector has a selection vector
  bool lists_contiguous = cv != nullptr;
  bool txid32 = true;
  const uint64_t first = n ? c.list_offset(0) : 0;
  for (uint32_t i = 0; i < n; i++) {
    if (c.tweak_size(i) != TWEAK_KEY_SIZE)
      return host_fail(CUDASP_ERR_INVALID_ARG, "tweak_key must be exactly 64 bytes, got %u bytes", c.tweak_size(i));
    const uint32_t ts = c.txid_size(i);
    ntx += ts;
    txid32 &= ts == 32;
    const uint64_t len = c.list_length(i);
    lists_contiguous &= len == 0 || c.list_offset(i) == first + nouts;
    nouts += len;
  }
  if (nouts && !cv && !c.has_child_blobs()) return host_fail(CUDASP_ERR_INVALID_ARG, "missing outputs child values");
  Feed* f = nullptr;
  int rc = feed_for(g, b, next_feed_index(g, l), &f);
  if (rc != CUDASP_OK) return rc;
  Reservation res;
  const double t0 = now_s();
  const bool nt = slot_nt();
  txid32 = txid32 && nt;
  rc = feed_reserve(*f, n, nouts, ntx, &res, txid32 ? RES_TXID32 : 0);
  if (rc != CUDASP_OK) return rc;
  const double t1 = now_s();
  FeedSlot& s = *res.slot;
  const uint32_t r0 = res.row0;
  if (const int32_t* h = c.heights())
    memcpy(s.heights.data() + r0, h, (size_t)n * sizeof(int32_t));
  else
    for (uint32_t i = 0; i < n; i++) s.heights[r0 + i] = c.height(i);
  uint8_t* tw = s.h_tweaks + (size_t)r0 * TWEAK_KEY_SIZE;
  size_t tx = res.tx0;
  uint8_t* txb = s.txid_bytes.data();
  if (txid32) {
    // one pass per row: its 64-byte tweak blob and its 32-byte txid (a TxRun:
    // no per-row txid offset or size), non-temporal where aligned
    uint8_t* tb = txb + tx;
    const bool tb16 = ((uintptr_t)tb & 15) == 0;
    for (uint32_t i = 0; i < n; i++) {
      cudasp_host::nt_copy64(tw + (size_t)i * TWEAK_KEY_SIZE, c.tweak(i));
      if (tb16)
        cudasp_host::nt_copy32(tb + 32 * (size_t)i, c.txid(i));
      else
        memcpy(tb + 32 * (size_t)i, c.txid(i), 32);
    }
  } else if (nt) {
    // one pass per row: its 64-byte tweak blob, then its txid (32-byte txids
    // at 16-byte aligned offsets take non-temporal stores too)
    for (uint32_t i = 0; i < n; i++) {
      cudasp_host::nt_copy64(tw + (size_t)i * TWEAK_KEY_SIZE, c.tweak(i));
      const uint32_t sz = c.txid_size(i);
      s.txid_off[r0 + i] = tx;
      s.txid_size[r0 + i] = sz;
      if (sz == 32 && ((uintptr_t)(txb + tx) & 15) == 0)
        cudasp_host::nt_copy32(txb + tx, c.txid(i));
      else if (sz)
        memcpy(txb + tx, c.txid(i), sz);
      tx += sz;
    }
  } else {
    for (uint32_t i = 0; i < n; i++) memcpy(tw + (size_t)i * TWEAK_KEY_SIZE, c.tweak(i), TWEAK_KEY_SIZE);
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t sz = c.txid_size(i);
      s.txid_off[r0 + i] = tx;
      s.txid_size[r0 + i] = sz;
      if (sz) memcpy(txb + tx, c.txid(i), sz);
      tx += sz;
    }
  }
  size_t o = res.word0;  // one word per output (no full_x here)
  if (lists_contiguous) {
    if (nouts) {
      if (nt)
        cudasp_host::nt_copy(s.h_outputs + o, cv + first, nouts * sizeof(int64_t));
      else
        memcpy(s.h_outputs + o, cv + first, nouts * sizeof(int64_t));
    }
    // an empty list's offset is its position in the run, whatever DuckDB
    // stored for it
    if (nt) {
      // through a small buffer, so the slot's offsets and lengths are
      // written non-temporally too
      uint32_t bo[CUDASP_TF_VECTOR_SIZE], bl[CUDASP_TF_VECTOR_SIZE];
      size_t run = o;
      for (uint32_t i = 0; i < n; i++) {
        bo[i] = (uint32_t)run;
        bl[i] = (uint32_t)c.list_length(i);
        run += bl[i];
      }
      cudasp_host::nt_copy(s.h_offs + r0, bo, (size_t)n * 4);
      cudasp_host::nt_copy(s.h_lens + r0, bl, (size_t)n * 4);
    } else {
      size_t run = o;
      for (uint32_t i = 0; i < n; i++) {
        s.h_offs[r0 + i] = (uint32_t)run;
        s.h_lens[r0 + i] = (uint32_t)c.list_length(i);
        run += s.h_lens[r0 + i];
      }
    }
  } else {
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t len = (uint32_t)c.list_length(i);
      const uint64_t off = c.list_offset(i);
      s.h_offs[r0 + i] = (uint32_t)o;
      s.h_lens[r0 + i] = len;
      if (len && cv)
        memcpy(s.h_outputs + o, cv + off, (size_t)len * sizeof(int64_t));
      else
        for (uint32_t k = 0; k < len; k++) s.h_outputs[o + k] = c.child_value(off + k);
      o += len;
    }
  }
  if (nt) cudasp_host::slot_copy_fence();
  return feed_commit(*f, s, t1 - t0, now_s() - t1);
}

template <class Rows>
int feed_chunk(const cudasp_tf_bind_data& b, cudasp_tf_global& g, cudasp_tf_local& l, const Rows& c) {
  const size_t ow = out_words(b);
  const uint32_t count = c.count();
  if (b.opt.full_x && count > 0 && !c.has_child_blobs())
    return host_fail(CUDASP_ERR_INVALID_ARG, "full_x needs the outputs column as BLOB[] (child_blob_data)");
  if (!b.opt.full_x && c.dense()) return feed_chunk_dense(b, g, l, c);
  uint32_t nrows = 0;
  size_t nouts = 0, ntx = 0;
  for (uint32_t i = 0; i < count; i++) {
    if (!c.row_ok(i)) continue;
    if (c.tweak_size(i) != TWEAK_KEY_SIZE)
      return host_fail(CUDASP_ERR_INVALID_ARG, "tweak_key must be exactly 64 bytes, got %u bytes", c.tweak_size(i));
    nrows++;
    ntx += c.txid_size(i);
    if (!c.list_ok(i)) continue;
    const uint64_t off = c.list_offset(i), len = c.list_length(i);
    for (uint64_t k = 0; k < len; k++) {
      const uint64_t ci = off + k;
      if (!c.child_ok(ci)) continue;
      if (b.opt.full_x) {
        uint32_t sz;
        (void)c.child_blob(ci, &sz);
        if (sz != XONLY_SIZE)
          return host_fail(CUDASP_ERR_INVALID_ARG, "full_x outputs must be 32-byte x-only keys, got %u bytes", sz);
      }
      nouts++;
    }
  }
  if (nrows == 0) return CUDASP_OK;
  if (nouts && !b.opt.full_x && !c.child_values() && !c.has_child_blobs())
    return host_fail(CUDASP_ERR_INVALID_ARG, "missing outputs child values");
  Feed* f = nullptr;
  int rc = feed_for(g, b, next_feed_index(g, l), &f);
  if (rc != CUDASP_OK) return rc;
  Reservation res;
  const double t0 = now_s();
  rc = feed_reserve(*f, nrows, nouts * ow, ntx, &res);
  if (rc != CUDASP_OK) return rc;
  const double t1 = now_s();
  FeedSlot& s = *res.slot;
  uint32_t r = res.row0;
  size_t o = res.word0 / ow;  // output index
  size_t tx = res.tx0;
  for (uint32_t i = 0; i < count; i++) {
    if (!c.row_ok(i)) continue;
    const uint32_t ts = c.txid_size(i);
    s.txid_off[r] = tx;
    s.txid_size[r] = ts;
    if (ts) memcpy(s.txid_bytes.data() + tx, c.txid(i), ts);
    tx += ts;
    s.heights[r] = c.height(i);
    memcpy(s.h_tweaks + (size_t)r * TWEAK_KEY_SIZE, c.tweak(i), TWEAK_KEY_SIZE);
    s.h_offs[r] = (uint32_t)o;
    uint32_t len = 0;
    if (c.list_ok(i)) {
      const uint64_t off = c.list_offset(i), ll = c.list_length(i);
      for (uint64_t k = 0; k < ll; k++) {
        const uint64_t ci = off + k;
        if (!c.child_ok(ci)) continue;
        if (b.opt.full_x) {
          uint32_t sz;
          memcpy(s.h_outputs + o * ow, c.child_blob(ci, &sz), XONLY_SIZE);
        } else {
          s.h_outputs[o] = c.child_value(ci);
        }
        o++;
        len++;
      }
    }
    s.h_lens[r] = len;
    r++;
  }
  return feed_commit(*f, s, t1 - t0, now_s() - t1);
}

// Columnar rows [r0, r1) of `c` (Arrow layout, cudasp_tf_columns), same row
// rules as feed_chunk.  Without validity bitmaps and with 64-byte tweaks the
// four columns are appended with bulk copies.
int feed_columns(const cudasp_tf_bind_data& b, cudasp_tf_global& g, cudasp_tf_local& l, const cudasp_tf_columns& c,
                 uint64_t r0, uint64_t r1) {
  const uint64_t n = r1 - r0;
  const size_t ow = out_words(b);
  const int32_t* txo = c.txid_offsets + c.txid_offset;
  const int32_t* lo = c.list_offsets + c.list_offset;
  // full_x: the outputs child is binary (child_blob_offsets) or
  // fixed_size_binary(child_blob_fixed_width) of 32-byte x-only keys.
  auto child_blob = [&](uint64_t k, uint32_t* size) -> const uint8_t* {
    const uint64_t ck = c.child_offset + k;
    if (c.child_blob_offsets) {
      *size = (uint32_t)(c.child_blob_offsets[ck + 1] - c.child_blob_offsets[ck]);
      return c.child_blob_data + c.child_blob_offsets[ck];
    }
    *size = (uint32_t)c.child_blob_fixed_width;
    return c.child_blob_data + ck * (uint64_t)c.child_blob_fixed_width;
  };
  auto tweak_ptr = [&](uint64_t i, uint32_t* size) -> const uint8_t* {
    if (c.tweak_offsets) {
      const int32_t* to = c.tweak_offsets + c.tweak_offset;
      *size = (uint32_t)(to[i + 1] - to[i]);
      return c.tweak_data + to[i];
    }
    *size = (uint32_t)c.tweak_fixed_width;
    return c.tweak_data + (c.tweak_offset + i) * (uint64_t)c.tweak_fixed_width;
  };
  auto row_ok = [&](uint64_t i) {
    return bit(c.txid_validity, c.txid_offset + i) && bit(c.height_validity, c.height_offset + i) &&
           bit(c.tweak_validity, c.tweak_offset + i);
  };
  bool fast = !c.txid_validity && !c.height_validity && !c.tweak_validity && !c.list_validity && !c.child_validity;
  if (fast && c.tweak_offsets) {
    const int32_t* to = c.tweak_offsets + c.tweak_offset;
    fast = (uint64_t)(to[r1] - to[r0]) == n * TWEAK_KEY_SIZE;  // every value 64 bytes
  } else if (fast) {
    fast = c.tweak_fixed_width == (int32_t)TWEAK_KEY_SIZE;
  }
  if (fast && b.opt.full_x) {  // bulk copy only for fixed 32-byte keys
    fast = !c.child_blob_offsets && c.child_blob_fixed_width == (int32_t)XONLY_SIZE;
  }
  uint32_t nrows = 0;
  size_t nouts = 0, ntx = 0;
  if (fast) {
    nrows = (uint32_t)n;
    nouts = (size_t)(lo[r1] - lo[r0]);
    ntx = (size_t)(txo[r1] - txo[r0]);
  } else {
    for (uint64_t i = r0; i < r1; i++) {
      if (!row_ok(i)) continue;
      uint32_t tsize;
      (void)tweak_ptr(i, &tsize);
      if (tsize != TWEAK_KEY_SIZE)
        return host_fail(CUDASP_ERR_INVALID_ARG, "tweak_key must be exactly 64 bytes, got %u bytes", tsize);
      nrows++;
      ntx += (size_t)(txo[i + 1] - txo[i]);
      if (!bit(c.list_validity, c.list_offset + i)) continue;
      for (int64_t k = lo[i]; k < lo[i + 1]; k++) {
        if (!bit(c.child_validity, c.child_offset + (uint64_t)k)) continue;
        if (b.opt.full_x) {
          uint32_t sz;
          (void)child_blob((uint64_t)k, &sz);
          if (sz != XONLY_SIZE)
            return host_fail(CUDASP_ERR_INVALID_ARG, "full_x outputs must be 32-byte x-only keys, got %u bytes", sz);
        }
        nouts++;
      }
    }
  }
  if (nrows == 0) return CUDASP_OK;
  Feed* f = nullptr;
  int rc = feed_for(g, b, next_feed_index(g, l), &f);
  if (rc != CUDASP_OK) return rc;
  Reservation res;
  const double t0 = now_s();
  // every txid 32 bytes (a fixed_size_binary(32) column, or uniform binary):
  // the rows become a TxRun, no per-row txid offsets
  bool txid32 = fast && slot_nt() && ntx == 32 * (size_t)n;
  if (txid32)
    for (uint64_t i = r0; i < r1 && txid32; i++) txid32 = txo[i + 1] - txo[i] == 32;
  rc = feed_reserve(*f, nrows, nouts * ow, ntx, &res, txid32 ? RES_TXID32 : 0);
  if (rc != CUDASP_OK) return rc;
  const double t1 = now_s();
  FeedSlot& s = *res.slot;
  const uint32_t rbase = res.row0;
  const size_t obase = res.word0 / ow;
  if (fast) {
    uint32_t sz;
    const auto copy = slot_nt() ? cudasp_host::nt_copy : [](void* d, const void* src, size_t bytes) {
      memcpy(d, src, bytes);
    };
    copy(s.h_tweaks + (size_t)rbase * TWEAK_KEY_SIZE, tweak_ptr(r0, &sz), n * TWEAK_KEY_SIZE);
    memcpy(s.heights.data() + rbase, c.height + c.height_offset + r0, n * sizeof(int32_t));
    if (ntx) copy(s.txid_bytes.data() + res.tx0, c.txid_data + txo[r0], ntx);
    const uint64_t first = (uint64_t)lo[r0];
    if (nouts) {
      if (b.opt.full_x)
        copy(s.h_outputs + obase * ow, c.child_blob_data + (c.child_offset + first) * XONLY_SIZE, nouts * XONLY_SIZE);
      else
        copy(s.h_outputs + obase, c.child_values + c.child_offset + first, nouts * sizeof(int64_t));
    }
    if (!txid32)
      for (uint64_t i = r0; i < r1; i++) {
        const uint32_t row = rbase + (uint32_t)(i - r0);
        s.txid_off[row] = res.tx0 + (size_t)(txo[i] - txo[r0]);
        s.txid_size[row] = (uint32_t)(txo[i + 1] - txo[i]);
      }
    if (slot_nt()) {
      uint32_t bo[CUDASP_TF_VECTOR_SIZE], bl[CUDASP_TF_VECTOR_SIZE];
      for (uint64_t i = r0; i < r1; i++) {
        bo[i - r0] = (uint32_t)(obase + ((uint64_t)lo[i] - first));
        bl[i - r0] = (uint32_t)(lo[i + 1] - lo[i]);
      }
      cudasp_host::nt_copy(s.h_offs + rbase, bo, (size_t)n * 4);
      cudasp_host::nt_copy(s.h_lens + rbase, bl, (size_t)n * 4);
      cudasp_host::slot_copy_fence();
    } else {
      for (uint64_t i = r0; i < r1; i++) {
        const uint32_t row = rbase + (uint32_t)(i - r0);
        s.h_offs[row] = (uint32_t)(obase + ((uint64_t)lo[i] - first));
        s.h_lens[row] = (uint32_t)(lo[i + 1] - lo[i]);
      }
    }
    return feed_commit(*f, s, t1 - t0, now_s() - t1);
  }
  uint32_t r = rbase;
  size_t o = obase, tx = res.tx0;
  for (uint64_t i = r0; i < r1; i++) {
    if (!row_ok(i)) continue;
    uint32_t tsize;
    const uint8_t* tw = tweak_ptr(i, &tsize);
    const uint32_t tl = (uint32_t)(txo[i + 1] - txo[i]);
    s.txid_off[r] = tx;
    s.txid_size[r] = tl;
    if (tl) memcpy(s.txid_bytes.data() + tx, c.txid_data + txo[i], tl);
    tx += tl;
    s.heights[r] = c.height[c.height_offset + i];
    memcpy(s.h_tweaks + (size_t)r * TWEAK_KEY_SIZE, tw, TWEAK_KEY_SIZE);
    s.h_offs[r] = (uint32_t)o;
    uint32_t len = 0;
    if (bit(c.list_validity, c.list_offset + i)) {
      for (int64_t k = lo[i]; k < lo[i + 1]; k++) {
        if (!bit(c.child_validity, c.child_offset + (uint64_t)k)) continue;
        if (b.opt.full_x) {
          uint32_t sz;
          memcpy(s.h_outputs + o * ow, child_blob((uint64_t)k, &sz), XONLY_SIZE);
        } else {
          s.h_outputs[o] = c.child_values[c.child_offset + (uint64_t)k];
        }
        o++;
        len++;
      }
    }
    s.h_lens[r] = len;
    r++;
  }
  return feed_commit(*f, s, t1 - t0, now_s() - t1);
}

// Drain a query's feeds (work still in flight after an error or an aborted
// query) and park their resources in the pool.
void feeds_release(cudasp_tf_global& g) {
  for (auto& fp : g.feeds) {
    if (!fp) continue;
    Feed& f = *fp;
    FeedRes* r = f.res;
    {
      std::unique_lock<std::mutex> lk(f.mu);
      for (FeedSlot& s : r->slots) {
        while (s.state == SLOT_CLOSED || s.state == SLOT_BUSY) f.cv.wait(lk);
        s.state = SLOT_FREE;
        s.writers = 0;
        s.in_ring = false;
      }
    }
    // The resources go back to the pool when the device is done with them
    // cleanly, whether or not the query failed (a bad row, a wait that hit
    // its timeout); anything else releases them.
    bool ok = true;
    {
      DeviceSet dg(r->device);
      // a streaming feed's kernel runs until its stream is closed: close it
      // (an aborted query's published batches finish first), allowing the
      // drain at least the default timeout even when the query's own waits
      // had a shorter one -- a slow kernel ends and the feed is pooled; one
      // that never ends is abandoned and leaked (release_res)
      if (r->stream) {
        (void)cudasp_stream_set_timeout(r->stream, std::max<uint32_t>(stream_timeout_ms(), 60000u));
        ok = cudasp_stream_finish(r->stream) == CUDASP_OK;
        if (cudasp_stream_abandoned(r->stream)) {
          // its kernel may still run, reading the slots and writing the
          // scanner's scratch: free nothing and wait for nothing (a scanner
          // sync would wait on that kernel, possibly forever) -- release_res
          // leaks the feed
          fp.reset();
          release_res(r);
          continue;
        }
        free_stale(*r);
      }
      for (int k = 0; k < r->nstreams; k++) ok = cudasp_scanner_sync(r->scanners[k]) == CUDASP_OK && ok;
      // a launch that failed after queueing its uploads left them on the
      // null stream, still reading the slot's pinned buffers
      if (!ok || f.error != CUDASP_OK) (void)hipStreamSynchronize((hipStream_t)0);
    }
    fp.reset();
    if (ok)
      pool_put(r);
    else
      release_res(r);
  }
  g.feeds.clear();
}

}  // namespace

extern "C" {

int cudasp_tf_bind(uint32_t arg_count, cudasp_tf_blob_arg scan_private_key, cudasp_tf_blob_arg spend_public_key,
                   int label_keys_is_list, const cudasp_tf_blob_arg* label_keys, uint32_t label_count,
                   int has_batch_size, int batch_size_is_integer, int64_t batch_size, cudasp_tf_bind_data** out,
                   char* err, size_t err_cap) {
  if (out) *out = nullptr;
  if (arg_count != 4) {
    write_err(err, err_cap,
              "cudasp_scan requires 4 arguments: TABLE, scan_private_key BLOB, spend_public_key BLOB, and "
              "label_keys LIST[BLOB]");
    return CUDASP_ERR_INVALID_ARG;
  }
  if (!scan_private_key.is_blob) {
    write_err(err, err_cap, "Second argument must be a BLOB (32-byte scan_private_key)");
    return CUDASP_ERR_INVALID_ARG;
  }
  if (scan_private_key.size != SCALAR_SIZE) {
    write_err(err, err_cap, "scan_private_key must be exactly 32 bytes, got %llu bytes",
              (unsigned long long)scan_private_key.size);
    return CUDASP_ERR_INVALID_ARG;
  }
  if (!spend_public_key.is_blob) {
    write_err(err, err_cap, "Third argument must be a BLOB (64-byte spend_public_key)");
    return CUDASP_ERR_INVALID_ARG;
  }
  if (spend_public_key.size != TWEAK_KEY_SIZE) {
    write_err(err, err_cap, "spend_public_key must be exactly 64 bytes, got %llu bytes",
              (unsigned long long)spend_public_key.size);
    return CUDASP_ERR_INVALID_ARG;
  }
  if (!label_keys_is_list) {
    write_err(err, err_cap, "Fourth argument must be a LIST[BLOB] (label keys)");
    return CUDASP_ERR_INVALID_ARG;
  }
  for (uint32_t i = 0; i < label_count; i++) {
    if (!label_keys[i].is_blob) {
      write_err(err, err_cap, "All elements in label_keys must be BLOBs");
      return CUDASP_ERR_INVALID_ARG;
    }
    if (label_keys[i].size != TWEAK_KEY_SIZE) {
      write_err(err, err_cap, "Each label key must be exactly 64 bytes, got %llu bytes",
                (unsigned long long)label_keys[i].size);
      return CUDASP_ERR_INVALID_ARG;
    }
  }
  uint64_t bs = CUDASP_TF_DEFAULT_BATCH;
  if (has_batch_size) {
    if (!batch_size_is_integer) {
      write_err(err, err_cap, "batch_size parameter must be an INTEGER");
      return CUDASP_ERR_INVALID_ARG;
    }
    if (batch_size <= 0) {
      write_err(err, err_cap, "batch_size must be positive, got %lld", (long long)batch_size);
      return CUDASP_ERR_INVALID_ARG;
    }
    if (batch_size > 10000000) {
      write_err(err, err_cap, "batch_size too large (max 10,000,000), got %lld", (long long)batch_size);
      return CUDASP_ERR_INVALID_ARG;
    }
    bs = (uint64_t)batch_size;
  }
  auto* b = new cudasp_tf_bind_data();
  b->batch_size = bs;
  b->scan_private_key_data.assign((const char*)scan_private_key.data, SCALAR_SIZE);
  b->spend_public_key_data.assign((const char*)spend_public_key.data, TWEAK_KEY_SIZE);
  for (uint32_t i = 0; i < label_count; i++) {
    b->label_keys_data.emplace_back((const char*)label_keys[i].data, TWEAK_KEY_SIZE);
    b->label_keys_flat.append((const char*)label_keys[i].data, TWEAK_KEY_SIZE);
  }
  *out = b;
  return CUDASP_OK;
}

int cudasp_tf_bind_options(cudasp_tf_bind_data* b, int has_output_count, int64_t output_count,
                           int has_label_negation, int label_negation, int has_full_x, int full_x, char* err,
                           size_t err_cap) {
  if (!b) {
    write_err(err, err_cap, "null bind data");
    return CUDASP_ERR_INVALID_ARG;
  }
  cudasp_scan_options o = b->opt;
  if (has_output_count) {
    if (output_count < 1 || output_count > CUDASP_MAX_OUTPUT_COUNT) {
      write_err(err, err_cap, "output_count must be between 1 and %d, got %lld", CUDASP_MAX_OUTPUT_COUNT,
                (long long)output_count);
      return CUDASP_ERR_INVALID_ARG;
    }
    o.output_count = (uint32_t)output_count;
  }
  if (has_label_negation) o.label_negation = label_negation ? 1u : 0u;
  if (has_full_x) o.full_x = full_x ? 1u : 0u;
  b->opt = o;
  return CUDASP_OK;
}

void cudasp_tf_bind_free(cudasp_tf_bind_data* b) { delete b; }

uint64_t cudasp_tf_bind_batch_size(const cudasp_tf_bind_data* b) { return b ? b->batch_size : 0; }

int cudasp_tf_init(const cudasp_tf_bind_data* b, cudasp_tf_global** out) {
  if (!b || !out) return host_fail(CUDASP_ERR_INVALID_ARG, "null argument");
  auto* g = new cudasp_tf_global();
  ST_HOST(110, 0, 0);
  if (tf_device_map(g->device_map) != CUDASP_OK) {
    delete g;
    return CUDASP_ERR_INVALID_ARG;
  }
  g->num_gpus = (int)g->device_map.size();
  g->bind = b;
  if (const char* e = getenv("CUDASP_TF_NULL_DEVICE")) g->null_device = atoi(e) != 0;
  const char* hq = getenv("GPU_MAX_HW_QUEUES");
  g->hw_queues = hq && atoi(hq) > 0 ? atoi(hq) : 4;
  int feeds_per_device = 0;
  for (int d : g->device_map) {
    int m = 0;
    for (int e : g->device_map) m += e == d;
    feeds_per_device = std::max(feeds_per_device, m);
  }
  g->feed_streams = feed_streams_for(b->batch_size, g->hw_queues, feeds_per_device);
  g->launch_streams = g->feed_streams;
  {
    const char* mode = getenv("CUDASP_TF_MODE");
    // one feed per device: a persistent kernel holds its hardware queue for
    // the whole query, so two feeds' kernels on one device could land on one
    // queue (HIP shares queues among streams) and the second would wait for
    // the first to end -- logical GPUs sharing a device (CUDASP_TF_DEVICE_MAP)
    // take the per-slot launches
    // (CUDASP_TF_MODE=stream forces streaming feeds even then -- each
    // kernel gets its share of the device's wave slots -- for rehearsing
    // the N-GPU host on one card with GPU_MAX_HW_QUEUES above the feeds)
    const bool force = mode && !strcmp(mode, "stream");
    g->streaming = !(mode && !strcmp(mode, "launch")) && b->opt.output_count <= CUDASP_STREAM_MAX_OUTPUT_COUNT &&
                   (feeds_per_device == 1 || force);
    if (g->streaming) g->feed_streams = 1;
  }
  g->feeds.resize(g->num_gpus);
  g->feed_ptr.reset(new std::atomic<Feed*>[g->num_gpus]);
  for (int lg = 0; lg < g->num_gpus; lg++) g->feed_ptr[lg].store(nullptr);
  g->feed_create_mu.reset(new std::mutex[g->num_gpus]);
  // The HIP runtime maps a process's streams on a device onto
  // GPU_MAX_HW_QUEUES hardware queues (4 unless set before HIP initialises),
  // one of them the null stream's; streams sharing a queue serialize their
  // kernels.  Report the setting and warn when this query's streams on one
  // device exceed the queues left (only with CUDASP_TF_STREAMS set).
  for (int lg = 0; lg < g->num_gpus; lg++) {
    int on_dev = 0;
    for (int d : g->device_map) on_dev += d == g->device_map[lg] ? g->feed_streams : 0;
    if (on_dev > g->max_streams_per_device) g->max_streams_per_device = on_dev;
  }
  static std::atomic<bool> warned{false};
  if (g->max_streams_per_device > g->hw_queues - 1 && !warned.exchange(true))
    fprintf(stderr,
            "cudasp_scan: %d streams per device exceed the %d hardware queues GPU_MAX_HW_QUEUES=%d leaves beside the "
            "null stream; streams that share a hardware queue run their kernels one after another\n",
            g->max_streams_per_device, g->hw_queues - 1, g->hw_queues);
  *out = g;
  return CUDASP_OK;
}

void cudasp_tf_global_free(cudasp_tf_global* g) {
  if (!g) return;
  feeds_release(*g);
  delete g;
}

int cudasp_tf_num_gpus(const cudasp_tf_global* g) { return g ? g->num_gpus : 0; }

int cudasp_tf_get_stats(cudasp_tf_global* g, cudasp_tf_stats* out) {
  if (!g || !out) return host_fail(CUDASP_ERR_INVALID_ARG, "null argument");
  memset(out, 0, sizeof(*out));
  out->streams_per_feed = (uint32_t)g->feed_streams;
  out->max_streams_per_device = (uint32_t)g->max_streams_per_device;
  out->hw_queues = (uint32_t)g->hw_queues;
  for (auto& fp : g->feeds) {
    if (!fp) continue;
    std::lock_guard<std::mutex> lock(fp->mu);
    out->feeds++;
    out->streaming_feeds += fp->res->stream ? 1u : 0u;
    out->launches += fp->launches;
    out->rows += fp->rows;
    out->harvest_wait_s += fp->harvest_wait_s;
    out->reserve_s += fp->reserve_s;
    out->copy_s += fp->copy_s;
    out->launch_s += fp->launch_s;
  }
  return CUDASP_OK;
}

int cudasp_tf_local_init(cudasp_tf_global* g, cudasp_tf_local** out) {
  if (!g || !out) return host_fail(CUDASP_ERR_INVALID_ARG, "null argument");
  g->currently_adding++;
  auto* l = new cudasp_tf_local();
  // Round-robin per thread (src/cudasp_extension.cu:523-529): the logical GPU
  // of the thread's first chunk; later chunks continue round-robin.
  l->assigned_gpu = g->num_gpus > 1 ? (int)cudasp_assign_gpu((uint64_t)g->next_gpu_assignment.fetch_add(1),
                                                             (uint32_t)g->num_gpus)
                                    : 0;
  l->device = g->device_map.empty() ? l->assigned_gpu : g->device_map[l->assigned_gpu];
  *out = l;
  return CUDASP_OK;
}

void cudasp_tf_local_free(cudasp_tf_local* l) { delete l; }

int cudasp_tf_local_gpu(const cudasp_tf_local* l) { return l ? l->assigned_gpu : -1; }

int cudasp_tf_local_device(const cudasp_tf_local* l) { return l ? l->device : -1; }

uint32_t cudasp_assign_gpu(uint64_t ordinal, uint32_t num_gpus) {
  return num_gpus > 1 ? (uint32_t)(ordinal % num_gpus) : 0u;
}

int cudasp_tf_prewarm(uint64_t batch_size, double* seconds) {
  const auto t0 = std::chrono::steady_clock::now();
  if (seconds) *seconds = 0;
  if (batch_size == 0) batch_size = CUDASP_TF_DEFAULT_BATCH;
  if (batch_size > 10000000) return host_fail(CUDASP_ERR_INVALID_ARG, "batch_size too large (max 10,000,000)");
  std::vector<int> map;
  int rc = tf_device_map(map);
  if (rc != CUDASP_OK) return rc;
  if (cudasp_device_count() <= 0) return host_fail(CUDASP_ERR_NO_DEVICE, "no GPU");
  // the default query shape: one streaming feed per device (cudasp_tf_init)
  int feeds_per_device = 0;
  for (int d : map) feeds_per_device = std::max(feeds_per_device, (int)std::count(map.begin(), map.end(), d));
  const char* mode = getenv("CUDASP_TF_MODE");
  if ((mode && !strcmp(mode, "launch")) || (feeds_per_device > 1 && !(mode && !strcmp(mode, "stream"))))
    return host_fail(CUDASP_ERR_INVALID_ARG, "prewarm covers streaming feeds (one feed per device)");
  // placeholder keys, rebound by the query that takes the feed: d = 1, B = G
  uint8_t scan[32] = {1};
  uint8_t spend[64];
  static const uint8_t gx[32] = {0x98, 0x17, 0xF8, 0x16, 0x5B, 0x81, 0xF2, 0x59, 0xD9, 0x28, 0xCE,
                                 0x2D, 0xDB, 0xFC, 0x9B, 0x02, 0x07, 0x0B, 0x87, 0xCE, 0x95, 0x62,
                                 0xA0, 0x55, 0xAC, 0xBB, 0xDC, 0xF9, 0x7E, 0x66, 0xBE, 0x79};
  static const uint8_t gy[32] = {0xB8, 0xD4, 0x10, 0xFB, 0x8F, 0xD0, 0x47, 0x9C, 0x19, 0x54, 0x85,
                                 0xA6, 0x48, 0xB4, 0x17, 0xFD, 0xA8, 0x08, 0x11, 0x0E, 0xFC, 0xFB,
                                 0xA4, 0x5D, 0x65, 0xC4, 0xA3, 0x26, 0x77, 0xDA, 0x3A, 0x48};
  memcpy(spend, gx, 32);
  memcpy(spend + 32, gy, 32);
  const uint32_t cap_rows = (uint32_t)(batch_size + CUDASP_TF_VECTOR_SIZE);
  // the logical GPUs' feeds in parallel (each device's table build, scanner,
  // stream and pinned slots are independent)
  std::vector<int> rcs(map.size(), CUDASP_OK);
  std::vector<std::string> msgs(map.size());
  auto warm_one = [&](size_t lg) {
    const int device = map[lg];
    const uint32_t blocks = stream_blocks_for(device, map);
    {
      std::lock_guard<std::mutex> lock(g_pool_mu);
      for (FeedRes* r : g_pool)
        if (r->device == device && r->cap_rows == cap_rows && r->nstreams == 1 && r->stream &&
            r->stream_blocks == blocks)
          return;  // already warm
    }
    DeviceSet dg(device);
    auto* r = new FeedRes();
    r->device = device;
    r->cap_rows = cap_rows;
    r->nstreams = 1;
    int e = cudasp_scanner_create(device, scan, spend, nullptr, 0, cap_rows, &r->scanners[0]);
    if (e == CUDASP_OK) e = cudasp_stream_create(r->scanners[0], blocks, &r->stream);
    if (e == CUDASP_OK) {
      r->stream_blocks = blocks;
      r->stream_slots = feed_stream_slots();
      // every slot with the capacity a first query opens it with (2 outputs
      // and 32 txid bytes per row; grown later like any slot)
      for (int k = 0; k < r->stream_slots && e == CUDASP_OK; k++)
        e = prepare_slot_streaming(*r, r->slots[k], (size_t)cap_rows * 2, (size_t)cap_rows * 32);
    }
    if (e != CUDASP_OK) {
      rcs[lg] = e;
      msgs[lg] = cudasp_last_error();
      release_res(r);
      return;
    }
    pool_put(r);
  };
  {
    std::vector<std::thread> th;
    for (size_t lg = 0; lg < map.size(); lg++) th.emplace_back(warm_one, lg);
    for (auto& t : th) t.join();
  }
  for (size_t lg = 0; lg < map.size(); lg++)
    if (rcs[lg] != CUDASP_OK)
      return host_fail(rcs[lg], "prewarm of GPU %zu (device %d): %s", lg, map[lg], msgs[lg].c_str());
  // One placeholder row through every parked feed, as a query would send it
  // (bind, a feed taken from the pool, its keys rebound, a batch published to
  // its streaming kernel, harvest, the feed parked again): the launch path's
  // first-time costs are paid here, not by the first query.
  {
    cudasp_tf_blob_arg a_scan{scan, 32, 1}, a_spend{spend, 64, 1};
    cudasp_tf_bind_data* bd = nullptr;
    char err[256];
    rc = cudasp_tf_bind(4, a_scan, a_spend, 1, nullptr, 0, 1, 1, (int64_t)batch_size, &bd, err, sizeof(err));
    if (rc != CUDASP_OK) return host_fail(rc, "prewarm bind: %s", err);
    cudasp_tf_global* g = nullptr;
    rc = cudasp_tf_init(bd, &g);
    std::vector<cudasp_tf_local*> ls;
    const uint8_t* txp = gx;
    const uint32_t txs = 32, tws = 64;
    const int32_t h = 0;
    const uint64_t lo = 0, ll = 1;
    const int64_t v = 0;
    const uint8_t* twp = spend;  // any 64-byte point: G
    cudasp_tf_chunk c{};
    c.count = 1;
    c.txid_data = &txp;
    c.txid_size = &txs;
    c.height = &h;
    c.tweak_data = &twp;
    c.tweak_size = &tws;
    c.list_offset = &lo;
    c.list_length = &ll;
    c.child_values = &v;
    for (size_t lg = 0; rc == CUDASP_OK && lg < map.size(); lg++) {
      cudasp_tf_local* l = nullptr;
      rc = cudasp_tf_local_init(g, &l);  // logical GPUs dealt round-robin
      if (rc == CUDASP_OK) {
        ls.push_back(l);
        rc = cudasp_tf_function(bd, g, l, &c);
        if (rc == CUDASP_TF_NEED_MORE_INPUT) rc = CUDASP_OK;
      }
    }
    auto* out = new cudasp_tf_output;
    for (cudasp_tf_local* l : ls) {
      while (rc == CUDASP_OK) {
        const int f = cudasp_tf_final(bd, g, l, out);
        if (f < 0) rc = f;
        if (f != CUDASP_TF_HAVE_MORE_OUTPUT) break;
      }
    }
    delete out;
    const std::string msg = rc == CUDASP_OK ? "" : cudasp_last_error();
    for (cudasp_tf_local* l : ls) cudasp_tf_local_free(l);
    cudasp_tf_global_free(g);
    cudasp_tf_bind_free(bd);
    if (rc != CUDASP_OK) return host_fail(rc, "prewarm query: %s", msg.c_str());
  }
  if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return CUDASP_OK;
}

void cudasp_tf_release_pool(void) {
  std::vector<FeedRes*> all;
  {
    std::lock_guard<std::mutex> lock(g_pool_mu);
    all.swap(g_pool);
  }
  for (FeedRes* r : all) release_res(r);
  // the pool held the last queries' keys: drop the cached scan-key digits too
  cudasp_internal_clear_key_cache();
}

uint32_t cudasp_tf_pool_size(void) {
  std::lock_guard<std::mutex> lock(g_pool_mu);
  return (uint32_t)g_pool.size();
}

int cudasp_tf_function(const cudasp_tf_bind_data* b, cudasp_tf_global* g, cudasp_tf_local* l,
                       const cudasp_tf_chunk* chunk) {
  if (!b || !g || !l || !chunk) return host_fail(CUDASP_ERR_INVALID_ARG, "null argument");
  // The batch slots hold batch_size + one vector of rows (a slot closes once
  // it holds >= batch_size), so a chunk may not exceed one vector.
  if (chunk->count > CUDASP_TF_VECTOR_SIZE)
    return host_fail(CUDASP_ERR_INVALID_ARG, "chunk of %u rows exceeds the vector size %d", chunk->count,
                     CUDASP_TF_VECTOR_SIZE);
  if (chunk->count > 0) {
    const int rc = feed_chunk(*b, *g, *l, ChunkRows{*chunk});
    if (rc != CUDASP_OK) return rc;
  }
  return CUDASP_TF_NEED_MORE_INPUT;
}

int cudasp_tf_function_vectors(const cudasp_tf_bind_data* b, cudasp_tf_global* g, cudasp_tf_local* l,
                               const cudasp_tf_vectors* vectors) {
  if (!b || !g || !l || !vectors) return host_fail(CUDASP_ERR_INVALID_ARG, "null argument");
  const cudasp_tf_vectors& v = *vectors;
  if (v.count > CUDASP_TF_VECTOR_SIZE)
    return host_fail(CUDASP_ERR_INVALID_ARG, "chunk of %u rows exceeds the vector size %d", v.count,
                     CUDASP_TF_VECTOR_SIZE);
  if (v.count == 0) return CUDASP_TF_NEED_MORE_INPUT;
  if (!v.txid.data || !v.height.data || !v.tweak.data || !v.outputs.data)
    return host_fail(CUDASP_ERR_INVALID_ARG, "missing column vector");
  const int rc = feed_chunk(*b, *g, *l, VectorRows{v});
  if (rc != CUDASP_OK) return rc;
  return CUDASP_TF_NEED_MORE_INPUT;
}

int cudasp_tf_function_columns(const cudasp_tf_bind_data* b, cudasp_tf_global* g, cudasp_tf_local* l,
                               const cudasp_tf_columns* cols) {
  if (!b || !g || !l || !cols) return host_fail(CUDASP_ERR_INVALID_ARG, "null argument");
  const cudasp_tf_columns& c = *cols;
  if (c.count > 0 && (!c.txid_offsets || !c.txid_data || !c.height || !c.tweak_data || !c.list_offsets ||
                      (!c.tweak_offsets && c.tweak_fixed_width <= 0)))
    return host_fail(CUDASP_ERR_INVALID_ARG, "missing column buffer");
  if (c.count > 0 && c.list_offsets[c.list_offset + c.count] > c.list_offsets[c.list_offset]) {
    // the outputs child: int64 values, or with full_x 32-byte keys
    const bool ok = b->opt.full_x ? (c.child_blob_data && (c.child_blob_offsets || c.child_blob_fixed_width > 0))
                                  : c.child_values != nullptr;
    if (!ok)
      return host_fail(CUDASP_ERR_INVALID_ARG, b->opt.full_x ? "full_x needs the outputs child as binary (child_blob_*)"
                                                              : "missing outputs child values");
  }
  // DuckDB-sized pieces, each fed like one chunk.
  for (uint64_t r0 = 0; r0 < c.count; r0 += CUDASP_TF_VECTOR_SIZE) {
    const uint64_t r1 = r0 + CUDASP_TF_VECTOR_SIZE < c.count ? r0 + CUDASP_TF_VECTOR_SIZE : c.count;
    const int rc = feed_columns(*b, *g, *l, c, r0, r1);
    if (rc != CUDASP_OK) return rc;
  }
  return CUDASP_TF_NEED_MORE_INPUT;
}

int cudasp_tf_final(const cudasp_tf_bind_data* b, cudasp_tf_global* g, cudasp_tf_local* l, cudasp_tf_output* out) {
  if (!b || !g || !l || !out) return host_fail(CUDASP_ERR_INVALID_ARG, "null argument");
  out->count = 0;
  if (!l->finalized) {
    ST_HOST(114, 0, 0);
    // A thread's rows are already in the device feeds.  The last thread to
    // finish launches every feed's partial slot, waits for all of them and
    // becomes the output thread (:554-624: the last thread emits).
    uint64_t remaining;
    {
      std::lock_guard<std::mutex> lock(g->finalize_lock);
      remaining = --g->currently_adding;
      l->finalized = true;
    }
    if (remaining != 0) return CUDASP_TF_FINISHED;
    bool expected = false;
    if (!g->output_thread_claimed.compare_exchange_strong(expected, true)) return CUDASP_TF_FINISHED;
    l->is_output_thread = true;
    const int rc = feeds_flush(*g);
    if (rc != CUDASP_OK) return rc;
  }
  if (!l->is_output_thread) return CUDASP_TF_FINISHED;
  size_t total = g->output_txids.size();
  if (g->output_position < total) {
    size_t cnt = total - g->output_position;
    if (cnt > CUDASP_TF_VECTOR_SIZE) cnt = CUDASP_TF_VECTOR_SIZE;
    for (size_t i = 0; i < cnt; i++) {
      size_t k = g->output_position + i;
      out->txid_data[i] = (const uint8_t*)g->output_txids[k].data();
      out->txid_size[i] = (uint32_t)g->output_txids[k].size();
      out->height[i] = g->output_heights[k];
      out->tweak_data[i] = (const uint8_t*)g->output_tweak_keys[k].data();
      out->tweak_size[i] = (uint32_t)g->output_tweak_keys[k].size();
    }
    out->count = (uint32_t)cnt;
    g->output_position += cnt;
    if (g->output_position < total) return CUDASP_TF_HAVE_MORE_OUTPUT;
  }
  return CUDASP_TF_FINISHED;
}

}  // extern "C"
