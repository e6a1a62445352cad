// Pinned tables (include/cudasp_host.h, cudasp_pinned_*): a tweak table copied
// once into coherent pinned host memory and scanned in place by the streaming
// kernel (cudasp_stream_*, include/cudasp_abi.h) for every query.
//
// The reference re-reads every row of every query into per-thread strings
// (src/cudasp_extension.cu:188-223) and copies each batch into managed buffers
// (:327-337, src/cudasp_gpu.cu:705-761); the table-function host of this
// library (cudasp_host.cpp) still copies each chunk into its batch slots, the
// host's cost per row.  Here a scan only publishes the
// pinned batches: the kernel reads the 64-byte tweak blobs, the outputs and
// their Arrow list offsets (cudasp_stream_batch.output_lengths NULL) over PCIe
// and writes the matching row indices back.  Same algorithm as the Python
// cudasp_amd.PinnedTable, without the interpreter in the publish loop.
//
// Placement CUDASP_TABLE_HBM keeps the batches resident in device memory
// instead, in k_scan_multi's layout (tweak x / y columns, the outputs CSR with
// per-row offsets and lengths), and a scan is one cudasp_scan_device_batches
// launch per logical GPU over all of its batches: the device-resident rate of
// bench.py's headline, for a table that fits in HBM (~93 B per row with 2
// outputs; 288 GB per MI355X).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/cudasp_abi.h"
#include "../../../include/cudasp_host.h"
#include "bind_data.hpp"

extern "C" void cudasp_internal_set_error(const char* msg);
extern "C" void* cudasp_internal_scanner_stream(cudasp_scanner* s);

namespace {

constexpr uint64_t TWEAK_KEY_SIZE = 64;      // CudaspScanBindData::TWEAK_KEY_SIZE
constexpr uint64_t MAX_BATCH = 10000000;     // CudaspScanBind's batch_size limit (:474-487)
constexpr uint64_t STREAM_RING = 64;         // batches published and not yet harvested, per stream
constexpr uint64_t MAX_WORDS = 0xFFFFFFFFu;  // a batch's outputs: u32 offsets

// Test hooks, read at cudasp_pinned_create:
//   CUDASP_TF_NULL_DEVICE=1           batches in plain host memory, no device
//                                     call (appends testable without a GPU;
//                                     a scan fails with CUDASP_ERR_NO_DEVICE)
//   CUDASP_PINNED_TEST_MAX_WORDS=w    a batch's outputs capped at w words
//                                     instead of 2^32 - 1 (the early close)
//   CUDASP_PINNED_TEST_SEAL_FAIL=k    the table's k-th batch close (1-based)
//                                     fails as an allocation would (the
//                                     append's rollback)
bool env_null_device() {
  const char* e = getenv("CUDASP_TF_NULL_DEVICE");
  return e && atoi(e) == 1;
}
uint64_t env_seal_fail() {
  const char* e = getenv("CUDASP_PINNED_TEST_SEAL_FAIL");
  const long long v = e ? atoll(e) : 0;
  return v > 0 ? (uint64_t)v : 0;
}
uint64_t env_max_words() {
  const char* e = getenv("CUDASP_PINNED_TEST_MAX_WORDS");
  const long long v = e ? atoll(e) : 0;
  return v > 0 && (uint64_t)v < MAX_WORDS ? (uint64_t)v : MAX_WORDS;
}

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  cudasp_internal_set_error(buf);
  return code;
}

inline bool bit(const uint8_t* bm, uint64_t i) { return bm == nullptr || ((bm[i >> 3] >> (i & 7)) & 1u); }

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

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

// One closed batch: pinned rows, outputs, Arrow offsets (n + 1) and match
// indices, a device mirror of its outputs, and the input numbers of its rows.
struct Batch {
  uint32_t n = 0;
  uint64_t words = 0;
  uint8_t* rows = nullptr;
  int64_t* outputs = nullptr;
  uint32_t* offsets = nullptr;
  uint32_t* matches = nullptr;
  int64_t* d_mirror = nullptr;
  int device = 0;
  uint32_t lg = 0;
  bool host_mem = false;      // null-device table: malloc'd, no mirror
  // CUDASP_TABLE_HBM: the batch on its device (no pinned buffers)
  uint32_t* d_x = nullptr;
  uint32_t* d_y = nullptr;
  int64_t* d_out = nullptr;
  uint32_t* d_offs = nullptr;
  uint32_t* d_lens = nullptr;
  uint8_t* d_flags = nullptr;
  uint32_t* d_rows = nullptr;
  uint64_t ord0 = 0;          // input number of row 0
  std::vector<uint64_t> ord;  // every row's input number, when rows were skipped (else ord0 + r)
  uint64_t number(uint32_t r) const { return ord.empty() ? ord0 + r : ord[r]; }
};

// The open batch, in pageable memory until it closes.
struct Staging {
  std::vector<uint8_t> rows;
  std::vector<int64_t> outputs;
  std::vector<uint32_t> offsets{0};
  std::vector<uint64_t> ord;
  bool dense = true;  // ord[r] == ord[0] + r
  uint64_t n() const { return ord.size(); }
};

struct Shape {
  uint32_t labels = 0, output_count = 0, negation = 0;
  bool operator==(const Shape& o) const {
    return labels == o.labels && output_count == o.output_count && negation == o.negation;
  }
};

}  // namespace

struct cudasp_pinned_table {
  uint64_t batch_size = CUDASP_TF_DEFAULT_BATCH;
  std::vector<int> devices;  // per logical GPU
  std::vector<uint32_t> blocks;
  std::vector<Batch> batches;
  Staging open;
  uint64_t appended = 0, pinned_rows = 0, pinned_bytes = 0;
  std::vector<cudasp_scanner*> scanners;
  std::vector<cudasp_stream*> streams;
  bool stream_ok = false;
  Shape shape;
  bool abandoned = false;  // a scan's kernel outlived its timeout: never free what it may touch
  bool host_only = false;  // CUDASP_TF_NULL_DEVICE
  bool hbm = false;        // CUDASP_TABLE_HBM
  uint64_t device_bytes = 0;
  std::vector<uint32_t*> d_counts;  // HBM: per logical GPU, one match count per batch
  std::vector<size_t> counts_cap;
  uint64_t max_words = MAX_WORDS;
  uint64_t seals = 0, seal_fail_at = 0;  // test hook CUDASP_PINNED_TEST_SEAL_FAIL
  uint64_t last_matches = 0;
  double last_scan_s = 0, last_publish_s = 0;
  mutable std::mutex mu;
};

namespace {

void free_batch(Batch& b) {
  if (b.host_mem) {
    free(b.rows);
    free(b.outputs);
    free(b.offsets);
    free(b.matches);
    b = Batch();
    return;
  }
  if (b.d_mirror || b.d_x) {
    DeviceSet ds(b.device);
    for (void* p : {(void*)b.d_mirror, (void*)b.d_x, (void*)b.d_y, (void*)b.d_out, (void*)b.d_offs, (void*)b.d_lens,
                    (void*)b.d_flags, (void*)b.d_rows})
      if (p) (void)hipFree(p);
  }
  cudasp_host_free(b.rows);
  cudasp_host_free(b.outputs);
  cudasp_host_free(b.offsets);
  cudasp_host_free(b.matches);
  b = Batch();
}

void reset_staging(cudasp_pinned_table& t) {
  Staging& s = t.open;
  s.rows.clear();
  s.outputs.clear();
  s.offsets.assign(1, 0);
  s.ord.clear();
  s.dense = true;
}

// CUDASP_TABLE_HBM: the open batch uploaded in k_scan_multi's layout (the
// blobs transposed on the device into x / y columns; per-row offsets and
// lengths from the Arrow offsets).
int seal_hbm(cudasp_pinned_table& t, Batch& b, size_t wb) {
  Staging& s = t.open;
  const uint64_t n = b.n;
  DeviceSet ds(b.device);
  std::vector<uint32_t> lens(n);
  for (uint64_t r = 0; r < n; r++) lens[r] = s.offsets[r + 1] - s.offsets[r];
  uint8_t* d_tmp = nullptr;
  // the uploads and the transpose on a private non-blocking stream, waited
  // for alone: an append does not wait for other work on the device (another
  // table's or query's persistent streaming kernel runs until its close)
  hipStream_t st = nullptr;
  bool ok = hipStreamCreateWithFlags(&st, hipStreamNonBlocking) == hipSuccess &&
            hipMalloc((void**)&b.d_x, n * 32) == hipSuccess && hipMalloc((void**)&b.d_y, n * 32) == hipSuccess &&
            hipMalloc((void**)&b.d_out, wb) == hipSuccess && hipMalloc((void**)&b.d_offs, n * 4) == hipSuccess &&
            hipMalloc((void**)&b.d_lens, n * 4) == hipSuccess && hipMalloc((void**)&b.d_flags, n) == hipSuccess &&
            hipMalloc((void**)&b.d_rows, n * 4) == hipSuccess && hipMalloc((void**)&d_tmp, n * TWEAK_KEY_SIZE) == hipSuccess;
  ok = ok && hipMemcpyAsync(d_tmp, s.rows.data(), n * TWEAK_KEY_SIZE, hipMemcpyHostToDevice, st) == hipSuccess &&
       (b.words == 0 || hipMemcpyAsync(b.d_out, s.outputs.data(), b.words * 8, hipMemcpyHostToDevice, st) == hipSuccess) &&
       hipMemcpyAsync(b.d_offs, s.offsets.data(), n * 4, hipMemcpyHostToDevice, st) == hipSuccess &&
       hipMemcpyAsync(b.d_lens, lens.data(), n * 4, hipMemcpyHostToDevice, st) == hipSuccess;
  if (ok) ok = cudasp_tweaks_to_columns(d_tmp, (uint32_t)n, b.d_x, b.d_y, st) == CUDASP_OK;
  if (st) {
    ok = hipStreamSynchronize(st) == hipSuccess && ok;  // the pageable sources stay alive until here
    (void)hipStreamDestroy(st);
  }
  if (d_tmp) (void)hipFree(d_tmp);
  if (!ok) {
    free_batch(b);
    return fail(CUDASP_ERR_HIP, "resident table: a batch of %llu rows on device %d: allocation or upload failed",
                (unsigned long long)n, t.devices[b.lg]);
  }
  if (!s.dense) b.ord = s.ord;
  t.device_bytes += n * (32 + 32 + 4 + 4 + 1 + 4) + wb;
  t.pinned_rows += n;
  t.batches.push_back(std::move(b));
  reset_staging(t);
  return CUDASP_OK;
}

// Close the open batch: copy it into pinned memory and give it its mirror on
// its logical GPU's device.
int seal(cudasp_pinned_table& t) {
  Staging& s = t.open;
  const uint64_t n = s.n();
  if (n == 0) return CUDASP_OK;
  if (t.seal_fail_at && ++t.seals == t.seal_fail_at)
    return fail(CUDASP_ERR_CAPACITY, "pinned table: batch close %llu failed (CUDASP_PINNED_TEST_SEAL_FAIL)",
                (unsigned long long)t.seals);
  Batch b;
  b.n = (uint32_t)n;
  b.words = s.outputs.size();
  b.lg = (uint32_t)(t.batches.size() % t.devices.size());
  b.device = t.devices[b.lg];
  b.ord0 = s.ord[0];
  const size_t wb = std::max<size_t>(1, b.words) * sizeof(int64_t);
  int rc = CUDASP_OK;
  if (t.hbm && !t.host_only) return seal_hbm(t, b, wb);
  if (t.host_only) {
    b.host_mem = true;
    b.rows = (uint8_t*)malloc(n * TWEAK_KEY_SIZE);
    b.outputs = (int64_t*)malloc(wb);
    b.offsets = (uint32_t*)malloc((n + 1) * sizeof(uint32_t));
    b.matches = (uint32_t*)malloc(n * sizeof(uint32_t));
    if (!b.rows || !b.outputs || !b.offsets || !b.matches) rc = CUDASP_ERR_CAPACITY;
  } else {
    rc = cudasp_host_alloc((void**)&b.rows, n * TWEAK_KEY_SIZE);
    if (rc == CUDASP_OK) rc = cudasp_host_alloc((void**)&b.outputs, wb);
    if (rc == CUDASP_OK) rc = cudasp_host_alloc((void**)&b.offsets, (n + 1) * sizeof(uint32_t));
    if (rc == CUDASP_OK) rc = cudasp_host_alloc((void**)&b.matches, n * sizeof(uint32_t));
  }
  if (rc != CUDASP_OK) {
    free_batch(b);
    return fail(CUDASP_ERR_CAPACITY, "pinned table: host allocation for a batch of %llu rows failed",
                (unsigned long long)n);
  }
  if (!t.host_only) {
    DeviceSet ds(b.device);
    if (hipMalloc((void**)&b.d_mirror, wb) != hipSuccess) {
      b.d_mirror = nullptr;
      free_batch(b);
      return fail(CUDASP_ERR_HIP, "pinned table: outputs mirror of %zu bytes on device %d: allocation failed", wb,
                  b.device);
    }
  }
  memcpy(b.rows, s.rows.data(), n * TWEAK_KEY_SIZE);
  if (b.words) memcpy(b.outputs, s.outputs.data(), b.words * sizeof(int64_t));
  memcpy(b.offsets, s.offsets.data(), (n + 1) * sizeof(uint32_t));
  if (!s.dense) b.ord = s.ord;
  t.pinned_bytes += n * TWEAK_KEY_SIZE + wb + (2 * n + 1) * sizeof(uint32_t);
  t.device_bytes += wb;  // the mirror
  t.pinned_rows += n;
  t.batches.push_back(std::move(b));
  reset_staging(t);
  return CUDASP_OK;
}

// Finish every stream after a failed scan; a stream whose kernel is still
// running after the timeout pins the table (nothing it reads may be freed).
void reset_streams(cudasp_pinned_table& t) {
  for (size_t lg = 0; lg < t.streams.size(); lg++) {
    if (!t.streams[lg]) continue;
    DeviceSet ds(t.devices[lg]);
    (void)cudasp_stream_finish(t.streams[lg]);
    if (cudasp_stream_abandoned(t.streams[lg])) {
      t.abandoned = true;
      continue;
    }
    cudasp_stream_destroy(t.streams[lg]);
    t.streams[lg] = nullptr;
  }
  t.stream_ok = false;
}

// The pinned placement's scan: every batch published in place to its logical
// GPU's streaming kernel (at most 64 in flight per stream, harvested in
// order); a failure finishes the streams.
int scan_streams(cudasp_pinned_table& t, std::vector<uint64_t>& hits, double* t_pub) {
  const size_t nl = t.devices.size();
  int rc = CUDASP_OK;
  t.stream_ok = false;  // until this scan finishes
  std::vector<std::deque<std::pair<size_t, uint64_t>>> pend(nl);  // (batch, seq) in publish order
  std::string msg;
  // a done batch's matches: the count is readable until 64 more batches are
  // published on its stream, the row indices stay in its buffer
  auto collect = [&](size_t lg) -> int {
    const auto [j, seq] = pend[lg].front();
    pend[lg].pop_front();
    cudasp_stream* st = t.streams[lg];
    int r = cudasp_stream_wait(st, seq);
    uint32_t m = 0;
    if (r == CUDASP_OK) r = cudasp_stream_matches(st, seq, &m);
    if (r != CUDASP_OK) return r;
    const Batch& bt = t.batches[j];
    if (m > bt.n) return fail(CUDASP_ERR_HIP, "pinned table: batch %zu reports %u matches of %u rows", j, m, bt.n);
    for (uint32_t k = 0; k < m; k++) {
      if (bt.matches[k] >= bt.n)
        return fail(CUDASP_ERR_HIP, "pinned table: batch %zu reports row %u of %u", j, bt.matches[k], bt.n);
      hits.push_back(bt.number(bt.matches[k]));
    }
    return CUDASP_OK;
  };
  for (size_t j = 0; j < t.batches.size() && rc == CUDASP_OK; j++) {
    const Batch& bt = t.batches[j];
    DeviceSet ds(t.devices[bt.lg]);
    if (pend[bt.lg].size() >= STREAM_RING) rc = collect(bt.lg);
    if (rc != CUDASP_OK) break;
    cudasp_stream_batch sb{};
    sb.tweak_keys = bt.rows;
    sb.outputs = bt.outputs;
    sb.output_offsets = bt.offsets;
    sb.output_lengths = nullptr;  // Arrow offsets: n + 1
    sb.n = bt.n;
    sb.match_rows = bt.matches;
    sb.d_mirror = bt.d_mirror;
    uint64_t seq = 0;
    rc = cudasp_stream_publish_batch(t.streams[bt.lg], &sb, &seq);
    if (rc == CUDASP_OK) pend[bt.lg].emplace_back(j, seq);
  }
  for (size_t lg = 0; lg < nl && rc == CUDASP_OK; lg++) {
    DeviceSet ds(t.devices[lg]);
    rc = cudasp_stream_close(t.streams[lg]);
  }
  *t_pub = now_s();
  for (size_t lg = 0; lg < nl && rc == CUDASP_OK; lg++) {
    DeviceSet ds(t.devices[lg]);
    while (!pend[lg].empty() && rc == CUDASP_OK) rc = collect(lg);
    if (rc == CUDASP_OK) rc = cudasp_stream_finish(t.streams[lg]);  // reset for the next scan
  }
  if (rc != CUDASP_OK) {
    msg = cudasp_last_error();
    reset_streams(t);
    return fail(rc, "%s", msg.c_str());
  }
  t.stream_ok = true;
  return CUDASP_OK;
}

// The HBM placement's scan: one cudasp_scan_device_batches launch per logical
// GPU over all of its resident batches (all launched before any is waited
// for), then each batch's match count and rows read back.
int scan_hbm(cudasp_pinned_table& t, std::vector<uint64_t>& hits) {
  const size_t nl = t.devices.size();
  std::vector<std::vector<size_t>> of(nl);  // batch indices per logical GPU
  for (size_t j = 0; j < t.batches.size(); j++) of[t.batches[j].lg].push_back(j);
  for (size_t lg = 0; lg < nl; lg++) {
    if (of[lg].empty()) continue;
    DeviceSet ds(t.devices[lg]);
    if (t.counts_cap[lg] < of[lg].size()) {
      if (t.d_counts[lg]) (void)hipFree(t.d_counts[lg]);
      t.d_counts[lg] = nullptr;
      t.counts_cap[lg] = 0;
      if (hipMalloc((void**)&t.d_counts[lg], of[lg].size() * 4) != hipSuccess)
        return fail(CUDASP_ERR_HIP, "resident table: match counts on device %d: allocation failed", t.devices[lg]);
      t.counts_cap[lg] = of[lg].size();
    }
    // the counts are added to: zeroed first, on the scanner's own stream
    // (the launch below runs there, after it)
    auto* st = (hipStream_t)cudasp_internal_scanner_stream(t.scanners[lg]);
    if (hipMemsetAsync(t.d_counts[lg], 0, of[lg].size() * 4, st) != hipSuccess)
      return fail(CUDASP_ERR_HIP, "resident table: zeroing the match counts on device %d failed", t.devices[lg]);
  }
  for (size_t lg = 0; lg < nl; lg++) {
    if (of[lg].empty()) continue;
    DeviceSet ds(t.devices[lg]);
    std::vector<cudasp_device_batch> db(of[lg].size());
    for (size_t k = 0; k < of[lg].size(); k++) {
      const Batch& bt = t.batches[of[lg][k]];
      db[k] = cudasp_device_batch{bt.d_x, bt.d_y, bt.d_out, bt.d_offs, bt.d_lens, bt.n, bt.d_flags, bt.d_rows,
                                  t.d_counts[lg] + k};
    }
    const int rc = cudasp_scan_device_batches(t.scanners[lg], db.data(), (uint32_t)db.size(), nullptr);
    if (rc != CUDASP_OK) return rc;
  }
  std::vector<uint32_t> cnt, idx;
  for (size_t lg = 0; lg < nl; lg++) {
    if (of[lg].empty()) continue;
    DeviceSet ds(t.devices[lg]);
    int rc = cudasp_scanner_sync(t.scanners[lg]);
    if (rc != CUDASP_OK) return rc;
    cnt.resize(of[lg].size());
    if (hipMemcpy(cnt.data(), t.d_counts[lg], cnt.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
      return fail(CUDASP_ERR_HIP, "resident table: reading the match counts on device %d failed", t.devices[lg]);
    for (size_t k = 0; k < of[lg].size(); k++) {
      const Batch& bt = t.batches[of[lg][k]];
      const uint32_t m = cnt[k];
      if (m == 0) continue;
      if (m > bt.n)
        return fail(CUDASP_ERR_HIP, "resident table: batch %zu reports %u matches of %u rows", of[lg][k], m, bt.n);
      idx.resize(m);
      if (hipMemcpy(idx.data(), bt.d_rows, (size_t)m * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(CUDASP_ERR_HIP, "resident table: reading batch %zu's matches failed", of[lg][k]);
      for (uint32_t r : idx) {
        if (r >= bt.n) return fail(CUDASP_ERR_HIP, "resident table: batch %zu reports row %u of %u", of[lg][k], r, bt.n);
        hits.push_back(bt.number(r));
      }
    }
  }
  return CUDASP_OK;
}

}  // namespace

extern "C" {

int cudasp_pinned_create(uint64_t batch_size, const int* devices, uint32_t device_count, cudasp_pinned_table** out) {
  return cudasp_pinned_create_placed(batch_size, devices, device_count, CUDASP_TABLE_PINNED, out);
}

int cudasp_pinned_create_placed(uint64_t batch_size, const int* devices, uint32_t device_count, int placement,
                                cudasp_pinned_table** out) {
  if (!out) return fail(CUDASP_ERR_INVALID_ARG, "null argument");
  *out = nullptr;
  if (placement != CUDASP_TABLE_PINNED && placement != CUDASP_TABLE_HBM)
    return fail(CUDASP_ERR_INVALID_ARG, "placement must be CUDASP_TABLE_PINNED or CUDASP_TABLE_HBM, got %d", placement);
  if (batch_size == 0) batch_size = CUDASP_TF_DEFAULT_BATCH;
  if (batch_size > MAX_BATCH)
    return fail(CUDASP_ERR_INVALID_ARG, "batch_size too large (max 10,000,000), got %llu",
                (unsigned long long)batch_size);
  if (devices && device_count == 0) return fail(CUDASP_ERR_INVALID_ARG, "device_count must be positive");
  const bool host_only = env_null_device();
  int ndev = 0;
  if (host_only)
    ndev = 1 << 16;
  else if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
    return fail(CUDASP_ERR_NO_DEVICE, "no GPU");
  auto* t = new cudasp_pinned_table();
  t->batch_size = batch_size;
  t->host_only = host_only;
  t->hbm = placement == CUDASP_TABLE_HBM;
  t->max_words = env_max_words();
  t->seal_fail_at = env_seal_fail();
  if (devices)
    t->devices.assign(devices, devices + device_count);
  else
    t->devices.assign(1, 0);
  for (int d : t->devices)
    if (d < 0 || d >= ndev) {
      delete t;
      return fail(CUDASP_ERR_INVALID_ARG, "device %d out of range (%d GPUs)", d, ndev);
    }
  // a logical GPU's grid: its device's wave slots shared by the logical GPUs
  // on it (0 = the whole device, 3 waves per SIMD)
  for (int d : t->devices) {
    const int m = (int)std::count(t->devices.begin(), t->devices.end(), d);
    int cus = 0;
    if (host_only) {
      t->blocks.push_back(0);
      continue;
    }
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || cus <= 0) cus = 256;
    t->blocks.push_back(m == 1 ? 0u : (uint32_t)(cus * 3 / m));
  }
  t->scanners.assign(t->devices.size(), nullptr);
  t->streams.assign(t->devices.size(), nullptr);
  t->d_counts.assign(t->devices.size(), nullptr);
  t->counts_cap.assign(t->devices.size(), 0);
  t->open.rows.reserve(std::min<uint64_t>(batch_size, 1u << 16) * TWEAK_KEY_SIZE);
  *out = t;
  return CUDASP_OK;
}

int cudasp_pinned_append(cudasp_pinned_table* t, const cudasp_tf_columns* cols) {
  if (!t || !cols) return fail(CUDASP_ERR_INVALID_ARG, "null argument");
  std::lock_guard<std::mutex> lk(t->mu);
  if (t->abandoned) return fail(CUDASP_ERR_HIP, "pinned table: a scan's kernel is still running");
  const cudasp_tf_columns& c = *cols;
  const uint64_t n = c.count;
  if (n == 0) return CUDASP_OK;
  if (!c.tweak_data || !c.list_offsets) return fail(CUDASP_ERR_INVALID_ARG, "tweak_key and outputs columns needed");
  if (!c.tweak_offsets && c.tweak_fixed_width <= 0)
    return fail(CUDASP_ERR_INVALID_ARG, "tweak_key: offsets or a fixed width needed");
  auto row_ok = [&](uint64_t i) {
    return bit(c.txid_validity, c.txid_offset + i) && bit(c.height_validity, c.height_offset + i) &&
           bit(c.tweak_validity, c.tweak_offset + i);
  };
  auto tweak_size = [&](uint64_t i) -> uint64_t {
    if (c.tweak_offsets) {
      const int32_t* to = c.tweak_offsets + c.tweak_offset;
      return (uint64_t)(to[i + 1] - to[i]);
    }
    return (uint64_t)c.tweak_fixed_width;
  };
  auto tweak_ptr = [&](uint64_t i) -> const uint8_t* {
    if (c.tweak_offsets) return c.tweak_data + c.tweak_offsets[c.tweak_offset + i];
    return c.tweak_data + (c.tweak_offset + i) * (uint64_t)c.tweak_fixed_width;
  };
  const int32_t* lo = c.list_offsets + c.list_offset;
  // the run is checked first: a bad tweak keeps nothing of it
  for (uint64_t i = 0; i < n; i++) {
    if (!row_ok(i)) continue;
    const uint64_t sz = tweak_size(i);
    if (sz != TWEAK_KEY_SIZE)
      return fail(CUDASP_ERR_INVALID_ARG, "tweak_key must be exactly 64 bytes, got %llu bytes", (unsigned long long)sz);
    if (bit(c.list_validity, c.list_offset + i) && lo[i + 1] > lo[i] && !c.child_values)
      return fail(CUDASP_ERR_INVALID_ARG, "pinned tables take int64 outputs (child_values)");
  }
  // All or nothing: a batch close that fails (allocation, upload) undoes the
  // whole run -- the batches closed during it are freed and the open batch
  // is restored to its state at entry -- so the input numbers handed out stay
  // t->appended + i of a run that was kept, and a retried run is numbered
  // the same.  The rows that were open at entry leave the staging at the
  // run's first close; that prefix is kept until the run succeeds.
  Staging& s = t->open;
  const size_t nb0 = t->batches.size();
  const uint64_t n0 = s.n(), w0 = s.outputs.size();
  const bool dense0 = s.dense;
  const uint64_t rows0 = t->pinned_rows, pbytes0 = t->pinned_bytes, dbytes0 = t->device_bytes;
  Staging entry;  // the entry prefix, once the first close took it away
  bool closed = false;
  auto close = [&]() -> int {
    if (!closed && n0) {
      entry.rows.assign(s.rows.begin(), s.rows.begin() + n0 * TWEAK_KEY_SIZE);
      entry.outputs.assign(s.outputs.begin(), s.outputs.begin() + w0);
      entry.offsets.assign(s.offsets.begin(), s.offsets.begin() + n0 + 1);
      entry.ord.assign(s.ord.begin(), s.ord.begin() + n0);
      entry.dense = dense0;
    }
    const int rc = seal(*t);
    if (rc == CUDASP_OK) closed = true;
    return rc;
  };
  auto rollback = [&](int rc) -> int {
    const std::string msg = cudasp_last_error();
    while (t->batches.size() > nb0) {
      free_batch(t->batches.back());
      t->batches.pop_back();
    }
    t->pinned_rows = rows0;
    t->pinned_bytes = pbytes0;
    t->device_bytes = dbytes0;
    if (closed) {
      s = std::move(entry);
      if (!n0) reset_staging(*t);
    } else {
      s.rows.resize(n0 * TWEAK_KEY_SIZE);
      s.outputs.resize(w0);
      s.offsets.resize(n0 + 1);
      s.ord.resize(n0);
      s.dense = dense0;
    }
    return fail(rc, "%s (the run of %llu rows was not appended)", msg.c_str(), (unsigned long long)n);
  };
  for (uint64_t i = 0; i < n; i++) {
    if (!row_ok(i)) continue;
    const bool lv = bit(c.list_validity, c.list_offset + i);
    const uint64_t len = lv ? (uint64_t)(lo[i + 1] - lo[i]) : 0;
    if (s.n() && s.outputs.size() + len > t->max_words) {  // keep u32 offsets: close the batch early
      const int rc = close();
      if (rc != CUDASP_OK) return rollback(rc);
    }
    const uint64_t num = t->appended + i;
    if (s.n() && num != s.ord[0] + s.n()) s.dense = false;
    s.ord.push_back(num);
    const uint8_t* tw = tweak_ptr(i);
    s.rows.insert(s.rows.end(), tw, tw + TWEAK_KEY_SIZE);
    if (len) {
      const int64_t* v = c.child_values + c.child_offset + lo[i];
      if (!c.child_validity) {
        s.outputs.insert(s.outputs.end(), v, v + len);
      } else {
        for (uint64_t k = 0; k < len; k++)
          if (bit(c.child_validity, c.child_offset + (uint64_t)lo[i] + k)) s.outputs.push_back(v[k]);
      }
    }
    s.offsets.push_back((uint32_t)s.outputs.size());
    if (s.n() == t->batch_size) {
      const int rc = close();
      if (rc != CUDASP_OK) return rollback(rc);
    }
  }
  t->appended += n;
  return CUDASP_OK;
}

int cudasp_pinned_scan(cudasp_pinned_table* t, const cudasp_tf_bind_data* b, uint64_t** rows, uint64_t* count) {
  if (!t || !b || !rows || !count) return fail(CUDASP_ERR_INVALID_ARG, "null argument");
  *rows = nullptr;
  *count = 0;
  std::lock_guard<std::mutex> lk(t->mu);
  if (t->abandoned) return fail(CUDASP_ERR_HIP, "pinned table: a scan's kernel is still running");
  if (b->opt.full_x) return fail(CUDASP_ERR_INVALID_ARG, "pinned tables do not take full_x outputs");
  if (t->host_only) return fail(CUDASP_ERR_NO_DEVICE, "pinned table without a device (CUDASP_TF_NULL_DEVICE)");
  const double t0 = now_s();
  int rc = seal(*t);
  if (rc != CUDASP_OK) return rc;
  const auto* scan = (const uint8_t*)b->scan_private_key_data.data();
  const auto* spend = (const uint8_t*)b->spend_public_key_data.data();
  const auto* labels = (const uint8_t*)b->label_keys_flat.data();
  const auto nlabels = (uint32_t)b->label_keys_data.size();
  const Shape shape{nlabels, b->opt.output_count, b->opt.label_negation ? 1u : 0u};
  const bool fresh = !t->stream_ok || !(shape == t->shape);
  const size_t nl = t->devices.size();
  // one scanner and streaming kernel per logical GPU, kept and rebound to
  // each scan's keys (creating them costs milliseconds; a 1M-row scan ~6 ms)
  for (size_t lg = 0; lg < nl; lg++) {
    DeviceSet ds(t->devices[lg]);
    if (!t->scanners[lg]) {
      // (the resident scan's per-batch path, taken for output_count > 1,
      // needs a batch's rows within the scanner's capacity)
      const uint64_t cap = t->hbm ? t->batch_size : std::min<uint64_t>(t->batch_size, CUDASP_TF_DEFAULT_BATCH);
      rc = cudasp_scanner_create(t->devices[lg], scan, spend, labels, nlabels, std::max<uint64_t>(1, cap),
                                 &t->scanners[lg]);
    } else {
      rc = cudasp_scanner_set_keys(t->scanners[lg], scan, spend, labels, nlabels);
    }
    if (rc == CUDASP_OK) rc = cudasp_scanner_set_options(t->scanners[lg], &b->opt);
    if (rc != CUDASP_OK) {
      t->stream_ok = false;
      return rc;  // the scanner call's message
    }
    if (t->hbm) continue;  // no streams
    if (!cudasp_stream_supported(t->scanners[lg])) {
      t->stream_ok = false;
      return fail(CUDASP_ERR_INVALID_ARG, "pinned table: the streaming scan cannot run %u label keys", nlabels);
    }
    // a stream is sized (scratch, grid) for its scanner's label count and
    // output indices when created: a new one when they change
    if (fresh || !t->streams[lg]) {
      if (t->streams[lg]) {
        cudasp_stream_destroy(t->streams[lg]);
        t->streams[lg] = nullptr;
      }
      rc = cudasp_stream_create(t->scanners[lg], t->blocks[lg], &t->streams[lg]);
      if (rc != CUDASP_OK) {
        t->streams[lg] = nullptr;
        t->stream_ok = false;
        return rc;
      }
    }
  }
  t->shape = shape;
  std::vector<uint64_t> hits;
  double t_pub = 0;
  if (t->hbm) {
    rc = scan_hbm(*t, hits);
    if (rc != CUDASP_OK) return rc;
    t_pub = now_s();
  } else {
    rc = scan_streams(*t, hits, &t_pub);
    if (rc != CUDASP_OK) return rc;
  }
  std::sort(hits.begin(), hits.end());
  auto* out = (uint64_t*)malloc(std::max<size_t>(1, hits.size()) * sizeof(uint64_t));
  if (!out) return fail(CUDASP_ERR_CAPACITY, "pinned table: %zu result rows: allocation failed", hits.size());
  if (!hits.empty()) memcpy(out, hits.data(), hits.size() * sizeof(uint64_t));
  *rows = out;
  *count = hits.size();
  t->last_matches = hits.size();
  t->last_publish_s = t_pub - t0;
  t->last_scan_s = now_s() - t0;
  return CUDASP_OK;
}

void cudasp_pinned_free_rows(uint64_t* rows) { free(rows); }

int cudasp_pinned_info(const cudasp_pinned_table* t, cudasp_pinned_info_t* out) {
  if (!t || !out) return fail(CUDASP_ERR_INVALID_ARG, "null argument");
  std::lock_guard<std::mutex> lk(t->mu);
  out->rows_appended = t->appended;
  out->rows_pinned = t->pinned_rows + t->open.n();
  out->batches = t->batches.size() + (t->open.n() ? 1 : 0);
  out->pinned_bytes = t->pinned_bytes;
  out->last_matches = t->last_matches;
  out->last_scan_s = t->last_scan_s;
  out->last_publish_s = t->last_publish_s;
  out->placement = t->hbm ? CUDASP_TABLE_HBM : CUDASP_TABLE_PINNED;
  out->device_bytes = t->device_bytes;
  return CUDASP_OK;
}

void cudasp_pinned_free(cudasp_pinned_table* t) {
  if (!t) return;
  {
    std::lock_guard<std::mutex> lk(t->mu);
    if (t->abandoned) return;  // its kernel may still read the batches
    for (size_t lg = 0; lg < t->streams.size(); lg++) {
      if (t->streams[lg]) {
        DeviceSet ds(t->devices[lg]);
        cudasp_stream_destroy(t->streams[lg]);
      }
      if (t->scanners[lg]) cudasp_scanner_destroy(t->scanners[lg]);
      if (t->d_counts[lg]) {
        DeviceSet ds(t->devices[lg]);
        (void)hipFree(t->d_counts[lg]);
      }
    }
    for (Batch& bt : t->batches) free_batch(bt);
  }
  delete t;
}

}  // extern "C"
