// cudasp_scan table-function host, DuckDB-independent (include/cudasp_host.h).
//
// Same state machine as the reference host (src/cudasp_extension.cu:87-659):
// bind validation with the same messages, per-thread accumulation with the
// same NULL rules, the `>= batch_size` trigger, round-robin GPU per thread,
// mutex-guarded global match list, last-thread-emits in 2048-row chunks.
// What differs, by design:
//   * rows are accumulated into flat columns (one byte arena for txids, one
//     n x 64 tweak array, a CSR for outputs) instead of two heap strings per
//     row (:202-204), and handed to the kernels in one copy, with no
//     column-major repack on the host (:249-341) and no u64[n][64] staging
//     (src/cudasp_gpu.cu:705-761);
//   * each thread keeps one scanner (keys bound once, device buffers reused)
//     instead of allocating and freeing per batch (src/cudasp_gpu.cu:487-666);
//   * rows are accumulated straight into pinned host buffers and batches run
//     asynchronously, double-buffered: while the GPU scans batch b (H2D,
//     transpose, both kernels, D2H of the flags, all on the thread's stream),
//     the DuckDB thread accumulates batch b+1; the reference blocks the thread
//     for the whole GPU round trip (README.md:140 "serial table scan overhead");
//   * a failed batch is reported (cudasp_tf_function/final return an error)
//     instead of being dropped silently (:325, :378);
//   * a tweak_key BLOB that is not 64 bytes is an error instead of an
//     out-of-bounds read (:333, ConvertTweakKeyToU32 always reads 64 bytes).
#include "../../../include/cudasp_host.h"

#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/cudasp_abi.h"

namespace {

constexpr uint64_t TWEAK_KEY_SIZE = 64;  // CudaspScanBindData::TWEAK_KEY_SIZE
constexpr uint64_t SCALAR_SIZE = 32;     // CudaspScanBindData::SCALAR_SIZE
constexpr uint32_t XONLY_SIZE = 32;      // full_x outputs: x-only keys
// int64 words per output in the host/device outputs buffers.
inline size_t out_words(const cudasp_tf_bind_data& b);

void write_err(char* err, size_t cap, const char* fmt, ...) {
  if (!err || cap == 0) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(err, cap, fmt, ap);
  va_end(ap);
}

}  // namespace

extern "C" void cudasp_internal_set_error(const char* msg);

struct cudasp_tf_bind_data {
  uint64_t batch_size = CUDASP_TF_DEFAULT_BATCH;
  cudasp_scan_options opt{1, 0, 0};  // named parameters output_count / label_negation / full_x
  std::string scan_private_key_data;
  std::string spend_public_key_data;
  std::vector<std::string> label_keys_data;
  std::string label_keys_flat;  // label_count x 64, back to back
};

namespace {
inline size_t out_words(const cudasp_tf_bind_data& b) { return b.opt.full_x ? XONLY_SIZE / 8 : 1; }
}  // namespace

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
};

// One accumulation/launch buffer set of a thread (double-buffered).
struct HostSlot {
  // row data for the kernels, pinned for asynchronous H2D
  uint8_t* h_tweaks = nullptr;  // cap_rows x 64
  uint32_t* h_offs = nullptr;
  uint32_t* h_lens = nullptr;
  uint8_t* h_flags = nullptr;
  int64_t* h_outputs = nullptr;
  size_t outputs_cap = 0;
  size_t n_outputs = 0;
  // row data for the emit (pageable)
  std::vector<uint8_t> txid_bytes;
  std::vector<uint64_t> txid_offset;
  std::vector<uint32_t> txid_size;
  std::vector<int32_t> heights;
  uint32_t rows = 0;
  // device side
  uint8_t* d_rows = nullptr;
  uint32_t* d_tx = nullptr;
  uint32_t* d_ty = nullptr;
  uint32_t* d_offs = nullptr;
  uint32_t* d_lens = nullptr;
  uint8_t* d_flags = nullptr;
  int64_t* d_outputs = nullptr;
  size_t d_outputs_cap = 0;
  hipEvent_t done = nullptr;
  bool in_flight = false;
  uint32_t launched_rows = 0;
};

struct cudasp_tf_local {
  bool finalized = false;
  bool is_output_thread = false;
  int assigned_gpu = -1;  // logical GPU (round-robin over num_gpus)
  int device = -1;        // the HIP device it runs on
  uint32_t cap_rows = 0;
  HostSlot slots[2];
  int cur = 0;
  cudasp_scanner* scanner = nullptr;
  hipStream_t stream = nullptr;
  uint32_t rows() const { return slots[cur].rows; }
};

namespace {

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

inline bool valid(const uint8_t* v, uint32_t i) { return v == nullptr || v[i] != 0; }

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

// need: int64 words; ow: words per output already held (n_outputs * ow used).
int ensure_outputs_cap(HostSlot& s, size_t need, size_t ow = 1) {
  if (need <= s.outputs_cap) return CUDASP_OK;
  size_t cap = s.outputs_cap ? s.outputs_cap : 4096;
  while (cap < need) cap *= 2;
  int64_t* p = nullptr;
  HOST_HIP(hipHostMalloc((void**)&p, cap * sizeof(int64_t), hipHostMallocDefault));
  if (s.n_outputs) memcpy(p, s.h_outputs, s.n_outputs * ow * sizeof(int64_t));
  if (s.h_outputs) (void)hipHostFree(s.h_outputs);
  s.h_outputs = p;
  s.outputs_cap = cap;
  return CUDASP_OK;
}

// GPU state of an executor thread (scanner, stream, pinned host and device
// buffers of both slots).  It is created on the thread's first row and, when
// the thread's local state is freed, parked in a process-wide pool instead of
// being released: the next query's threads take it back and only rebind the
// keys (cudasp_scanner_set_keys), so a query pays no pinned-memory or device
// allocations once the pool is warm.
struct GpuCtx {
  int device = -1;
  uint32_t cap_rows = 0;
  cudasp_scanner* scanner = nullptr;
  hipStream_t stream = nullptr;
  HostSlot slots[2];
};

constexpr size_t POOL_MAX = 64;
std::mutex g_pool_mu;
std::vector<GpuCtx*> g_pool;

void reset_slot_state(HostSlot& s) {
  s.txid_bytes.clear();
  s.txid_offset.clear();
  s.txid_size.clear();
  s.heights.clear();
  s.rows = 0;
  s.n_outputs = 0;
  s.in_flight = false;
  s.launched_rows = 0;
}

void release_ctx(GpuCtx* c) {
  DeviceSet dg(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (HostSlot& s : c->slots) {
    void* host[] = {s.h_tweaks, s.h_offs, s.h_lens, s.h_flags, s.h_outputs};
    for (void* p : host)
      if (p) (void)hipHostFree(p);
    void* dev[] = {s.d_rows, s.d_tx, s.d_ty, s.d_offs, s.d_lens, s.d_flags, s.d_outputs};
    for (void* p : dev)
      if (p) (void)hipFree(p);
    if (s.done) (void)hipEventDestroy(s.done);
  }
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->scanner) cudasp_scanner_destroy(c->scanner);
  delete c;
}

// A pooled context for (device, at least cap_rows), or nullptr.
GpuCtx* pool_take(int device, uint32_t cap_rows) {
  std::lock_guard<std::mutex> lock(g_pool_mu);
  for (size_t i = 0; i < g_pool.size(); i++) {
    GpuCtx* c = g_pool[i];
    if (c->device == device && c->cap_rows >= cap_rows) {
      g_pool[i] = g_pool.back();
      g_pool.pop_back();
      return c;
    }
  }
  return nullptr;
}

void pool_put(GpuCtx* c) {
  {
    std::lock_guard<std::mutex> lock(g_pool_mu);
    if (g_pool.size() < POOL_MAX) {
      g_pool.push_back(c);
      return;
    }
  }
  release_ctx(c);
}

void ctx_to_local(GpuCtx* c, cudasp_tf_local& l) {
  l.cap_rows = c->cap_rows;
  l.scanner = c->scanner;
  l.stream = c->stream;
  for (int i = 0; i < 2; i++) {
    l.slots[i] = std::move(c->slots[i]);
    reset_slot_state(l.slots[i]);
  }
  l.cur = 0;
  c->scanner = nullptr;
  c->stream = nullptr;
  delete c;
}

int ensure_local_gpu(const cudasp_tf_bind_data& b, cudasp_tf_local& l) {
  if (l.scanner) return CUDASP_OK;
  DeviceSet dg(l.device);
  const uint32_t cap_rows = (uint32_t)(b.batch_size + CUDASP_TF_VECTOR_SIZE);
  const auto* scan = (const uint8_t*)b.scan_private_key_data.data();
  const auto* spend = (const uint8_t*)b.spend_public_key_data.data();
  const auto* labels = (const uint8_t*)b.label_keys_flat.data();
  const auto nlabels = (uint32_t)b.label_keys_data.size();
  if (GpuCtx* c = pool_take(l.device, cap_rows)) {
    int rc = cudasp_scanner_set_keys(c->scanner, scan, spend, labels, nlabels);
    if (rc == CUDASP_OK) rc = cudasp_scanner_set_options(c->scanner, &b.opt);
    if (rc != CUDASP_OK) {
      pool_put(c);
      return host_fail(rc, "Failed to bind scanner on GPU %d: %s", l.assigned_gpu, cudasp_last_error());
    }
    ctx_to_local(c, l);
    return CUDASP_OK;
  }
  l.cap_rows = cap_rows;
  int rc = cudasp_scanner_create(l.device, scan, spend, labels, nlabels, l.cap_rows, &l.scanner);
  if (rc == CUDASP_OK) rc = cudasp_scanner_set_options(l.scanner, &b.opt);
  if (rc != CUDASP_OK)
    return host_fail(rc, "Failed to create scanner on GPU %d: %s", l.assigned_gpu, cudasp_last_error());
  HOST_HIP(hipStreamCreateWithFlags(&l.stream, hipStreamNonBlocking));
  for (HostSlot& s : l.slots) {
    size_t n = l.cap_rows;
    HOST_HIP(hipHostMalloc((void**)&s.h_tweaks, n * 64, hipHostMallocDefault));
    HOST_HIP(hipHostMalloc((void**)&s.h_offs, n * 4, hipHostMallocDefault));
    HOST_HIP(hipHostMalloc((void**)&s.h_lens, n * 4, hipHostMallocDefault));
    HOST_HIP(hipHostMalloc((void**)&s.h_flags, n, hipHostMallocDefault));
    HOST_HIP(hipMalloc((void**)&s.d_rows, n * 64));
    HOST_HIP(hipMalloc((void**)&s.d_tx, n * 32));
    HOST_HIP(hipMalloc((void**)&s.d_ty, n * 32));
    HOST_HIP(hipMalloc((void**)&s.d_offs, n * 4));
    HOST_HIP(hipMalloc((void**)&s.d_lens, n * 4));
    HOST_HIP(hipMalloc((void**)&s.d_flags, n));
    HOST_HIP(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    rc = ensure_outputs_cap(s, (size_t)n * 2);
    if (rc != CUDASP_OK) return rc;
  }
  return CUDASP_OK;
}

// Park the thread's GPU state in the pool (after its work has drained).
void free_local_gpu(cudasp_tf_local& l) {
  if (!l.scanner && !l.stream) return;
  GpuCtx* c = new GpuCtx();
  c->device = l.device;
  c->cap_rows = l.cap_rows;
  c->scanner = l.scanner;
  c->stream = l.stream;
  for (int i = 0; i < 2; i++) {
    c->slots[i] = std::move(l.slots[i]);
    l.slots[i] = HostSlot();
  }
  l.scanner = nullptr;
  l.stream = nullptr;
  {
    DeviceSet dg(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
  }
  if (!c->scanner || !c->stream) {
    release_ctx(c);
    return;
  }
  pool_put(c);
}

// AccumulateInput (src/cudasp_extension.cu:154-224), into the current slot.
int accumulate(const cudasp_tf_bind_data& b, cudasp_tf_local& l, const cudasp_tf_chunk& c) {
  int rc = ensure_local_gpu(b, l);
  if (rc != CUDASP_OK) return rc;
  HostSlot& s = l.slots[l.cur];
  const size_t ow = out_words(b);
  if (b.opt.full_x && c.count > 0 && (!c.child_blob_data || !c.child_blob_size))
    return host_fail(CUDASP_ERR_INVALID_ARG, "full_x needs the outputs column as BLOB[] (child_blob_data)");
  for (uint32_t i = 0; i < c.count; i++) {
    // Only rows with valid txid, height and tweak_key (:195-197).
    if (!(valid(c.txid_valid, i) && valid(c.height_valid, i) && valid(c.tweak_valid, i))) continue;
    if (c.tweak_size[i] != TWEAK_KEY_SIZE)
      return host_fail(CUDASP_ERR_INVALID_ARG, "tweak_key must be exactly 64 bytes, got %u bytes", c.tweak_size[i]);
    uint32_t r = s.rows;
    s.txid_offset.push_back(s.txid_bytes.size());
    s.txid_size.push_back(c.txid_size[i]);
    s.txid_bytes.insert(s.txid_bytes.end(), c.txid_data[i], c.txid_data[i] + c.txid_size[i]);
    s.heights.push_back(c.height[i]);
    memcpy(s.h_tweaks + (size_t)r * TWEAK_KEY_SIZE, c.tweak_data[i], TWEAK_KEY_SIZE);
    // Outputs: NULL list -> length 0; NULL elements dropped (:206-221).
    s.h_offs[r] = (uint32_t)s.n_outputs;
    uint32_t len = 0;
    if (valid(c.list_valid, i)) {
      rc = ensure_outputs_cap(s, (s.n_outputs + c.list_length[i]) * ow, ow);
      if (rc != CUDASP_OK) return rc;
      for (uint64_t k = 0; k < c.list_length[i]; k++) {
        uint64_t ci = c.list_offset[i] + k;
        if (!valid(c.child_valid, (uint32_t)ci)) continue;
        if (b.opt.full_x) {
          if (c.child_blob_size[ci] != XONLY_SIZE)
            return host_fail(CUDASP_ERR_INVALID_ARG, "full_x outputs must be 32-byte x-only keys, got %u bytes",
                             c.child_blob_size[ci]);
          memcpy(s.h_outputs + s.n_outputs * ow, c.child_blob_data[ci], XONLY_SIZE);
          s.n_outputs++;
        } else {
          s.h_outputs[s.n_outputs++] = c.child_values[ci];
        }
        len++;
      }
    }
    s.h_lens[r] = len;
    s.rows = r + 1;
  }
  return CUDASP_OK;
}

// Columnar rows [r0, r1) of `c` (Arrow layout, cudasp_tf_columns) into the
// current slot, same row rules as accumulate().  Without validity bitmaps and
// with 64-byte tweaks the four columns are appended with bulk copies.
inline bool bit(const uint8_t* bm, uint64_t i) { return bm == nullptr || ((bm[i >> 3] >> (i & 7)) & 1u); }

int accumulate_columns(const cudasp_tf_bind_data& b, cudasp_tf_local& l, const cudasp_tf_columns& c, uint64_t r0,
                       uint64_t r1) {
  int rc = ensure_local_gpu(b, l);
  if (rc != CUDASP_OK) return rc;
  HostSlot& s = l.slots[l.cur];
  const uint64_t n = r1 - r0;
  const size_t ow = out_words(b);
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
  auto push_output = [&](uint64_t k) -> int {
    if (!b.opt.full_x) {
      s.h_outputs[s.n_outputs++] = c.child_values[c.child_offset + k];
      return CUDASP_OK;
    }
    uint32_t sz;
    const uint8_t* p = child_blob(k, &sz);
    if (sz != XONLY_SIZE)
      return host_fail(CUDASP_ERR_INVALID_ARG, "full_x outputs must be 32-byte x-only keys, got %u bytes", sz);
    memcpy(s.h_outputs + s.n_outputs * ow, p, XONLY_SIZE);
    s.n_outputs++;
    return CUDASP_OK;
  };
  const int32_t* txo = c.txid_offsets + c.txid_offset;
  const int32_t* lo = c.list_offsets + c.list_offset;
  auto tweak_ptr = [&](uint64_t i, uint32_t* size) -> const uint8_t* {
    if (c.tweak_offsets) {
      const int32_t* to = c.tweak_offsets + c.tweak_offset;
      *size = (uint32_t)(to[i + 1] - to[i]);
      return c.tweak_data + to[i];
    }
    *size = (uint32_t)c.tweak_fixed_width;
    return c.tweak_data + (c.tweak_offset + i) * (uint64_t)c.tweak_fixed_width;
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
  if (fast) {
    const uint32_t r = s.rows;
    uint32_t sz;
    memcpy(s.h_tweaks + (size_t)r * TWEAK_KEY_SIZE, tweak_ptr(r0, &sz), n * TWEAK_KEY_SIZE);
    s.heights.insert(s.heights.end(), c.height + c.height_offset + r0, c.height + c.height_offset + r1);
    const size_t tbase = s.txid_bytes.size();
    s.txid_bytes.insert(s.txid_bytes.end(), c.txid_data + txo[r0], c.txid_data + txo[r1]);
    const uint64_t first = (uint64_t)lo[r0], total = (uint64_t)lo[r1] - first;
    rc = ensure_outputs_cap(s, (s.n_outputs + total) * ow, ow);
    if (rc != CUDASP_OK) return rc;
    if (b.opt.full_x)
      memcpy(s.h_outputs + s.n_outputs * ow, c.child_blob_data + (c.child_offset + first) * XONLY_SIZE,
             total * XONLY_SIZE);
    else
      memcpy(s.h_outputs + s.n_outputs, c.child_values + c.child_offset + first, total * sizeof(int64_t));
    for (uint64_t i = r0; i < r1; i++) {
      const uint32_t row = r + (uint32_t)(i - r0);
      s.txid_offset.push_back(tbase + (size_t)(txo[i] - txo[r0]));
      s.txid_size.push_back((uint32_t)(txo[i + 1] - txo[i]));
      s.h_offs[row] = (uint32_t)(s.n_outputs + ((uint64_t)lo[i] - first));
      s.h_lens[row] = (uint32_t)(lo[i + 1] - lo[i]);
    }
    s.n_outputs += total;
    s.rows = r + (uint32_t)n;
    return CUDASP_OK;
  }
  for (uint64_t i = r0; i < r1; i++) {
    if (!(bit(c.txid_validity, c.txid_offset + i) && bit(c.height_validity, c.height_offset + i) &&
          bit(c.tweak_validity, c.tweak_offset + i)))
      continue;
    uint32_t tsize;
    const uint8_t* tw = tweak_ptr(i, &tsize);
    if (tsize != TWEAK_KEY_SIZE)
      return host_fail(CUDASP_ERR_INVALID_ARG, "tweak_key must be exactly 64 bytes, got %u bytes", tsize);
    const uint32_t r = s.rows;
    s.txid_offset.push_back(s.txid_bytes.size());
    s.txid_size.push_back((uint32_t)(txo[i + 1] - txo[i]));
    s.txid_bytes.insert(s.txid_bytes.end(), c.txid_data + txo[i], c.txid_data + txo[i + 1]);
    s.heights.push_back(c.height[c.height_offset + i]);
    memcpy(s.h_tweaks + (size_t)r * TWEAK_KEY_SIZE, tw, TWEAK_KEY_SIZE);
    s.h_offs[r] = (uint32_t)s.n_outputs;
    uint32_t len = 0;
    if (bit(c.list_validity, c.list_offset + i)) {
      rc = ensure_outputs_cap(s, (s.n_outputs + (uint64_t)(lo[i + 1] - lo[i])) * ow, ow);
      if (rc != CUDASP_OK) return rc;
      for (int64_t k = lo[i]; k < lo[i + 1]; k++) {
        if (bit(c.child_validity, c.child_offset + (uint64_t)k)) {
          rc = push_output((uint64_t)k);
          if (rc != CUDASP_OK) return rc;
          len++;
        }
      }
    }
    s.h_lens[r] = len;
    s.rows = r + 1;
  }
  return CUDASP_OK;
}

// Collect a finished batch's matches into the global list (ProcessBatch
// :378-392) and reset the slot.
int harvest(cudasp_tf_global& g, cudasp_tf_local& l, HostSlot& s) {
  if (!s.in_flight) return CUDASP_OK;
  {
    DeviceSet dg(l.device);
    HOST_HIP(hipEventSynchronize(s.done));
  }
  s.in_flight = false;
  uint32_t n = s.launched_rows;
  {
    std::lock_guard<std::mutex> lock(g.output_lock);
    for (uint32_t i = 0; i < n; i++) {
      if (!s.h_flags[i]) continue;
      g.output_txids.emplace_back((const char*)s.txid_bytes.data() + s.txid_offset[i], s.txid_size[i]);
      g.output_heights.push_back(s.heights[i]);
      g.output_tweak_keys.emplace_back((const char*)s.h_tweaks + (size_t)i * TWEAK_KEY_SIZE, TWEAK_KEY_SIZE);
    }
  }
  s.txid_bytes.clear();
  s.txid_offset.clear();
  s.txid_size.clear();
  s.heights.clear();
  s.rows = 0;
  s.n_outputs = 0;
  return CUDASP_OK;
}

// ProcessBatch (src/cudasp_extension.cu:226-410), asynchronous: enqueue the
// current slot on the thread's stream and switch to the other slot, first
// harvesting it if its previous batch is still outstanding.
int launch_batch(const cudasp_tf_bind_data& b, cudasp_tf_global& g, cudasp_tf_local& l) {
  HostSlot& s = l.slots[l.cur];
  uint32_t n = s.rows;
  if (n > 0) {
    DeviceSet dg(l.device);
    hipStream_t st = l.stream;
    const size_t words = s.n_outputs * out_words(b);
    if (words > s.d_outputs_cap) {
      if (s.d_outputs) HOST_HIP(hipFree(s.d_outputs));
      s.d_outputs = nullptr;
      size_t cap = s.outputs_cap;
      HOST_HIP(hipMalloc((void**)&s.d_outputs, cap * sizeof(int64_t)));
      s.d_outputs_cap = cap;
    }
    HOST_HIP(hipMemcpyAsync(s.d_rows, s.h_tweaks, (size_t)n * 64, hipMemcpyHostToDevice, st));
    HOST_HIP(hipMemcpyAsync(s.d_offs, s.h_offs, (size_t)n * 4, hipMemcpyHostToDevice, st));
    HOST_HIP(hipMemcpyAsync(s.d_lens, s.h_lens, (size_t)n * 4, hipMemcpyHostToDevice, st));
    if (words) HOST_HIP(hipMemcpyAsync(s.d_outputs, s.h_outputs, words * sizeof(int64_t), hipMemcpyHostToDevice, st));
    int rc = cudasp_tweaks_to_columns(s.d_rows, n, s.d_tx, s.d_ty, st);
    if (rc == CUDASP_OK)
      rc = cudasp_scan_device(l.scanner, s.d_tx, s.d_ty, s.d_outputs, s.d_offs, s.d_lens, n, s.d_flags, nullptr,
                              nullptr, st);
    if (rc != CUDASP_OK) return host_fail(rc, "cudasp_scan batch of %u rows failed: %s", n, cudasp_last_error());
    HOST_HIP(hipMemcpyAsync(s.h_flags, s.d_flags, n, hipMemcpyDeviceToHost, st));
    HOST_HIP(hipEventRecord(s.done, st));
    s.in_flight = true;
    s.launched_rows = n;
  }
  l.cur ^= 1;
  return harvest(g, l, l.slots[l.cur]);
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
  // Reference: cudaGetDeviceCount, falling back to 1 (:129-132).
  g->num_gpus = cudasp_device_count();
  if (g->num_gpus <= 0) g->num_gpus = 1;
  for (int d = 0; d < g->num_gpus; d++) g->device_map.push_back(d);
  // Test hook: CUDASP_TF_DEVICE_MAP="0,0" makes the host see 2 logical GPUs
  // that both run on device 0, so the num_gpus > 1 round-robin can be
  // exercised on a one-GPU box.
  if (const char* m = getenv("CUDASP_TF_DEVICE_MAP")) {
    std::vector<int> map;
    const int ndev = cudasp_device_count();
    for (const char* p = m; *p;) {
      char* end = nullptr;
      const long d = strtol(p, &end, 10);
      if (end == p || d < 0 || (ndev > 0 && d >= ndev)) {
        delete g;
        return host_fail(CUDASP_ERR_INVALID_ARG, "CUDASP_TF_DEVICE_MAP: bad device list \"%s\"", m);
      }
      map.push_back((int)d);
      p = *end == ',' ? end + 1 : end;
    }
    if (!map.empty()) {
      g->device_map = map;
      g->num_gpus = (int)map.size();
    }
  }
  *out = g;
  return CUDASP_OK;
}

void cudasp_tf_global_free(cudasp_tf_global* g) { delete g; }

int cudasp_tf_num_gpus(const cudasp_tf_global* g) { return g ? g->num_gpus : 0; }

int cudasp_tf_local_init(cudasp_tf_global* g, cudasp_tf_local** out) {
  if (!g || !out) return host_fail(CUDASP_ERR_INVALID_ARG, "null argument");
  g->currently_adding++;
  auto* l = new cudasp_tf_local();
  // Round-robin per thread (src/cudasp_extension.cu:523-529).
  l->assigned_gpu = g->num_gpus > 1 ? (int)cudasp_assign_gpu((uint64_t)g->next_gpu_assignment.fetch_add(1),
                                                             (uint32_t)g->num_gpus)
                                    : 0;
  l->device = g->device_map.empty() ? l->assigned_gpu : g->device_map[l->assigned_gpu];
  *out = l;
  return CUDASP_OK;
}

void cudasp_tf_local_free(cudasp_tf_local* l) {
  if (!l) return;
  free_local_gpu(*l);
  delete l;
}

int cudasp_tf_local_gpu(const cudasp_tf_local* l) { return l ? l->assigned_gpu : -1; }

int cudasp_tf_local_device(const cudasp_tf_local* l) { return l ? l->device : -1; }

uint32_t cudasp_assign_gpu(uint64_t ordinal, uint32_t num_gpus) {
  return num_gpus > 1 ? (uint32_t)(ordinal % num_gpus) : 0u;
}

void cudasp_tf_release_pool(void) {
  std::vector<GpuCtx*> all;
  {
    std::lock_guard<std::mutex> lock(g_pool_mu);
    all.swap(g_pool);
  }
  for (GpuCtx* c : all) release_ctx(c);
}

uint32_t cudasp_tf_pool_size(void) {
  std::lock_guard<std::mutex> lock(g_pool_mu);
  return (uint32_t)g_pool.size();
}

int cudasp_tf_function(const cudasp_tf_bind_data* b, cudasp_tf_global* g, cudasp_tf_local* l,
                       const cudasp_tf_chunk* chunk) {
  if (!b || !g || !l || !chunk) return host_fail(CUDASP_ERR_INVALID_ARG, "null argument");
  // The batch slots hold batch_size + one vector of rows (the >= batch_size
  // trigger runs after each chunk), so a chunk may not exceed one vector.
  if (chunk->count > CUDASP_TF_VECTOR_SIZE)
    return host_fail(CUDASP_ERR_INVALID_ARG, "chunk of %u rows exceeds the vector size %d", chunk->count,
                     CUDASP_TF_VECTOR_SIZE);
  if (chunk->count > 0) {
    int rc = accumulate(*b, *l, *chunk);
    if (rc != CUDASP_OK) return rc;
    // ShouldProcessBatch: accumulated >= batch_size (:416-418).
    if (l->rows() >= b->batch_size) {
      rc = launch_batch(*b, *g, *l);
      if (rc != CUDASP_OK) return rc;
    }
  }
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
  // DuckDB-sized pieces, with the same trigger as cudasp_tf_function.
  for (uint64_t r0 = 0; r0 < c.count; r0 += CUDASP_TF_VECTOR_SIZE) {
    const uint64_t r1 = r0 + CUDASP_TF_VECTOR_SIZE < c.count ? r0 + CUDASP_TF_VECTOR_SIZE : c.count;
    int rc = accumulate_columns(*b, *l, c, r0, r1);
    if (rc != CUDASP_OK) return rc;
    if (l->rows() >= b->batch_size) {
      rc = launch_batch(*b, *g, *l);
      if (rc != CUDASP_OK) return rc;
    }
  }
  return CUDASP_TF_NEED_MORE_INPUT;
}

int cudasp_tf_final(const cudasp_tf_bind_data* b, cudasp_tf_global* g, cudasp_tf_local* l, cudasp_tf_output* out) {
  if (!b || !g || !l || !out) return host_fail(CUDASP_ERR_INVALID_ARG, "null argument");
  out->count = 0;
  if (!l->finalized) {
    // Flush this thread's last rows and wait for both slots.
    int rc = CUDASP_OK;
    if (l->rows() > 0) rc = launch_batch(*b, *g, *l);
    for (HostSlot& s : l->slots)
      if (rc == CUDASP_OK) rc = harvest(*g, *l, s);
    if (rc != CUDASP_OK) return rc;
  }
  if (!l->finalized) {
    std::lock_guard<std::mutex> lock(g->finalize_lock);
    g->currently_adding--;
    l->finalized = true;
  }
  if (!l->is_output_thread) {
    if (g->currently_adding.load() != 0) return CUDASP_TF_FINISHED;
    bool expected = false;
    if (!g->output_thread_claimed.compare_exchange_strong(expected, true)) return CUDASP_TF_FINISHED;
    l->is_output_thread = true;
  }
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
