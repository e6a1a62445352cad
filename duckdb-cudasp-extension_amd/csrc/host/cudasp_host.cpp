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
//   * a failed batch is reported (cudasp_tf_function/final return an error)
//     instead of being dropped silently (:325, :378);
//   * a tweak_key BLOB that is not 64 bytes is an error instead of an
//     out-of-bounds read (:333, ConvertTweakKeyToU32 always reads 64 bytes).
#include "../../../include/cudasp_host.h"

#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../../include/cudasp_abi.h"

namespace {

constexpr uint64_t TWEAK_KEY_SIZE = 64;  // CudaspScanBindData::TWEAK_KEY_SIZE
constexpr uint64_t SCALAR_SIZE = 32;     // CudaspScanBindData::SCALAR_SIZE

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
  std::string scan_private_key_data;
  std::string spend_public_key_data;
  std::vector<std::string> label_keys_data;
  std::string label_keys_flat;  // label_count x 64, back to back
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
};

struct cudasp_tf_local {
  bool finalized = false;
  bool is_output_thread = false;
  int assigned_gpu = -1;
  // accumulated rows, flat
  std::vector<uint8_t> txid_bytes;
  std::vector<uint64_t> txid_offset;
  std::vector<uint32_t> txid_size;
  std::vector<int32_t> heights;
  std::vector<uint8_t> tweaks;  // n x 64
  std::vector<int64_t> outputs;
  std::vector<uint32_t> output_offset;
  std::vector<uint32_t> output_length;
  std::vector<uint8_t> flags;
  cudasp_scanner* scanner = nullptr;
  uint32_t rows() const { return (uint32_t)heights.size(); }
  void clear() {
    txid_bytes.clear();
    txid_offset.clear();
    txid_size.clear();
    heights.clear();
    tweaks.clear();
    outputs.clear();
    output_offset.clear();
    output_length.clear();
  }
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

// AccumulateInput (src/cudasp_extension.cu:154-224).
int accumulate(cudasp_tf_local& l, const cudasp_tf_chunk& c) {
  for (uint32_t i = 0; i < c.count; i++) {
    // Only rows with valid txid, height and tweak_key (:195-197).
    if (!(valid(c.txid_valid, i) && valid(c.height_valid, i) && valid(c.tweak_valid, i))) continue;
    if (c.tweak_size[i] != TWEAK_KEY_SIZE)
      return host_fail(CUDASP_ERR_INVALID_ARG, "tweak_key must be exactly 64 bytes, got %u bytes", c.tweak_size[i]);
    l.txid_offset.push_back(l.txid_bytes.size());
    l.txid_size.push_back(c.txid_size[i]);
    l.txid_bytes.insert(l.txid_bytes.end(), c.txid_data[i], c.txid_data[i] + c.txid_size[i]);
    l.heights.push_back(c.height[i]);
    l.tweaks.insert(l.tweaks.end(), c.tweak_data[i], c.tweak_data[i] + TWEAK_KEY_SIZE);
    // Outputs: NULL list -> length 0; NULL elements dropped (:206-221).
    l.output_offset.push_back((uint32_t)l.outputs.size());
    uint32_t len = 0;
    if (valid(c.list_valid, i)) {
      for (uint64_t k = 0; k < c.list_length[i]; k++) {
        uint64_t ci = c.list_offset[i] + k;
        if (valid(c.child_valid, (uint32_t)ci)) {
          l.outputs.push_back(c.child_values[ci]);
          len++;
        }
      }
    }
    l.output_length.push_back(len);
  }
  return CUDASP_OK;
}

// ProcessBatch (src/cudasp_extension.cu:226-410).
int process_batch(const cudasp_tf_bind_data& b, cudasp_tf_global& g, cudasp_tf_local& l) {
  uint32_t n = l.rows();
  if (n == 0) return CUDASP_OK;
  if (!l.scanner) {
    // One scanner per thread on its assigned GPU; capacity covers the largest
    // batch the >= trigger can produce (batch_size - 1 + one 2048-row chunk).
    uint64_t cap = b.batch_size + CUDASP_TF_VECTOR_SIZE;
    int rc = cudasp_scanner_create(l.assigned_gpu, (const uint8_t*)b.scan_private_key_data.data(),
                                   (const uint8_t*)b.spend_public_key_data.data(),
                                   (const uint8_t*)b.label_keys_flat.data(), (uint32_t)b.label_keys_data.size(),
                                   (uint32_t)cap, &l.scanner);
    if (rc != CUDASP_OK)
      return host_fail(rc, "Failed to create scanner on GPU %d: %s", l.assigned_gpu, cudasp_last_error());
  }
  l.flags.resize(n);
  int rc = cudasp_scan_host(l.scanner, l.tweaks.data(), l.outputs.data(), l.outputs.size(), l.output_offset.data(),
                            l.output_length.data(), n, l.flags.data());
  if (rc != CUDASP_OK) return host_fail(rc, "cudasp_scan batch of %u rows failed: %s", n, cudasp_last_error());
  {
    std::lock_guard<std::mutex> lock(g.output_lock);
    for (uint32_t i = 0; i < n; i++) {
      if (!l.flags[i]) continue;
      g.output_txids.emplace_back((const char*)l.txid_bytes.data() + l.txid_offset[i], l.txid_size[i]);
      g.output_heights.push_back(l.heights[i]);
      g.output_tweak_keys.emplace_back((const char*)l.tweaks.data() + (size_t)i * TWEAK_KEY_SIZE, TWEAK_KEY_SIZE);
    }
  }
  l.clear();
  return CUDASP_OK;
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

void cudasp_tf_bind_free(cudasp_tf_bind_data* b) { delete b; }

uint64_t cudasp_tf_bind_batch_size(const cudasp_tf_bind_data* b) { return b ? b->batch_size : 0; }

int cudasp_tf_init(const cudasp_tf_bind_data* b, cudasp_tf_global** out) {
  if (!b || !out) return host_fail(CUDASP_ERR_INVALID_ARG, "null argument");
  auto* g = new cudasp_tf_global();
  // Reference: cudaGetDeviceCount, falling back to 1 (:129-132).
  g->num_gpus = cudasp_device_count();
  if (g->num_gpus <= 0) g->num_gpus = 1;
  *out = g;
  return CUDASP_OK;
}

void cudasp_tf_global_free(cudasp_tf_global* g) { delete g; }

int cudasp_tf_num_gpus(const cudasp_tf_global* g) { return g ? g->num_gpus : 0; }

int cudasp_tf_local_init(cudasp_tf_global* g, cudasp_tf_local** out) {
  if (!g || !out) return host_fail(CUDASP_ERR_INVALID_ARG, "null argument");
  g->currently_adding++;
  auto* l = new cudasp_tf_local();
  l->assigned_gpu = g->num_gpus > 1 ? g->next_gpu_assignment.fetch_add(1) % g->num_gpus : 0;
  *out = l;
  return CUDASP_OK;
}

void cudasp_tf_local_free(cudasp_tf_local* l) {
  if (!l) return;
  if (l->scanner) cudasp_scanner_destroy(l->scanner);
  delete l;
}

int cudasp_tf_local_gpu(const cudasp_tf_local* l) { return l ? l->assigned_gpu : -1; }

int cudasp_tf_function(const cudasp_tf_bind_data* b, cudasp_tf_global* g, cudasp_tf_local* l,
                       const cudasp_tf_chunk* chunk) {
  if (!b || !g || !l || !chunk) return host_fail(CUDASP_ERR_INVALID_ARG, "null argument");
  if (chunk->count > 0) {
    int rc = accumulate(*l, *chunk);
    if (rc != CUDASP_OK) return rc;
    // ShouldProcessBatch: accumulated >= batch_size (:416-418).
    if (l->rows() >= b->batch_size) {
      rc = process_batch(*b, *g, *l);
      if (rc != CUDASP_OK) return rc;
    }
  }
  return CUDASP_TF_NEED_MORE_INPUT;
}

int cudasp_tf_final(const cudasp_tf_bind_data* b, cudasp_tf_global* g, cudasp_tf_local* l, cudasp_tf_output* out) {
  if (!b || !g || !l || !out) return host_fail(CUDASP_ERR_INVALID_ARG, "null argument");
  out->count = 0;
  if (!l->finalized && l->rows() > 0) {
    int rc = process_batch(*b, *g, *l);
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
