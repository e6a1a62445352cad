// End-to-end rate of the table-function host (include/cudasp_host.h): a
// synthetic columnar table in host memory is fed to T executor threads in
// DuckDB-sized chunks (<= 2048 rows, handed out like morsels), through bind ->
// local init -> in_out_function -> in_out_function_final, exactly the calls a
// DuckDB executor makes (duckdb_ext/cudasp_extension.cpp).  This is the
// PCIe-inclusive counterpart of bench.py's device-resident number (it includes
// host accumulation, H2D of tweaks and outputs, D2H of flags and the emit).
//
//   host_e2e [rows] [threads] [batch_size] [labels] [outputs_per_row]
// Prints one JSON line.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "../include/cudasp_abi.h"
#include "../include/cudasp_host.h"

static const char* SCAN_HEX = "2c1f0cb94db3946522cc1487256535dd33a1f911946baff817a72880064e690f";
static const char* SPEND_HEX =
    "36cf8fcd4d4890ab6c1083aeb5b50c260c20acda7839120e3575836f6d85c95ce0d705e31ff9fdcce67a8f3598871c6dfbe6bcde8a51cb7b48b0f95be0ea94de";
static const char* LABEL_HEX =
    "cd63f9212a2deebde8a71e9ea23f6f958c47c41d2ed74b9617fe6fb554d1524e292fabddbdcbb643eafc328875c46d75a1d697b2b31c42d38aa93f85eab34bc1";
// SHA256("cudasp-synth-v1") mod n, little-endian (same s0 as bench.py)
static void synth_s0(uint8_t out[32]);

static void hex2bin(const char* h, uint8_t* out) {
  size_t n = strlen(h) / 2;
  for (size_t i = 0; i < n; i++) sscanf(h + 2 * i, "%2hhx", &out[i]);
}

static uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

#define CK(x)                                                                             \
  do {                                                                                    \
    int rc_ = (x);                                                                        \
    if (rc_ < 0) {                                                                        \
      fprintf(stderr, "%s failed (%d): %s\n", #x, rc_, cudasp_last_error());              \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)
#define HK(x)                                                                             \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess) {                                                               \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                             \
      exit(1);                                                                            \
    }                                                                                     \
  } while (0)

int main(int argc, char** argv) {
  // As the DuckDB extension does when it loads (duckdb_ext/cudasp_extension.cpp):
  // 16 hardware queues unless the environment sets a value; before any HIP call.
  setenv("GPU_MAX_HW_QUEUES", "16", 0);
  uint64_t rows = argc > 1 ? strtoull(argv[1], 0, 10) : 32700000ull;
  int threads = argc > 2 ? atoi(argv[2]) : 16;
  int64_t batch = argc > 3 ? atoll(argv[3]) : 300000;
  int nlabels = argc > 4 ? atoi(argv[4]) : 0;
  int k = argc > 5 ? atoi(argv[5]) : 2;
  // "rows": DuckDB-style 2048-row chunks of per-row pointers (cudasp_tf_function);
  // "columns": Arrow-layout column runs (cudasp_tf_function_columns).
  const bool columnar = argc > 6 && strcmp(argv[6], "columns") == 0;
  uint8_t scan[32], spend[64], label[64];
  hex2bin(SCAN_HEX, scan);
  hex2bin(SPEND_HEX, spend);
  hex2bin(LABEL_HEX, label);
  std::vector<uint8_t> labels;
  for (int j = 0; j < nlabels; j++) labels.insert(labels.end(), label, label + 64);  // same key repeated

  // ---------------- synthetic table (generation not timed) -----------------
  auto g0 = std::chrono::steady_clock::now();
  std::vector<uint8_t> tweaks(rows * 64);
  std::vector<uint8_t> txids(rows * 32, 0);
  std::vector<int32_t> heights(rows);
  std::vector<int64_t> outputs(rows * (uint64_t)k);
  std::vector<uint64_t> list_off(rows), list_len(rows, (uint64_t)k);
  // Arrow-layout offsets for the columnar mode (int32, rows + 1 entries)
  std::vector<int32_t> txid_offsets(rows + 1), list_off32(rows + 1);
  for (uint64_t i = 0; i <= rows; i++) {
    txid_offsets[i] = (int32_t)(i * 32);
    list_off32[i] = (int32_t)(i * k);
  }
  uint8_t s0[32];
  synth_s0(s0);
  const uint32_t chunk = 1u << 22;
  uint32_t *d_x, *d_y;
  int64_t* d_vals;
  HK(hipMalloc(&d_x, (size_t)chunk * 32));
  HK(hipMalloc(&d_y, (size_t)chunk * 32));
  std::vector<uint32_t> hx((size_t)chunk * 8), hy((size_t)chunk * 8);
  for (uint64_t base = 0; base < rows; base += chunk) {
    uint32_t m = (uint32_t)std::min<uint64_t>(chunk, rows - base);
    CK(cudasp_synth_tweak_columns(0, s0, base, m, d_x, d_y, nullptr));
    HK(hipDeviceSynchronize());
    HK(hipMemcpy(hx.data(), d_x, (size_t)m * 32, hipMemcpyDeviceToHost));
    HK(hipMemcpy(hy.data(), d_y, (size_t)m * 32, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < m; i++) {
      uint32_t* row = (uint32_t*)(tweaks.data() + (base + i) * 64);
      for (int j = 0; j < 8; j++) {
        row[j] = hx[(size_t)j * m + i];
        row[8 + j] = hy[(size_t)j * m + i];
      }
    }
  }
  for (uint64_t i = 0; i < rows; i++) {
    for (int b = 0; b < 8; b++) txids[i * 32 + 31 - b] = (uint8_t)(i >> (8 * b));
    heights[i] = 800000 + (int32_t)(i / 4000);
    list_off[i] = i * k;
    for (int j = 0; j < k; j++) outputs[i * k + j] = (int64_t)splitmix64(0xC0DA5EEDull ^ (i * k + j));
  }
  // plant the true base value on every 1000th row (computed by the kernels)
  uint64_t planted = 0;
  {
    cudasp_scanner* sc;
    std::vector<uint64_t> idx;
    for (uint64_t i = 0; i < rows; i += 1000) idx.push_back(i);
    uint32_t m = (uint32_t)idx.size();
    CK(cudasp_scanner_create(0, scan, spend, labels.data(), nlabels, m, &sc));
    std::vector<uint32_t> px((size_t)m * 8), py((size_t)m * 8);
    for (uint32_t r = 0; r < m; r++) {
      const uint32_t* row = (const uint32_t*)(tweaks.data() + idx[r] * 64);
      for (int j = 0; j < 8; j++) {
        px[(size_t)j * m + r] = row[j];
        py[(size_t)j * m + r] = row[8 + j];
      }
    }
    uint32_t *dpx, *dpy, *dt;
    HK(hipMalloc(&dpx, (size_t)m * 32));
    HK(hipMalloc(&dpy, (size_t)m * 32));
    HK(hipMalloc(&dt, (size_t)m * 32));
    HK(hipMalloc(&d_vals, (size_t)m * 8 * (1 + nlabels)));
    HK(hipMemcpy(dpx, px.data(), (size_t)m * 32, hipMemcpyHostToDevice));
    HK(hipMemcpy(dpy, py.data(), (size_t)m * 32, hipMemcpyHostToDevice));
    CK(cudasp_row_values_device(sc, dpx, dpy, m, dt, d_vals, nullptr));
    CK(cudasp_scanner_sync(sc));
    std::vector<int64_t> vals(m);
    HK(hipMemcpy(vals.data(), d_vals, (size_t)m * 8, hipMemcpyDeviceToHost));
    for (uint32_t r = 0; r < m; r++) outputs[idx[r] * k] = vals[r];
    planted = m;
    cudasp_scanner_destroy(sc);
  }
  double gen_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - g0).count();

  // ---------------- the query --------------------------------------------
  char stats[512] = "";
  auto run = [&](double* secs, uint64_t* found) {
    cudasp_tf_blob_arg a_scan{scan, 32, 1}, a_spend{spend, 64, 1};
    std::vector<cudasp_tf_blob_arg> a_lab(nlabels);
    for (int j = 0; j < nlabels; j++) a_lab[j] = {labels.data() + 64 * j, 64, 1};
    cudasp_tf_bind_data* bd;
    char err[512];
    if (cudasp_tf_bind(4, a_scan, a_spend, 1, a_lab.data(), nlabels, 1, 1, batch, &bd, err, sizeof(err)) != 0) {
      fprintf(stderr, "bind: %s\n", err);
      exit(1);
    }
    cudasp_tf_global* gs;
    CK(cudasp_tf_init(bd, &gs));
    std::vector<cudasp_tf_local*> ls(threads);
    for (int t = 0; t < threads; t++) CK(cudasp_tf_local_init(gs, &ls[t]));
    std::atomic<uint64_t> next{0};
    std::atomic<uint64_t> emitted{0};
    // per thread: seconds inside the table-function calls, inside final (the
    // last batch and the wait for it), and until the thread is done
    std::vector<double> t_calls(threads, 0.0), t_final(threads, 0.0), t_done(threads, 0.0), t_long(threads, 0.0);
    auto t0 = std::chrono::steady_clock::now();
    auto now_s = [&t0]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
    std::vector<std::thread> th;
    for (int t = 0; t < threads && columnar; t++) {
      th.emplace_back([&, t]() {
        const uint64_t piece = 65536;
        for (;;) {
          uint64_t c0 = next.fetch_add(piece);
          if (c0 >= rows) break;
          cudasp_tf_columns c{};
          c.count = std::min<uint64_t>(piece, rows - c0);
          c.txid_offsets = txid_offsets.data();
          c.txid_data = txids.data();
          c.txid_offset = c0;
          c.height = heights.data();
          c.height_offset = c0;
          c.tweak_data = tweaks.data();
          c.tweak_fixed_width = 64;
          c.tweak_offset = c0;
          c.list_offsets = list_off32.data();
          c.list_offset = c0;
          c.child_values = outputs.data();
          const double c0s = now_s();
          CK(cudasp_tf_function_columns(bd, gs, ls[t], &c));
          const double dt = now_s() - c0s;
          t_calls[t] += dt;
          if (dt > 5e-4) t_long[t] += dt;  // calls that launched a batch / waited for one
        }
        const double f0s = now_s();
        cudasp_tf_output* out = new cudasp_tf_output;
        for (;;) {
          int rc = cudasp_tf_final(bd, gs, ls[t], out);
          CK(rc);
          emitted += out->count;
          if (rc != CUDASP_TF_HAVE_MORE_OUTPUT) break;
        }
        delete out;
        t_final[t] = now_s() - f0s;
        t_done[t] = now_s();
      });
    }
    for (int t = 0; t < threads && !columnar; t++) {
      th.emplace_back([&, t]() {
        std::vector<const uint8_t*> txp(CUDASP_TF_VECTOR_SIZE), twp(CUDASP_TF_VECTOR_SIZE);
        std::vector<uint32_t> txs(CUDASP_TF_VECTOR_SIZE, 32), tws(CUDASP_TF_VECTOR_SIZE, 64);
        std::vector<uint64_t> loff(CUDASP_TF_VECTOR_SIZE);
        for (;;) {
          uint64_t c0 = next.fetch_add(CUDASP_TF_VECTOR_SIZE);
          if (c0 >= rows) break;
          uint32_t cnt = (uint32_t)std::min<uint64_t>(CUDASP_TF_VECTOR_SIZE, rows - c0);
          for (uint32_t i = 0; i < cnt; i++) {
            txp[i] = txids.data() + (c0 + i) * 32;
            twp[i] = tweaks.data() + (c0 + i) * 64;
            loff[i] = list_off[c0 + i] - list_off[c0];
          }
          cudasp_tf_chunk c{};
          c.count = cnt;
          c.txid_data = txp.data();
          c.txid_size = txs.data();
          c.height = heights.data() + c0;
          c.tweak_data = twp.data();
          c.tweak_size = tws.data();
          c.list_offset = loff.data();
          c.list_length = list_len.data() + c0;
          c.child_values = outputs.data() + list_off[c0];
          const double c0s = now_s();
          CK(cudasp_tf_function(bd, gs, ls[t], &c));
          const double dt = now_s() - c0s;
          t_calls[t] += dt;
          if (dt > 5e-4) t_long[t] += dt;  // calls that launched a batch / waited for one
        }
        const double f0s = now_s();
        cudasp_tf_output* out = new cudasp_tf_output;
        for (;;) {
          int rc = cudasp_tf_final(bd, gs, ls[t], out);
          CK(rc);
          emitted += out->count;
          if (rc != CUDASP_TF_HAVE_MORE_OUTPUT) break;
        }
        delete out;
        t_final[t] = now_s() - f0s;
        t_done[t] = now_s();
      });
    }
    for (auto& x : th) x.join();
    *secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    *found = emitted.load();
    auto mean = [](const std::vector<double>& v) { double a = 0; for (double x : v) a += x; return a / v.size(); };
    snprintf(stats, sizeof(stats),
             "\"thread_call_s_mean\": %.4f, \"thread_long_call_s_mean\": %.4f, \"thread_final_s_mean\": %.4f, "
             "\"thread_done_s_min\": %.4f, \"thread_done_s_max\": %.4f",
             mean(t_calls), mean(t_long), mean(t_final), *std::min_element(t_done.begin(), t_done.end()),
             *std::max_element(t_done.begin(), t_done.end()));
    for (auto* l : ls) cudasp_tf_local_free(l);
    cudasp_tf_global_free(gs);
    cudasp_tf_bind_free(bd);
  };
  double warm_s;
  uint64_t warm_found;
  run(&warm_s, &warm_found);  // warm-up (scanner creation, table build)
  double secs;
  uint64_t found;
  run(&secs, &found);
  printf("{\"what\": \"table-function host end-to-end (host memory -> matches, PCIe-inclusive)\", \"input\": \"%s\", "
         "\"rows\": %llu, \"threads\": %d, \"batch_size\": %lld, \"labels\": %d, \"outputs_per_row\": %d, "
         "\"seconds\": %.4f, \"tx_per_s\": %.1f, \"matches\": %llu, \"planted\": %llu, \"warmup_seconds\": %.3f, "
         "\"generate_seconds\": %.2f, \"devices\": %d, \"gpu_max_hw_queues\": \"%s\", %s}\n",
         columnar ? "arrow columns" : "2048-row chunks", (unsigned long long)rows, threads, (long long)batch, nlabels,
         k, secs, rows / secs,
         (unsigned long long)found, (unsigned long long)planted, warm_s, gen_s, cudasp_device_count(),
         getenv("GPU_MAX_HW_QUEUES") ? getenv("GPU_MAX_HW_QUEUES") : "", stats);
  return found == planted ? 0 : 2;
}

// SHA-256 of "cudasp-synth-v1" reduced mod n (precomputed by bench.py's formula).
static void synth_s0(uint8_t out[32]) {
  // int.from_bytes(sha256(b"cudasp-synth-v1"), "big") % n, little-endian
  static const char* S0_LE_HEX = "f59571862b00db0109281d9bf2326d7eaf05b1b837ccafce4c2e335f439cf6ab";
  hex2bin(S0_LE_HEX, out);
}
