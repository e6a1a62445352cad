// End-to-end rate of the table-function host (include/cudasp_host.h): a
// synthetic table in host memory is fed to T executor threads in DuckDB-sized
// chunks (<= 2048 rows, handed out like morsels), through bind -> local init
// -> in_out_function -> in_out_function_final, exactly the calls a DuckDB
// executor makes (duckdb_ext/cudasp_extension.cpp).  This is the
// PCIe-inclusive counterpart of bench.py's device-resident number: it includes
// the host copies into the batch slots, H2D of tweaks and outputs, D2H of the
// flags and the emit.  The host uses every visible GPU (or the logical GPUs of
// CUDASP_TF_DEVICE_MAP).
//
// The table is bench.py's: T_g = (s0 + g) G, txid = BE64(g)
// padded to 32 bytes, height 800000 + g / 4000, outputs from the library's
// own generators (cudasp_synth_outputs: k per row; cudasp_synth_output_lengths
// / _values: 1..kmax per row, mean (kmax + 1) / 2).  Planted matches: the
// true base value on every row g = 0 mod 1000 and, with L labels, label
// j = (g / 1000) mod L's value on row g = 1 mod 1000 (every label index of
// the reference's label loop, src/cudasp_gpu.cu:153-172), computed by the
// product's values path (which the test suite pins to the oracle), written
// into the first slot of the row's outputs list.  A query passes when the
// emitted rows are exactly the planted ones (decoded from the txids).
//
//   host_e2e [--rows N] [--threads T] [--batch B] [--labels L --labels-file F]
//            [--outputs K | --outputs-max KMAX] [--input rows|columns|vectors]
//            [--reps R] [--warm-reps W [--warm-ms MS]] [--plant-sample FILE]
//            [--null-device [--cpu-table]] [--output-count K] [--label-negation]
//            [--pinned DEVICES [--hbm]] [--table-out FILE | --table-in FILE [--cold-phases]]
// (W more queries, each started right after MS ms of a busy kernel on every
// GPU: the rate at full clock, without the ramp from idle; warm_tx_per_s)
// --plant-sample writes 256 planted rows and 256 unplanted rows, strided over
// the table (row index, tweak, outputs list, the planted value's column,
// whether the last timed query emitted it) with the keys, as JSON, for a
// checker that recomputes them with the C oracle (oracle.check_planted_sample:
// the planted values above come from the GPU's own values path).
// --null-device (measurement only) sets CUDASP_TF_NULL_DEVICE=1: the host's
// feeds mark every slot done at launch, with no device work, so tx_per_s is
// the executor threads' own ceiling (reserve, copies into the pinned slots,
// harvest) -- the host's capacity to feed N GPUs; a query then passes when
// it emits nothing.  --cpu-table (with --null-device) fills the table on the
// CPU (pseudo-random tweak bytes, the same splitmix64 outputs, no plants), so
// the host's ceiling can be measured with no GPU at all.  host_call_tx_per_s
// in the output = rows / the threads' mean time inside the host's calls
// (cudasp_tf_function*): the host's own rate, without this driver's chunk
// building (DuckDB's side of the vectors).
// --output-count / --label-negation bind the protocol variants (DESIGN.md
// section 6b); the planted values stay the reference's (output index 0, labels
// added), which every variant still matches, and no other row may match.
// --pinned DEVICES (e.g. 0 or 0,0,0,0): instead of table-function queries,
// the C pinned table (cudasp_pinned_*, include/cudasp_host.h): the table is
// appended once in 65536-row Arrow runs, then scanned R + 1 times (the first
// warms the scanners and streams; each scan binds the keys like a query),
// batches round-robin over DEVICES (a device listed m times: m logical GPUs
// on it); a scan passes when its row numbers are exactly the planted rows.
// With --null-device only the appends run (no scan).  --hbm: the table
// resident in device memory instead (CUDASP_TABLE_HBM, k_scan_multi per scan).
// --table-out FILE writes the generated table (rows, outputs, plants) and
// exits; --table-in FILE reads it instead of generating, so the process makes
// no GPU call before its first query except the runtime's initialisation
// (hip_init_s, a device count): the first query then pays everything a fresh
// DuckDB process pays -- the fixed-base table, scanners, pinned slots, code
// object load -- and is reported as first_query_s beside the warm queries'
// median (cold start).  --cold-phases (with --table-in)
// times a scanner's creation on device 0 before the first query instead
// (scanner_create_s: the fixed-base table and its fold), as a breakdown;
// --prewarm calls cudasp_tf_prewarm first, as the DuckDB extension does at
// LOAD (prewarm_s), so first_query_s is then the first query after it.
// --input vectors hands each 2048-row chunk over as DuckDB holds it
// (cudasp_tf_function_vectors: string_t txids and tweaks pointing into the
// table, the heights, list_entry_t lists and the child values in place), the
// extension's pass-through form; rows builds per-row pointer arrays
// (cudasp_tf_function), columns Arrow runs (cudasp_tf_function_columns).
// Label keys: F holds L 64-byte keys (x || y, little-endian, bench.label_keys);
// without F, L must be 0 or 1 (the SQL test's label, test/sql/cudasp.test:104).
// Prints one JSON line; exit 0 iff every timed query emitted exactly the
// planted rows.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../include/cudasp_abi.h"
#include "../include/cudasp_host.h"

static const char* SCAN_HEX = "2c1f0cb94db3946522cc1487256535dd33a1f911946baff817a72880064e690f";
static const char* SPEND_HEX =
    "36cf8fcd4d4890ab6c1083aeb5b50c260c20acda7839120e3575836f6d85c95ce0d705e31ff9fdcce67a8f3598871c6dfbe6bcde8a51cb7b48b0f95be0ea94de";
static const char* LABEL_HEX =
    "cd63f9212a2deebde8a71e9ea23f6f958c47c41d2ed74b9617fe6fb554d1524e292fabddbdcbb643eafc328875c46d75a1d697b2b31c42d38aa93f85eab34bc1";
// int.from_bytes(sha256(b"cudasp-synth-v1"), "big") % n, little-endian (bench.synth_s0)
static const char* S0_LE_HEX = "f59571862b00db0109281d9bf2326d7eaf05b1b837ccafce4c2e335f439cf6ab";
static const uint64_t OUTPUT_SEED = 0xC0DA5EEDull;
static const uint64_t PLANT_EVERY = 1000;

static void hex2bin(const char* h, uint8_t* out) {
  size_t n = strlen(h) / 2;
  for (size_t i = 0; i < n; i++) sscanf(h + 2 * i, "%2hhx", &out[i]);
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

struct Args {
  uint64_t rows = 32700000ull;
  int threads = 8;
  int64_t batch = 300000;
  int labels = 0;
  std::string labels_file;
  int k = 2;     // fixed outputs per row
  int kmax = 0;  // > 0: 1..kmax outputs per row
  bool columnar = false;
  bool vectors = false;  // --input vectors: DuckDB's vectors (string_t, list_entry_t) through cudasp_tf_function_vectors
  int reps = 1;
  int warm_reps = 0;    // more queries, each right after a busy kernel on every GPU (clock at speed)
  int warm_ms = 30;
  std::string plant_sample;  // JSON sample of planted / unplanted rows for the oracle check
  bool null_device = false;  // measurement only: no device work in the host's feeds
  bool cpu_table = false;    // with null_device: table generated on the CPU, no GPU needed
  int output_count = 1;        // protocol variant: output indices per row (bind option output_count)
  bool label_negation = false;  // protocol variant: labels also negated (bind option label_negation)
  std::vector<int> pinned;      // --pinned: the pinned table's devices (empty: table-function queries)
  bool hbm = false;             // --hbm: CUDASP_TABLE_HBM placement
  std::string table_out, table_in;  // --table-out / --table-in FILE
  bool cold_phases = false;     // --cold-phases: time a scanner's creation before the first query
  bool prewarm = false;         // --prewarm: cudasp_tf_prewarm before the first query (the extension's LOAD)
};

static Args parse(int argc, char** argv) {
  Args a;
  for (int i = 1; i < argc; i++) {
    std::string s = argv[i];
    auto val = [&]() -> const char* {
      if (i + 1 >= argc) {
        fprintf(stderr, "%s needs a value\n", s.c_str());
        exit(1);
      }
      return argv[++i];
    };
    if (s == "--rows") a.rows = strtoull(val(), 0, 10);
    else if (s == "--threads") a.threads = atoi(val());
    else if (s == "--batch") a.batch = atoll(val());
    else if (s == "--labels") a.labels = atoi(val());
    else if (s == "--labels-file") a.labels_file = val();
    else if (s == "--outputs") a.k = atoi(val());
    else if (s == "--outputs-max") a.kmax = atoi(val());
    else if (s == "--input") {
      const std::string v = val();
      a.columnar = v == "columns";
      a.vectors = v == "vectors";
      if (!a.columnar && !a.vectors && v != "rows") {
        fprintf(stderr, "--input rows|columns|vectors\n");
        exit(1);
      }
    }
    else if (s == "--reps") a.reps = std::max(1, atoi(val()));
    else if (s == "--warm-reps") a.warm_reps = std::max(0, atoi(val()));
    else if (s == "--warm-ms") a.warm_ms = std::max(1, atoi(val()));
    else if (s == "--plant-sample") a.plant_sample = val();
    else if (s == "--null-device") a.null_device = true;
    else if (s == "--cpu-table") a.cpu_table = true;
    else if (s == "--output-count") a.output_count = atoi(val());
    else if (s == "--label-negation") a.label_negation = true;
    else if (s == "--hbm") a.hbm = true;
    else if (s == "--table-out") a.table_out = val();
    else if (s == "--table-in") a.table_in = val();
    else if (s == "--cold-phases") a.cold_phases = true;
    else if (s == "--prewarm") a.prewarm = true;
    else if (s == "--pinned") {
      std::string v = val();
      for (size_t p = 0; p <= v.size();) {
        const size_t q = v.find(',', p);
        a.pinned.push_back(atoi(v.substr(p, q == std::string::npos ? std::string::npos : q - p).c_str()));
        if (q == std::string::npos) break;
        p = q + 1;
      }
    }
    else {
      fprintf(stderr, "unknown argument %s\n", s.c_str());
      exit(1);
    }
  }
  if (a.threads < 1 || a.rows == 0 || (a.kmax == 0 && a.k < 1) || a.kmax < 0 || a.labels < 0 ||
      (a.cpu_table && !a.null_device)) {
    fprintf(stderr, "bad arguments\n");
    exit(1);
  }
  return a;
}

struct Table {
  uint64_t rows = 0;
  std::vector<uint8_t> tweaks, txids;
  std::vector<int32_t> heights;
  std::vector<int64_t> outputs;
  std::vector<uint64_t> list_off, list_len;         // list entries (offset into outputs, length)
  std::vector<uint64_t> planted;                    // planted row indices, sorted
  std::vector<int> planted_col;                     // their values column: 0 = base, 1 + j = label j
  uint32_t labels_planted_mask = 0;                 // label indices planted (bit j)
};

static uint64_t splitmix64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// --cpu-table: the table's shape without a GPU (tweak bytes are not curve
// points; nothing is scanned, --null-device only).
static void generate_cpu(const Args& a, Table& t) {
  const uint64_t rows = t.rows = a.rows;
  t.tweaks.resize(rows * 64);
  t.txids.assign(rows * 32, 0);
  t.heights.resize(rows);
  t.list_off.resize(rows);
  t.list_len.resize(rows);
  uint64_t* tw = reinterpret_cast<uint64_t*>(t.tweaks.data());
  for (uint64_t i = 0; i < rows * 8; i++) tw[i] = splitmix64(i);
  t.outputs.reserve(a.kmax ? rows * (a.kmax + 1) / 2 : rows * a.k);
  for (uint64_t g = 0; g < rows; g++) {
    const uint32_t len = a.kmax ? 1u + (uint32_t)(splitmix64(~OUTPUT_SEED ^ g) % a.kmax) : (uint32_t)a.k;
    t.list_off[g] = t.outputs.size();
    t.list_len[g] = len;
    for (uint32_t j = 0; j < len; j++) t.outputs.push_back((int64_t)splitmix64(OUTPUT_SEED ^ (g * len + j)));
    for (int b = 0; b < 8; b++) t.txids[g * 32 + 31 - b] = (uint8_t)(g >> (8 * b));
    t.heights[g] = 800000 + (int32_t)(g / 4000);
  }
}

static void generate(const Args& a, const uint8_t scan[32], const uint8_t spend[64],
                     const std::vector<uint8_t>& labels, Table& t) {
  if (a.cpu_table) {
    generate_cpu(a, t);
    return;
  }
  const uint64_t rows = t.rows = a.rows;
  t.tweaks.resize(rows * 64);
  t.txids.assign(rows * 32, 0);
  t.heights.resize(rows);
  t.list_off.resize(rows);
  t.list_len.resize(rows);
  uint8_t s0[32];
  hex2bin(S0_LE_HEX, s0);
  const uint32_t chunk = 1u << 22;
  const uint32_t kcap = a.kmax ? (uint32_t)a.kmax : (uint32_t)a.k;
  uint32_t *d_x, *d_y, *d_offs, *d_lens;
  int64_t* d_outs;
  HK(hipMalloc(&d_x, (size_t)chunk * 32));
  HK(hipMalloc(&d_y, (size_t)chunk * 32));
  HK(hipMalloc(&d_offs, (size_t)chunk * 4));
  HK(hipMalloc(&d_lens, (size_t)chunk * 4));
  HK(hipMalloc(&d_outs, (size_t)chunk * kcap * 8));
  std::vector<uint32_t> hx((size_t)chunk * 8), hy((size_t)chunk * 8), hl(chunk), ho(chunk);
  t.outputs.reserve(a.kmax ? rows * (a.kmax + 1) / 2 + rows / 8 : rows * a.k);
  for (uint64_t base = 0; base < rows; base += chunk) {
    const uint32_t m = (uint32_t)std::min<uint64_t>(chunk, rows - base);
    CK(cudasp_synth_tweak_columns(0, s0, base, m, d_x, d_y, nullptr));
    if (a.kmax) {
      CK(cudasp_synth_output_lengths(OUTPUT_SEED, base, m, (uint32_t)a.kmax, d_lens, nullptr));
      HK(hipDeviceSynchronize());
      HK(hipMemcpy(hl.data(), d_lens, (size_t)m * 4, hipMemcpyDeviceToHost));
      uint32_t acc = 0;
      for (uint32_t i = 0; i < m; i++) {
        ho[i] = acc;
        acc += hl[i];
      }
      HK(hipMemcpy(d_offs, ho.data(), (size_t)m * 4, hipMemcpyHostToDevice));
      CK(cudasp_synth_output_values(OUTPUT_SEED, base, m, d_offs, d_lens, d_outs, nullptr));
    } else {
      CK(cudasp_synth_outputs(OUTPUT_SEED, base, m, (uint32_t)a.k, d_outs, d_offs, d_lens, nullptr));
      HK(hipDeviceSynchronize());
      HK(hipMemcpy(hl.data(), d_lens, (size_t)m * 4, hipMemcpyDeviceToHost));
      HK(hipMemcpy(ho.data(), d_offs, (size_t)m * 4, hipMemcpyDeviceToHost));
    }
    HK(hipDeviceSynchronize());
    HK(hipMemcpy(hx.data(), d_x, (size_t)m * 32, hipMemcpyDeviceToHost));
    HK(hipMemcpy(hy.data(), d_y, (size_t)m * 32, hipMemcpyDeviceToHost));
    const uint64_t nouts = (uint64_t)ho[m - 1] + hl[m - 1];
    const size_t out0 = t.outputs.size();
    t.outputs.resize(out0 + nouts);
    HK(hipMemcpy(t.outputs.data() + out0, d_outs, nouts * 8, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < m; i++) {
      const uint64_t g = base + i;
      uint32_t* row = (uint32_t*)(t.tweaks.data() + g * 64);
      for (int j = 0; j < 8; j++) {
        row[j] = hx[(size_t)j * m + i];
        row[8 + j] = hy[(size_t)j * m + i];
      }
      for (int b = 0; b < 8; b++) t.txids[g * 32 + 31 - b] = (uint8_t)(g >> (8 * b));
      t.heights[g] = 800000 + (int32_t)(g / 4000);
      t.list_off[g] = out0 + ho[i];
      t.list_len[g] = hl[i];
    }
  }
  HK(hipFree(d_x));
  HK(hipFree(d_y));
  HK(hipFree(d_offs));
  HK(hipFree(d_lens));
  HK(hipFree(d_outs));

  // ---- planted values: base on g = 0 mod 1000, label j on g = 1 mod 1000
  const int L = a.labels;
  std::vector<uint64_t> idx;
  std::vector<int> lab;  // -1 = base, else label index
  for (uint64_t g = 0; g < rows; g += PLANT_EVERY) {
    idx.push_back(g);
    lab.push_back(-1);
    if (L && g + 1 < rows) {
      idx.push_back(g + 1);
      lab.push_back((int)((g / PLANT_EVERY) % L));
    }
  }
  const uint32_t m = (uint32_t)idx.size();
  cudasp_scanner* sc;
  CK(cudasp_scanner_create(0, scan, spend, L ? labels.data() : nullptr, (uint32_t)L, m, &sc));
  std::vector<uint32_t> px((size_t)m * 8), py((size_t)m * 8);
  for (uint32_t r = 0; r < m; r++) {
    const uint32_t* row = (const uint32_t*)(t.tweaks.data() + idx[r] * 64);
    for (int j = 0; j < 8; j++) {
      px[(size_t)j * m + r] = row[j];
      py[(size_t)j * m + r] = row[8 + j];
    }
  }
  uint32_t *dpx, *dpy, *dt;
  int64_t* dv;
  HK(hipMalloc(&dpx, (size_t)m * 32));
  HK(hipMalloc(&dpy, (size_t)m * 32));
  HK(hipMalloc(&dt, (size_t)m * 32));
  HK(hipMalloc(&dv, (size_t)m * 8 * (1 + L)));
  HK(hipMemcpy(dpx, px.data(), (size_t)m * 32, hipMemcpyHostToDevice));
  HK(hipMemcpy(dpy, py.data(), (size_t)m * 32, hipMemcpyHostToDevice));
  CK(cudasp_row_values_device(sc, dpx, dpy, m, dt, dv, nullptr));
  CK(cudasp_scanner_sync(sc));
  std::vector<int64_t> vals((size_t)m * (1 + L));
  HK(hipMemcpy(vals.data(), dv, vals.size() * 8, hipMemcpyDeviceToHost));
  for (uint32_t r = 0; r < m; r++) {
    const int v = lab[r] < 0 ? 0 : 1 + lab[r];  // values row: 0 = base, 1 + j = label j
    t.outputs[t.list_off[idx[r]]] = vals[(size_t)v * m + r];
    if (lab[r] >= 0) t.labels_planted_mask |= 1u << (lab[r] & 31);
  }
  t.planted = idx;  // ascending: g, then g + 1 for the label plant
  t.planted_col.resize(m);
  for (uint32_t r = 0; r < m; r++) t.planted_col[r] = lab[r] < 0 ? 0 : 1 + lab[r];
  HK(hipFree(dpx));
  HK(hipFree(dpy));
  HK(hipFree(dt));
  HK(hipFree(dv));
  cudasp_scanner_destroy(sc);
}

// --table-out / --table-in: the table as little-endian binary vectors.
template <class T>
static bool put(FILE* f, const std::vector<T>& v) {
  const uint64_t n = v.size();
  return fwrite(&n, 8, 1, f) == 1 && (n == 0 || fwrite(v.data(), sizeof(T), n, f) == n);
}
template <class T>
static bool get(FILE* f, std::vector<T>& v) {
  uint64_t n = 0;
  if (fread(&n, 8, 1, f) != 1 || n > (1ull << 40) / sizeof(T)) return false;
  v.resize(n);
  return n == 0 || fread(v.data(), sizeof(T), n, f) == n;
}
static const uint64_t TABLE_MAGIC = 0x31656c6261745045ull;  // "EPtable1"

static bool write_table(const std::string& path, const Table& t) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) return false;
  bool ok = fwrite(&TABLE_MAGIC, 8, 1, f) == 1 && fwrite(&t.rows, 8, 1, f) == 1 &&
            fwrite(&t.labels_planted_mask, 4, 1, f) == 1 && put(f, t.tweaks) && put(f, t.txids) &&
            put(f, t.heights) && put(f, t.outputs) && put(f, t.list_off) && put(f, t.list_len) &&
            put(f, t.planted) && put(f, t.planted_col);
  return fclose(f) == 0 && ok;
}

static bool read_table(const std::string& path, Table& t) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  uint64_t magic = 0;
  bool ok = fread(&magic, 8, 1, f) == 1 && magic == TABLE_MAGIC && fread(&t.rows, 8, 1, f) == 1 &&
            fread(&t.labels_planted_mask, 4, 1, f) == 1 && get(f, t.tweaks) && get(f, t.txids) &&
            get(f, t.heights) && get(f, t.outputs) && get(f, t.list_off) && get(f, t.list_len) &&
            get(f, t.planted) && get(f, t.planted_col);
  fclose(f);
  return ok && t.tweaks.size() == t.rows * 64 && t.list_off.size() == t.rows;
}

struct QueryResult {
  double secs = 0;
  uint64_t emitted = 0;
  bool exact = false;  // emitted rows == planted rows
  cudasp_tf_stats stats{};
  int logical_gpus = 0;
  std::vector<uint64_t> got;  // emitted row indices, sorted
  double call_s_mean = 0, final_s_mean = 0, done_min = 0, done_max = 0;
};

// A GPU left idle lowers its clock, and the first milliseconds of the next
// work run below speed (tools/stream_probe.py --gap-ms / --prewarm: 100 ms of
// idle costs k_scan_multi 1.2 ms at 1M rows, 3.4 ms at 9.4M).  The warm
// queries start right after this: every wave slot busy with FMAs for `ms`
// (the 100 MHz constant clock; an iteration cap bounds it regardless).
__global__ void k_busy(uint64_t ticks, float* sink) {
  const uint64_t t0 = wall_clock64();
  float v = (float)threadIdx.x, m = 1.0000001f;
  for (uint32_t it = 0; it < (1u << 22); it++) {
#pragma unroll
    for (int j = 0; j < 32; j++) v = fmaf(v, m, 1e-7f);
    if (wall_clock64() - t0 > ticks) break;
  }
  if (v == 12345.0f) sink[threadIdx.x] = v;
}

static void busy_all_gpus(int ms) {
  int n = 0;
  HK(hipGetDeviceCount(&n));
  std::vector<float*> sinks(n);
  for (int d = 0; d < n; d++) {
    HK(hipSetDevice(d));
    HK(hipMalloc(&sinks[d], 1024 * sizeof(float)));
    hipDeviceProp_t p;
    HK(hipGetDeviceProperties(&p, d));
    k_busy<<<p.multiProcessorCount * 8, 256>>>((uint64_t)ms * 100000ull, sinks[d]);
    HK(hipGetLastError());
  }
  for (int d = 0; d < n; d++) {
    HK(hipSetDevice(d));
    HK(hipDeviceSynchronize());
    HK(hipFree(sinks[d]));
  }
  HK(hipSetDevice(0));
}

static QueryResult run_query(const Args& a, const uint8_t scan[32], const uint8_t spend[64],
                             const std::vector<uint8_t>& labels, const Table& t, int warm_ms = 0) {
  const int L = a.labels, T = a.threads;
  const uint64_t rows = t.rows;
  cudasp_tf_blob_arg a_scan{scan, 32, 1}, a_spend{spend, 64, 1};
  std::vector<cudasp_tf_blob_arg> a_lab(std::max(1, L));
  for (int j = 0; j < L; j++) a_lab[j] = {labels.data() + 64 * j, 64, 1};
  cudasp_tf_bind_data* bd;
  char err[512];
  if (cudasp_tf_bind(4, a_scan, a_spend, 1, a_lab.data(), (uint32_t)L, 1, 1, a.batch, &bd, err, sizeof(err)) != 0) {
    fprintf(stderr, "bind: %s\n", err);
    exit(1);
  }
  if ((a.output_count != 1 || a.label_negation) &&
      cudasp_tf_bind_options(bd, 1, a.output_count, 1, a.label_negation ? 1 : 0, 0, 0, err, sizeof(err)) != 0) {
    fprintf(stderr, "bind options: %s\n", err);
    exit(1);
  }
  cudasp_tf_global* gs;
  CK(cudasp_tf_init(bd, &gs));
  std::vector<cudasp_tf_local*> ls(T);
  for (int i = 0; i < T; i++) CK(cudasp_tf_local_init(gs, &ls[i]));
  std::atomic<uint64_t> next{0};
  std::vector<uint64_t> got;  // emitted row indices (from the txids)
  size_t torn = 0;            // emitted rows whose tweak or height is not their txid's row
  std::vector<double> t_calls(T, 0.0), t_final(T, 0.0), t_done(T, 0.0);
  if (warm_ms) busy_all_gpus(warm_ms);
  const auto t0 = std::chrono::steady_clock::now();
  auto now_s = [&t0]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(); };
  auto finish = [&](int th) {
    const double f0 = now_s();
    cudasp_tf_output* out = new cudasp_tf_output;
    for (;;) {
      const int rc = cudasp_tf_final(bd, gs, ls[th], out);
      CK(rc);
      for (uint32_t i = 0; i < out->count; i++) {
        uint64_t g = 0;
        for (int b = 0; b < 8; b++) g |= (uint64_t)out->txid_data[i][31 - b] << (8 * b);
        got.push_back(g);  // only the output thread gets here
        // the emitted row's other columns belong to the row its txid names
        if (g >= rows || out->txid_size[i] != 32 || out->tweak_size[i] != 64 || out->height[i] != t.heights[g] ||
            memcmp(out->tweak_data[i], t.tweaks.data() + g * 64, 64) != 0)
          torn++;
      }
      if (rc != CUDASP_TF_HAVE_MORE_OUTPUT) break;
    }
    delete out;
    t_final[th] = now_s() - f0;
    t_done[th] = now_s();
  };
  std::vector<std::thread> th;
  for (int i = 0; i < T; i++) {
    th.emplace_back([&, i]() {
      if (a.columnar) {
        // Arrow record batches of 65536 rows: int32 offsets per batch, the
        // buffers starting at the batch's first row (a 100M-row table has
        // more than 2^31 txid bytes in all)
        const uint64_t piece = 65536;
        std::vector<int32_t> txo(piece + 1), lo(piece + 1);
        for (;;) {
          const uint64_t c0 = next.fetch_add(piece);
          if (c0 >= rows) break;
          const uint64_t m = std::min<uint64_t>(piece, rows - c0);
          for (uint64_t r = 0; r <= m; r++) {
            txo[r] = (int32_t)(r * 32);
            lo[r] = (int32_t)((c0 + r < rows ? t.list_off[c0 + r] : t.outputs.size()) - t.list_off[c0]);
          }
          cudasp_tf_columns c{};
          c.count = m;
          c.txid_offsets = txo.data();
          c.txid_data = t.txids.data() + c0 * 32;
          c.height = t.heights.data() + c0;
          c.tweak_data = t.tweaks.data() + c0 * 64;
          c.tweak_fixed_width = 64;
          c.list_offsets = lo.data();
          c.child_values = t.outputs.data() + t.list_off[c0];
          const double s = now_s();
          CK(cudasp_tf_function_columns(bd, gs, ls[i], &c));
          t_calls[i] += now_s() - s;
        }
      } else if (a.vectors) {
        // DuckDB's side: the chunk's vectors as a flat DataChunk holds them
        // (txids and tweaks as string_t over the table's bytes, offsets of the
        // lists relative to the chunk's child vector)
        std::vector<cudasp_tf_string> txs(CUDASP_TF_VECTOR_SIZE), tws(CUDASP_TF_VECTOR_SIZE);
        std::vector<cudasp_tf_list_entry> le(CUDASP_TF_VECTOR_SIZE);
        for (;;) {
          const uint64_t c0 = next.fetch_add(CUDASP_TF_VECTOR_SIZE);
          if (c0 >= rows) break;
          const uint32_t cnt = (uint32_t)std::min<uint64_t>(CUDASP_TF_VECTOR_SIZE, rows - c0);
          for (uint32_t r = 0; r < cnt; r++) {
            const uint8_t* tx = t.txids.data() + (c0 + r) * 32;
            const uint8_t* tk = t.tweaks.data() + (c0 + r) * 64;
            txs[r].length = 32;
            memcpy(txs[r].prefix, tx, 4);
            txs[r].ptr = tx;
            tws[r].length = 64;
            memcpy(tws[r].prefix, tk, 4);
            tws[r].ptr = tk;
            le[r].offset = t.list_off[c0 + r] - t.list_off[c0];
            le[r].length = t.list_len[c0 + r];
          }
          cudasp_tf_vectors v{};
          v.count = cnt;
          v.txid.data = txs.data();
          v.height.data = t.heights.data() + c0;
          v.tweak.data = tws.data();
          v.outputs.data = le.data();
          v.child.data = t.outputs.data() + t.list_off[c0];
          const double s = now_s();
          CK(cudasp_tf_function_vectors(bd, gs, ls[i], &v));
          t_calls[i] += now_s() - s;
        }
      } else {
        std::vector<const uint8_t*> txp(CUDASP_TF_VECTOR_SIZE), twp(CUDASP_TF_VECTOR_SIZE);
        std::vector<uint32_t> txs(CUDASP_TF_VECTOR_SIZE, 32), tws(CUDASP_TF_VECTOR_SIZE, 64);
        std::vector<uint64_t> loff(CUDASP_TF_VECTOR_SIZE);
        for (;;) {
          const uint64_t c0 = next.fetch_add(CUDASP_TF_VECTOR_SIZE);
          if (c0 >= rows) break;
          const uint32_t cnt = (uint32_t)std::min<uint64_t>(CUDASP_TF_VECTOR_SIZE, rows - c0);
          for (uint32_t r = 0; r < cnt; r++) {
            txp[r] = t.txids.data() + (c0 + r) * 32;
            twp[r] = t.tweaks.data() + (c0 + r) * 64;
            loff[r] = t.list_off[c0 + r] - t.list_off[c0];
          }
          cudasp_tf_chunk c{};
          c.count = cnt;
          c.txid_data = txp.data();
          c.txid_size = txs.data();
          c.height = t.heights.data() + c0;
          c.tweak_data = twp.data();
          c.tweak_size = tws.data();
          c.list_offset = loff.data();
          c.list_length = t.list_len.data() + c0;
          c.child_values = t.outputs.data() + t.list_off[c0];
          const double s = now_s();
          CK(cudasp_tf_function(bd, gs, ls[i], &c));
          t_calls[i] += now_s() - s;
        }
      }
      finish(i);
    });
  }
  for (auto& x : th) x.join();
  QueryResult q;
  q.secs = now_s();
  CK(cudasp_tf_get_stats(gs, &q.stats));
  q.logical_gpus = cudasp_tf_num_gpus(gs);
  for (auto* l : ls) cudasp_tf_local_free(l);
  cudasp_tf_global_free(gs);
  cudasp_tf_bind_free(bd);
  q.emitted = got.size();
  std::sort(got.begin(), got.end());
  q.exact = a.null_device ? got.empty() : got == t.planted;
  if (!q.exact || torn) {  // which rows differ (stderr; the JSON keeps the verdict)
    std::vector<uint64_t> extra, missing;
    std::set_difference(got.begin(), got.end(), t.planted.begin(), t.planted.end(), std::back_inserter(extra));
    std::set_difference(t.planted.begin(), t.planted.end(), got.begin(), got.end(), std::back_inserter(missing));
    fprintf(stderr, "query not exact: %zu emitted, %zu planted, %zu extra, %zu missing, %zu torn rows (txid and "
            "tweak/height of different rows)\n", got.size(), t.planted.size(), extra.size(), missing.size(),
            (size_t)torn);
    for (size_t k = 0; k < extra.size() && k < 8; k++) fprintf(stderr, "  extra g=%llu\n", (unsigned long long)extra[k]);
    for (size_t k = 0; k < missing.size() && k < 8; k++)
      fprintf(stderr, "  missing g=%llu\n", (unsigned long long)missing[k]);
  }
  q.exact = q.exact && torn == 0;
  q.got.swap(got);
  auto mean = [](const std::vector<double>& v) {
    double s = 0;
    for (double x : v) s += x;
    return s / v.size();
  };
  q.call_s_mean = mean(t_calls);
  q.final_s_mean = mean(t_final);
  q.done_min = *std::min_element(t_done.begin(), t_done.end());
  q.done_max = *std::max_element(t_done.begin(), t_done.end());
  return q;
}

// --pinned: the C pinned table over the same rows (see the header).
static int run_pinned(const Args& a, const uint8_t scan[32], const uint8_t spend[64],
                      const std::vector<uint8_t>& labels, const Table& t, double gen_s) {
  const int L = a.labels;
  const uint64_t rows = t.rows;
  const auto t0 = std::chrono::steady_clock::now();
  auto since = [](std::chrono::steady_clock::time_point x) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - x).count();
  };
  cudasp_pinned_table* pt;
  CK(cudasp_pinned_create_placed((uint64_t)a.batch, a.pinned.data(), (uint32_t)a.pinned.size(),
                                 a.hbm ? CUDASP_TABLE_HBM : CUDASP_TABLE_PINNED, &pt));
  const uint64_t piece = 65536;
  std::vector<int32_t> txo(piece + 1), lo(piece + 1);
  for (uint64_t c0 = 0; c0 < rows; c0 += piece) {
    const uint64_t m = std::min<uint64_t>(piece, rows - c0);
    for (uint64_t r = 0; r <= m; r++) {
      txo[r] = (int32_t)(r * 32);
      lo[r] = (int32_t)((c0 + r < rows ? t.list_off[c0 + r] : t.outputs.size()) - t.list_off[c0]);
    }
    cudasp_tf_columns c{};
    c.count = m;
    c.txid_offsets = txo.data();
    c.txid_data = t.txids.data() + c0 * 32;
    c.height = t.heights.data() + c0;
    c.tweak_data = t.tweaks.data() + c0 * 64;
    c.tweak_fixed_width = 64;
    c.list_offsets = lo.data();
    c.child_values = t.outputs.data() + t.list_off[c0];
    CK(cudasp_pinned_append(pt, &c));
  }
  const double pin_s = since(t0);
  cudasp_pinned_info_t inf{};
  CK(cudasp_pinned_info(pt, &inf));
  std::vector<double> secs;
  bool exact = true;
  uint64_t matches = 0;
  for (int r = 0; !a.null_device && r <= a.reps; r++) {
    const auto s0 = std::chrono::steady_clock::now();
    cudasp_tf_blob_arg a_scan{scan, 32, 1}, a_spend{spend, 64, 1};
    std::vector<cudasp_tf_blob_arg> a_lab(std::max(1, L));
    for (int j = 0; j < L; j++) a_lab[j] = {labels.data() + 64 * j, 64, 1};
    cudasp_tf_bind_data* bd;
    char err[512];
    if (cudasp_tf_bind(4, a_scan, a_spend, 1, a_lab.data(), (uint32_t)L, 1, 1, a.batch, &bd, err, sizeof(err)) != 0 ||
        ((a.output_count != 1 || a.label_negation) &&
         cudasp_tf_bind_options(bd, 1, a.output_count, 1, a.label_negation ? 1 : 0, 0, 0, err, sizeof(err)) != 0)) {
      fprintf(stderr, "bind: %s\n", err);
      return 1;
    }
    uint64_t* got = nullptr;
    uint64_t n = 0;
    CK(cudasp_pinned_scan(pt, bd, &got, &n));
    cudasp_tf_bind_free(bd);
    const double sec = since(s0);
    const bool ok = n == t.planted.size() && std::equal(got, got + n, t.planted.begin());
    if (!ok) fprintf(stderr, "pinned scan %d not exact: %llu rows, %zu planted\n", r, (unsigned long long)n,
                     t.planted.size());
    cudasp_pinned_free_rows(got);
    if (r > 0) {  // scan 0 warms the scanners and streams
      secs.push_back(sec);
      exact = exact && ok;
      matches = n;
    }
  }
  CK(cudasp_pinned_info(pt, &inf));
  cudasp_pinned_free(pt);
  std::vector<double> sorted = secs;
  std::sort(sorted.begin(), sorted.end());
  const double med = sorted.empty() ? 0.0 : sorted[sorted.size() / 2];
  std::string all = "[", devs = "[";
  for (size_t i = 0; i < secs.size(); i++) all += (i ? ", " : "") + std::to_string(secs[i]);
  for (size_t i = 0; i < a.pinned.size(); i++) devs += (i ? ", " : "") + std::to_string(a.pinned[i]);
  all += "]";
  devs += "]";
  printf("{\"what\": \"C pinned table (cudasp_pinned_*): appended once, scanned in place per query\", \"placement\": \"%s\", "
         "\"rows\": %llu, \"batch_size\": %lld, \"labels\": %d, \"outputs_total\": %llu, \"devices\": %s, "
         "\"batches\": %llu, \"rows_pinned\": %llu, \"pinned_bytes\": %llu, \"pin_s\": %.3f, "
         "\"generate_seconds\": %.2f, \"reps\": %d, \"seconds\": %.5f, \"seconds_all\": %s, \"tx_per_s\": %.1f, "
         "\"matches\": %llu, \"planted\": %zu, \"emitted_equal_planted\": %s, \"last_publish_s\": %.5f, "
         "\"device_bytes\": %llu, \"null_device\": %s}\n",
         a.hbm ? "hbm" : "pinned", (unsigned long long)rows, (long long)a.batch, L,
         (unsigned long long)t.outputs.size(), devs.c_str(),
         (unsigned long long)inf.batches, (unsigned long long)inf.rows_pinned, (unsigned long long)inf.pinned_bytes,
         pin_s, gen_s, (int)secs.size(), med, all.c_str(), med > 0 ? rows / med : 0.0, (unsigned long long)matches,
         t.planted.size(), exact ? "true" : "false", inf.last_publish_s, (unsigned long long)inf.device_bytes,
         a.null_device ? "true" : "false");
  return exact ? 0 : 1;
}

static std::string hex(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s(2 * n, '0');
  for (size_t i = 0; i < n; i++) {
    s[2 * i] = d[p[i] >> 4];
    s[2 * i + 1] = d[p[i] & 15];
  }
  return s;
}

// 256 planted and 256 unplanted rows, strided over the table, as JSON (see
// the header): what the oracle recomputes to tie the e2e leg to it.
static bool write_plant_sample(const std::string& path, const Table& t, const uint8_t scan[32],
                               const uint8_t spend[64], const std::vector<uint8_t>& labels, int L,
                               const std::vector<uint64_t>& got) {
  FILE* f = fopen(path.c_str(), "w");
  if (!f) return false;
  uint8_t s0[32];
  hex2bin(S0_LE_HEX, s0);
  fprintf(f, "{\"scan\": \"%s\", \"spend\": \"%s\", \"s0_le\": \"%s\", \"labels\": [", hex(scan, 32).c_str(),
          hex(spend, 64).c_str(), hex(s0, 32).c_str());
  for (int j = 0; j < L; j++) fprintf(f, "%s\"%s\"", j ? ", " : "", hex(labels.data() + 64 * j, 64).c_str());
  fprintf(f, "], \"rows_total\": %llu, \"planted_total\": %zu, \"rows\": [", (unsigned long long)t.rows,
          t.planted.size());
  std::vector<std::pair<uint64_t, int>> pick;  // (row, column or -1)
  const size_t np = t.planted.size(), want = 256;
  for (size_t i = 0; i < std::min(want, np); i++) {
    const size_t k = i * np / std::min(want, np);
    pick.emplace_back(t.planted[k], t.planted_col[k]);
  }
  const uint64_t unplanted = t.rows / PLANT_EVERY;  // rows g = 500 mod 1000 (never planted)
  for (uint64_t i = 0; i < std::min<uint64_t>(want, unplanted); i++) {
    const uint64_t g = (i * unplanted / std::min<uint64_t>(want, unplanted)) * PLANT_EVERY + PLANT_EVERY / 2;
    if (g < t.rows) pick.emplace_back(g, -1);
  }
  for (size_t i = 0; i < pick.size(); i++) {
    const uint64_t g = pick[i].first;
    fprintf(f, "%s{\"g\": %llu, \"tweak\": \"%s\", \"column\": %d, \"emitted\": %d, \"outputs\": [", i ? ", " : "",
            (unsigned long long)g, hex(t.tweaks.data() + g * 64, 64).c_str(), pick[i].second,
            std::binary_search(got.begin(), got.end(), g) ? 1 : 0);
    for (uint64_t k = 0; k < t.list_len[g]; k++)
      fprintf(f, "%s%lld", k ? ", " : "", (long long)t.outputs[t.list_off[g] + k]);
    fprintf(f, "]}");
  }
  fprintf(f, "]}\n");
  return fclose(f) == 0;
}

int main(int argc, char** argv) {
  const Args a = parse(argc, argv);
  if (a.null_device) setenv("CUDASP_TF_NULL_DEVICE", "1", 1);
  uint8_t scan[32], spend[64];
  hex2bin(SCAN_HEX, scan);
  hex2bin(SPEND_HEX, spend);
  std::vector<uint8_t> labels;
  if (!a.labels_file.empty()) {
    FILE* fp = fopen(a.labels_file.c_str(), "rb");
    if (!fp) {
      fprintf(stderr, "cannot open %s\n", a.labels_file.c_str());
      return 1;
    }
    labels.resize((size_t)64 * a.labels);
    const size_t got = fread(labels.data(), 1, labels.size(), fp);
    fclose(fp);
    if (got != labels.size()) {
      fprintf(stderr, "%s: %zu bytes, %zu expected for %d labels\n", a.labels_file.c_str(), got, labels.size(),
              a.labels);
      return 1;
    }
  } else if (a.labels == 1) {
    labels.resize(64);
    hex2bin(LABEL_HEX, labels.data());
  } else if (a.labels > 1) {
    fprintf(stderr, "--labels %d needs --labels-file (bench.label_keys)\n", a.labels);
    return 1;
  }

  auto since = [](std::chrono::steady_clock::time_point x) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - x).count();
  };
  const auto g0 = std::chrono::steady_clock::now();
  Table t;
  double hip_init_s = 0, scanner_create_s = 0, prewarm_s = 0;
  if (!a.table_in.empty()) {
    if (!read_table(a.table_in, t) || t.rows != a.rows) {
      fprintf(stderr, "cannot read a %llu-row table from %s\n", (unsigned long long)a.rows, a.table_in.c_str());
      return 1;
    }
  } else {
    generate(a, scan, spend, labels, t);
  }
  const double gen_s = since(g0);
  if (!a.table_out.empty()) {
    if (!write_table(a.table_out, t)) {
      fprintf(stderr, "cannot write %s\n", a.table_out.c_str());
      return 1;
    }
    printf("{\"table_out\": \"%s\", \"rows\": %llu, \"generate_seconds\": %.2f}\n", a.table_out.c_str(),
           (unsigned long long)t.rows, gen_s);
    return 0;
  }
  if (!a.table_in.empty()) {
    const auto h0 = std::chrono::steady_clock::now();
    const int ndev = cudasp_device_count();  // the HIP runtime's initialisation, nothing of the library's
    hip_init_s = since(h0);
    if (ndev <= 0) {
      fprintf(stderr, "no GPU\n");
      return 1;
    }
    if (a.cold_phases) {
      const auto c0 = std::chrono::steady_clock::now();
      cudasp_scanner* sc;
      CK(cudasp_scanner_create(0, scan, spend, a.labels ? labels.data() : nullptr, (uint32_t)a.labels, 1, &sc));
      CK(cudasp_scanner_sync(sc));
      scanner_create_s = since(c0);
      cudasp_scanner_destroy(sc);
    }
  }
  if (a.prewarm) CK(cudasp_tf_prewarm((uint64_t)a.batch, &prewarm_s));
  if (!a.pinned.empty()) return run_pinned(a, scan, spend, labels, t, gen_s);

  const QueryResult warm = run_query(a, scan, spend, labels, t);  // scanners, slots, tables
  std::vector<QueryResult> qs;
  for (int r = 0; r < a.reps; r++) qs.push_back(run_query(a, scan, spend, labels, t));
  std::vector<double> warm_secs;
  bool warm_exact = true;
  for (int r = 0; r < a.warm_reps; r++) {
    const QueryResult w = run_query(a, scan, spend, labels, t, a.warm_ms);
    warm_secs.push_back(w.secs);
    warm_exact = warm_exact && w.exact;
  }
  std::sort(warm_secs.begin(), warm_secs.end());
  const double warm_med = warm_secs.empty() ? 0.0 : warm_secs[warm_secs.size() / 2];
  std::vector<double> secs;
  bool all_exact = warm.exact && warm_exact;
  for (const auto& q : qs) {
    secs.push_back(q.secs);
    all_exact = all_exact && q.exact;
  }
  std::vector<double> sorted = secs;
  std::sort(sorted.begin(), sorted.end());
  const double med = sorted[sorted.size() / 2];
  const QueryResult& q = qs[std::find(secs.begin(), secs.end(), med) - secs.begin()];
  std::string all = "[";
  for (size_t i = 0; i < secs.size(); i++) all += (i ? ", " : "") + std::to_string(secs[i]);
  all += "]";
  int planted_labels = 0;
  for (int j = 0; j < 32; j++) planted_labels += (t.labels_planted_mask >> j) & 1;
  const char* hq = getenv("GPU_MAX_HW_QUEUES");
  if (!a.plant_sample.empty() &&
      !write_plant_sample(a.plant_sample, t, scan, spend, labels, a.labels, qs.back().got)) {
    fprintf(stderr, "cannot write %s\n", a.plant_sample.c_str());
    return 1;
  }
  printf("{\"what\": \"table-function host end-to-end (host memory -> matches, PCIe-inclusive)\", \"input\": \"%s\", "
         "\"rows\": %llu, \"threads\": %d, \"batch_size\": %lld, \"labels\": %d, \"outputs_per_row\": %s, "
         "\"outputs_total\": %llu, \"reps\": %d, \"seconds\": %.5f, \"seconds_all\": %s, \"seconds_min\": %.5f, "
         "\"tx_per_s\": %.1f, \"matches\": %llu, \"planted\": %llu, \"label_indices_planted\": %d, "
         "\"emitted_equal_planted\": %s, \"warmup_seconds\": %.3f, \"generate_seconds\": %.2f, \"devices\": %d, "
         "\"feeds\": %u, \"streams_per_feed\": %u, \"max_streams_per_device\": %u, \"gpu_max_hw_queues\": %u, "
         "\"gpu_max_hw_queues_env\": \"%s\", \"launches\": %llu, \"rows_per_launch\": %.0f, "
         "\"harvest_wait_s\": %.4f, \"reserve_s\": %.4f, \"copy_s\": %.4f, \"launch_s\": %.4f, "
         "\"thread_call_s_mean\": %.4f, \"thread_final_s_mean\": %.4f, "
         "\"thread_done_s_min\": %.4f, \"thread_done_s_max\": %.4f, \"streaming_feeds\": %u, \"logical_gpus\": %d, "
         "\"warm_reps\": %d, \"warm_ms\": %d, \"warm_seconds\": %.5f, \"warm_tx_per_s\": %.1f, "
         "\"null_device\": %s, \"host_cpus_online\": %ld, \"host_call_tx_per_s\": %.1f, "
         "\"table_in\": %s, \"hip_init_s\": %.4f, \"first_query_s\": %.5f, \"scanner_create_s\": %.4f, "
         "\"first_query_exact\": %s, \"prewarm_s\": %.4f}\n",
         a.columnar ? "arrow columns" : (a.vectors ? "2048-row DuckDB vectors" : "2048-row chunks"), (unsigned long long)t.rows, a.threads, (long long)a.batch,
         a.labels,
         a.kmax ? ("\"1.." + std::to_string(a.kmax) + "\"").c_str() : std::to_string(a.k).c_str(),
         (unsigned long long)t.outputs.size(), a.reps, med, all.c_str(), sorted[0], t.rows / med,
         (unsigned long long)q.emitted, (unsigned long long)t.planted.size(), planted_labels,
         all_exact ? "true" : "false", warm.secs, gen_s, cudasp_device_count(), q.stats.feeds,
         q.stats.streams_per_feed, q.stats.max_streams_per_device, q.stats.hw_queues, hq ? hq : "",
         (unsigned long long)q.stats.launches, q.stats.launches ? (double)q.stats.rows / q.stats.launches : 0.0,
         q.stats.harvest_wait_s, q.stats.reserve_s, q.stats.copy_s, q.stats.launch_s, q.call_s_mean, q.final_s_mean, q.done_min, q.done_max,
         q.stats.streaming_feeds, q.logical_gpus, a.warm_reps, a.warm_ms, warm_med,
         warm_med > 0 ? t.rows / warm_med : 0.0, a.null_device ? "true" : "false", sysconf(_SC_NPROCESSORS_ONLN),
         q.call_s_mean > 0 ? t.rows / q.call_s_mean : 0.0, a.table_in.empty() ? "false" : "true", hip_init_s,
         warm.secs, scanner_create_s, warm.exact ? "true" : "false", prewarm_s);
  return all_exact ? 0 : 2;
}
