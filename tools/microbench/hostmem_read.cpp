// CPU read/write speed of the pinned host buffers the streaming feeds use
// (cudasp_host_alloc: hipHostMallocCoherent | Mapped | Portable) against
// hipHostMallocDefault and malloc: is coherent pinned memory cached for the
// CPU?  Prints one JSON line.  Measurement tool only.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/cudasp_abi.h"

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

static void run(const char* name, uint8_t* p, size_t n, bool last) {
  for (size_t i = 0; i < n; i++) p[i] = (uint8_t)(i * 7);
  volatile uint64_t sink = 0;
  double t = now();
  uint64_t s = 0;
  for (size_t i = 0; i < n; i += 8) {
    uint64_t v;
    memcpy(&v, p + i, 8);
    s += v;
  }
  const double seq = now() - t;
  t = now();
  uint32_t x = 12345;
  for (int k = 0; k < 100000; k++) {
    x = x * 1664525u + 1013904223u;
    s += p[x % n];
  }
  const double rnd = now() - t;
  std::vector<uint32_t> idx(4096);
  for (size_t i = 0; i < idx.size(); i++) idx[i] = (uint32_t)((i * 2654435761u) % 100000);
  uint32_t* q = reinterpret_cast<uint32_t*>(p);
  memcpy(q, idx.data(), idx.size() * 4);
  t = now();
  std::sort(q, q + idx.size());
  const double srt = now() - t;
  t = now();
  std::vector<uint8_t> dst(n);
  memcpy(dst.data(), p, n);
  const double cpy_out = now() - t;
  t = now();
  memcpy(p, dst.data(), n);
  const double cpy_in = now() - t;
  sink = s;
  (void)sink;
  printf("\"%s\": {\"seq_read_GBps\": %.2f, \"random_byte_read_ns\": %.1f, \"sort_4096_u32_us\": %.1f, "
         "\"memcpy_out_GBps\": %.2f, \"memcpy_in_GBps\": %.2f}%s",
         name, n / seq / 1e9, rnd / 100000 * 1e9, srt * 1e6, n / cpy_out / 1e9, n / cpy_in / 1e9, last ? "" : ", ");
}

int main() {
  const size_t n = 64 << 20;
  void* a = nullptr;
  if (cudasp_host_alloc(&a, n) != 0) return 1;
  void* b = nullptr;
  if (hipHostMalloc(&b, n, hipHostMallocDefault) != hipSuccess) return 1;
  void* c = nullptr;
  if (hipHostMalloc(&c, n, hipHostMallocNonCoherent) != hipSuccess) return 1;
  uint8_t* m = (uint8_t*)malloc(n);
  printf("{");
  run("cudasp_host_alloc_coherent", (uint8_t*)a, n, false);
  run("hipHostMallocDefault", (uint8_t*)b, n, false);
  run("hipHostMallocNonCoherent", (uint8_t*)c, n, false);
  run("malloc", m, n, true);
  printf("}\n");
  return 0;
}
