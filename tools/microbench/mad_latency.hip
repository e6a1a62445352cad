// Dependent-chain throughput of v_mad_u64_u32 on gfx950: CH independent chains
// per lane, W waves per SIMD (blocks of 256 threads = 4 waves, one per SIMD).
// cycles/instr/wave = elapsed SIMD cycles / instructions issued per wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s\n", hipGetErrorString(e_)); exit(1);} } while (0)

#define R2(x) x x
#define R8(x) R2(R2(R2(x)))

template <int CH>
__global__ __launch_bounds__(256) void chain(uint64_t* out, int iters, uint32_t seed) {
  uint32_t a = seed * threadIdx.x + 1, b = a ^ 0x9e3779b9u;
  uint64_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; c++) acc[c] = c + a;
  for (int it = 0; it < iters; ++it) {
    // one asm block per 8 mads per chain (the hazard recognizer pads between
    // asm statements, not inside them)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      if constexpr (CH == 1) {
        asm volatile(R8("v_mad_u64_u32 %0, vcc, %1, %2, %0\n") : "+v"(acc[0]) : "v"(a), "v"(b) : "vcc");
      } else if constexpr (CH == 2) {
        asm volatile(R8("v_mad_u64_u32 %0, vcc, %2, %3, %0\nv_mad_u64_u32 %1, vcc, %2, %3, %1\n")
                     : "+v"(acc[0]), "+v"(acc[1]) : "v"(a), "v"(b) : "vcc");
      } else {
        asm volatile(R8("v_mad_u64_u32 %0, vcc, %4, %5, %0\nv_mad_u64_u32 %1, vcc, %4, %5, %1\n"
                        "v_mad_u64_u32 %2, vcc, %4, %5, %2\nv_mad_u64_u32 %3, vcc, %4, %5, %3\n")
                     : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]) : "v"(a), "v"(b) : "vcc");
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) s ^= acc[c];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int CH>
void run(int waves_per_simd, uint64_t* d, int cus) {
  int blocks = cus * waves_per_simd;  // 4 waves per block, one per SIMD
  int iters = 400;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(chain<CH>, dim3(blocks), dim3(256), 0, 0, d, 4, 1u);
  CHK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; rep++) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(chain<CH>, dim3(blocks), dim3(256), 0, 0, d, iters, 3u + rep);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms; CHK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double instr_per_wave = (double)iters * 32 * CH;
  double simd_cycles = best * 1e-3 * 2.4e9;
  // each SIMD runs waves_per_simd waves concurrently
  printf("chains/lane %d  waves/SIMD %d : %.2f cycles per wave-instr per wave, SIMD issue %.2f cycles/instr\n", CH,
         waves_per_simd, simd_cycles / instr_per_wave, simd_cycles / (instr_per_wave * waves_per_simd));
}

int main() {
  hipDeviceProp_t p; CHK(hipGetDeviceProperties(&p, 0));
  uint64_t* d; CHK(hipMalloc(&d, (size_t)p.multiProcessorCount * 16 * 256 * 8));
  int cus = p.multiProcessorCount;
  for (int w : {1, 2, 3, 4, 8}) { run<1>(w, d, cus); }
  for (int w : {1, 2, 4}) { run<2>(w, d, cus); }
  for (int w : {1, 2, 4}) { run<4>(w, d, cus); }
  CHK(hipFree(d));
  return 0;
}
