// Issue-rate probe for the kernels' group operations on gfx950: a loop of
// ITERS doublings (or mixed additions, multiplications, squarings) per lane,
// W waves per SIMD (blocks of 256 threads = one wave per SIMD), no memory
// traffic inside the loop.  Prints SIMD cycles per operation; with the static
// VALU count of one operation (tools/isa/isa_count.py, or --valu below) that
// gives cycles per VALU instruction, the figure the stage-A kernel is bound by.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -o group_ops group_ops.hip
//   ./group_ops
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include "../../duckdb-cudasp-extension_amd/csrc/secp256k1_group.hpp"
using namespace cudasp;
#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "HIP %s\n", hipGetErrorString(e_)); exit(1);} } while (0)

__device__ void seed_fe(fe& a, uint32_t s) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) {
    s = s * 1664525u + 1013904223u;
    a.n[i] = s & ((1u << FE_BITS) - 1);
  }
  a.n[FE_LIMBS - 1] &= 0xFFFFu;
}

// Doubling variants for cost attribution (not valid arithmetic for X > 0):
// X = 1 drops the 3/2 X^2 chain (L = X^2), X = 2 also drops the doubled
// operand of the squarings (plain products), X = 3 the final negation.
template <int X>
__device__ __forceinline__ void dbl_exp(gej& r, const gej& a) {
  fe S, L, T, U;
  fe_mul(r.z, a.z, a.y);
  fe_sqr(S, a.y);
  if constexpr (X >= 1) {
    fe_sqr(L, a.x);
  } else {
    fe_sqr(L, a.x);
    fe_mul_int(L, L, 3);
    fe_half(L, L);
    fe_normalize_weak(L);
  }
  fe_mul(T, S, a.x);
  fe_negate<1>(T, T);
  fe_add(U, T, T);
  fe_sqr_add(r.x, L, U);
  fe_add(U, r.x, T);
  fe_mulsqr(r.y, L, U, S);
  if constexpr (X < 3) fe_negate<1>(r.y, r.y);
}

template <int OP>
__global__ __launch_bounds__(256) void loop(uint32_t* out, int iters, uint32_t seed) {
  uint32_t s = seed * 2654435761u + blockIdx.x * 256 + threadIdx.x;
  gej R;
  ge Q;
  seed_fe(R.x, s);
  seed_fe(R.y, s + 1);
  seed_fe(R.z, s + 2);
  seed_fe(Q.x, s + 3);
  seed_fe(Q.y, s + 4);
  for (int it = 0; it < iters; ++it) {
    if constexpr (OP == 20) {
      gej_double_neg_yh(R, R);  // the stage-A ladder's doubling (Yh form)
    } else if constexpr (OP == 21) {
      gej_add_ge_yh(R, R, Q);  // the stage-A ladder's mixed addition (Yh form)
    } else if constexpr (OP == 0) {
      gej_double(R, R);
    } else if constexpr (OP == 1) {
      gej_add_ge(R, R, Q);
    } else if constexpr (OP >= 10) {
      dbl_exp<OP - 10>(R, R);
    } else if constexpr (OP == 2) {
      fe_mul(R.x, R.x, R.y);
      fe_mul(R.y, R.y, R.z);
    } else {
      fe_sqr(R.x, R.x);
      fe_sqr(R.y, R.y);
    }
  }
  uint32_t h = 0;
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) h ^= R.x.n[i] ^ R.y.n[i] ^ R.z.n[i];
  out[blockIdx.x * 256 + threadIdx.x] = h;
}

template <int OP>
void run(const char* name, int waves_per_simd, uint32_t* d, int cus, int per_iter) {
  int blocks = cus * waves_per_simd;
  int iters = (OP <= 1 || OP >= 10) ? 200 : 400;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(loop<OP>, dim3(blocks), dim3(256), 0, 0, d, 4, 1u);
  CHK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 3; rep++) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(loop<OP>, dim3(blocks), dim3(256), 0, 0, d, iters, 3u + rep);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double ops_per_wave = (double)iters * per_iter;
  double simd_cycles = best * 1e-3 * 2.4e9;
  printf("%-5s waves/SIMD %d : %8.1f SIMD cycles per op\n", name, waves_per_simd,
         simd_cycles / (ops_per_wave * waves_per_simd));
  CHK(hipEventDestroy(e0));
  CHK(hipEventDestroy(e1));
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  int cus = p.multiProcessorCount;
  uint32_t* d;
  CHK(hipMalloc(&d, (size_t)cus * 8 * 256 * 4));
  // ~2 s of load first: the engine clock ramps up over the first launches,
  // and the comparisons below assume a steady clock.
  for (int i = 0; i < 20; i++) hipLaunchKernelGGL(loop<0>, dim3(cus * 3), dim3(256), 0, 0, d, 20000, 7u);
  CHK(hipDeviceSynchronize());
  for (int w : {1, 2, 3, 4}) run<0>("dbl", w, d, cus, 1);
  for (int w : {1, 2, 3, 4}) run<1>("madd", w, d, cus, 1);
  for (int w : {3}) run<10>("dbl0", w, d, cus, 1);
  for (int w : {3}) run<11>("dbl1", w, d, cus, 1);
  for (int w : {3}) run<13>("dbl3", w, d, cus, 1);
  for (int w : {1, 2, 3, 4}) run<2>("mul", w, d, cus, 2);
  for (int w : {1, 2, 3, 4}) run<3>("sqr", w, d, cus, 2);
  for (int w : {3}) run<0>("dbl", w, d, cus, 1);
  for (int w : {3}) run<10>("dbl0", w, d, cus, 1);
  for (int w : {2, 3, 4}) run<20>("ydbl", w, d, cus, 1);
  for (int w : {2, 3, 4}) run<21>("yadd", w, d, cus, 1);
  CHK(hipFree(d));
  return 0;
}
