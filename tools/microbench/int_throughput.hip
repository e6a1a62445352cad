// Microbenchmark: per-instruction VALU throughput on gfx950 for the integer
// primitives a 256-bit field multiply can be built from. Each lane runs 8
// independent chains so the measurement is issue-throughput, not latency.
// Output: one line per op with lane-ops/s and lane-ops per CU per cycle at the
// measured clock (2.4 GHz nominal).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

template <int OP>
__global__ __launch_bounds__(256) void bench(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a[8], b[8];
  uint64_t acc[8];
  double f[8];
  uint32_t smask;
  asm volatile("s_mov_b32 %0, 0x1fffffff" : "=s"(smask));
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a[i] = seed * (threadIdx.x + 3 * i + 1) + blockIdx.x;
    b[i] = a[i] ^ 0x9e3779b9u;
    acc[i] = (uint64_t)a[i] * 7u + b[i];
    f[i] = (double)a[i] * 1e-9;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        if constexpr (OP == 0) {  // v_mad_u64_u32 with carry-out
          uint64_t c;
          asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[k]), "=s"(c) : "v"(a[k]), "v"(b[k]));
        } else if constexpr (OP == 1) {
          asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b[k]));
        } else if constexpr (OP == 2) {
          asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b[k]));
        } else if constexpr (OP == 3) {
          asm volatile("v_add_co_u32 %0, vcc, %0, %1\n\tv_addc_co_u32 %1, vcc, %1, %0, vcc"
                       : "+v"(a[k]), "+v"(b[k]) : : "vcc");
        } else if constexpr (OP == 4) {
          asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b[k]));
        } else if constexpr (OP == 5) {
          asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(f[k]) : "v"(f[(k + 1) & 7]));
        } else if constexpr (OP == 6) {
          asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(a[k]) : "v"(b[k]), "v"(b[(k+1)&7]));
        } else if constexpr (OP == 7) {
          asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a[k]) : "v"(b[k]));
        } else if constexpr (OP == 8) {  // 3-input add
          asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(b[k]), "v"(b[(k+1)&7]));
        } else if constexpr (OP == 9) {  // carry-in add into 3rd word from sgpr mask
          uint64_t c = 0;
          asm volatile("v_addc_co_u32_e64 %0, %1, %0, 0, %1" : "+v"(a[k]), "+s"(c));
        } else if constexpr (OP == 10) {  // v_lshl_add / alignbit
          asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[k]) : "v"(b[k]));
        } else if constexpr (OP == 11) {  // 64-bit add via v_lshl_add_u64 (gfx940+)
          asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(acc[k]) : "v"(acc[(k+1)&7]));
        } else if constexpr (OP == 12) {  // VOP2 with a 32-bit literal (8 bytes)
          asm volatile("v_and_b32_e32 %0, 0x1fffffff, %0" : "+v"(a[k]));
        } else if constexpr (OP == 13) {  // the same with the mask in an SGPR (4 bytes)
          asm volatile("v_and_b32_e32 %0, %1, %0" : "+v"(a[k]) : "s"(smask));
        } else if constexpr (OP == 14) {  // the same op in the VOP3 encoding (8 bytes)
          asm volatile("v_and_b32_e64 %0, %1, %0" : "+v"(a[k]) : "v"(b[k]));
        } else if constexpr (OP == 15) {  // VOP2 subtract from a literal (fe_negate's form)
          asm volatile("v_sub_u32_e32 %0, 0x3ffffffe, %0" : "+v"(a[k]));
        } else if constexpr (OP == 16) {  // the same from an SGPR
          asm volatile("v_sub_u32_e32 %0, %1, %0" : "+v"(a[k]) : "s"(smask));
        } else if constexpr (OP == 17) {  // 64-bit shift (the reductions' carry)
          asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(acc[k]));
        } else if constexpr (OP == 18) {  // one mad + one literal and (a reduction's pair)
          asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_and_b32_e32 %1, 0x1fffffff, %1"
                       : "+v"(acc[k]), "+v"(a[k]) : "v"(b[k]), "v"(b[(k + 1) & 7]) : "vcc");
        } else if constexpr (OP == 19) {  // one mad + one SGPR-mask and
          asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_and_b32_e32 %1, %4, %1"
                       : "+v"(acc[k]), "+v"(a[k]) : "v"(b[k]), "v"(b[(k + 1) & 7]), "s"(smask) : "vcc");
        } else if constexpr (OP == 20) {  // four mads + one literal and (~the ladder's ratio)
          asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_mad_u64_u32 %0, vcc, %3, %2, %0\n\t"
                       "v_mad_u64_u32 %0, vcc, %2, %2, %0\n\tv_mad_u64_u32 %0, vcc, %3, %3, %0\n\t"
                       "v_and_b32_e32 %1, 0x1fffffff, %1"
                       : "+v"(acc[k]), "+v"(a[k]) : "v"(b[k]), "v"(b[(k + 1) & 7]) : "vcc");
        } else if constexpr (OP == 21) {  // four mads + one SGPR-mask and
          asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_mad_u64_u32 %0, vcc, %3, %2, %0\n\t"
                       "v_mad_u64_u32 %0, vcc, %2, %2, %0\n\tv_mad_u64_u32 %0, vcc, %3, %3, %0\n\t"
                       "v_and_b32_e32 %1, %4, %1"
                       : "+v"(acc[k]), "+v"(a[k]) : "v"(b[k]), "v"(b[(k + 1) & 7]), "s"(smask) : "vcc");
        } else if constexpr (OP == 22) {  // four mads alone (the base of 20/21)
          asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0\n\tv_mad_u64_u32 %0, vcc, %2, %1, %0\n\t"
                       "v_mad_u64_u32 %0, vcc, %1, %1, %0\n\tv_mad_u64_u32 %0, vcc, %2, %2, %0"
                       : "+v"(acc[k]) : "v"(b[k]), "v"(b[(k + 1) & 7]) : "vcc");
        } else if constexpr (OP == 23) {  // mad with an SGPR multiplier (the reductions' fold terms)
          asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[k]) : "v"(b[k]), "s"(smask) : "vcc");
        } else if constexpr (OP == 24) {  // mad with an inline-constant multiplier
          asm volatile("v_mad_u64_u32 %0, vcc, %1, 8, %0" : "+v"(acc[k]) : "v"(b[k]) : "vcc");
        } else if constexpr (OP == 25) {  // VOP2 add of two VGPRs in the VOP3 encoding
          asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a[k]) : "v"(b[k]));
        } else if constexpr (OP == 26) {  // VOP2 shift by an inline constant
          asm volatile("v_lshlrev_b32_e32 %0, 1, %0" : "+v"(a[k]));
        } else if constexpr (OP == 27) {  // doubling as an add of the same VGPR twice
          asm volatile("v_add_u32_e32 %0, %0, %0" : "+v"(a[k]));
        } else if constexpr (OP == 28) {  // VOP2 and with an inline constant
          asm volatile("v_and_b32_e32 %0, 1, %0" : "+v"(a[k]));
        } else if constexpr (OP == 29) {  // VOP2 shift right by an inline constant
          asm volatile("v_lshrrev_b32_e32 %0, 29, %0" : "+v"(a[k]));
        } else if constexpr (OP == 30) {  // VOP2 add of a literal
          asm volatile("v_add_u32_e32 %0, 0x3ffffffe, %0" : "+v"(a[k]));
        } else if constexpr (OP == 31) {  // VOP2 shift by a VGPR amount
          asm volatile("v_lshlrev_b32_e32 %0, %1, %0" : "+v"(a[k]) : "v"(b[k]));
        } else if constexpr (OP == 32) {  // VOP1 move of a VGPR
          asm volatile("v_mov_b32_e32 %0, %1" : "=v"(a[k]) : "v"(b[(k + 1) & 7]));
        } else if constexpr (OP == 33) {  // VOP2 and of two VGPRs
          asm volatile("v_and_b32_e32 %0, %0, %1" : "+v"(a[k]) : "v"(b[k]));
        } else if constexpr (OP == 34) {  // VOP2 sub of two VGPRs
          asm volatile("v_sub_u32_e32 %0, %1, %0" : "+v"(a[k]) : "v"(b[k]));
        } else if constexpr (OP == 35) {  // 4 mads + 1 shift by inline constant (the sqr prologue's form)
          asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_mad_u64_u32 %0, vcc, %3, %2, %0\n\t"
                       "v_mad_u64_u32 %0, vcc, %2, %2, %0\n\tv_mad_u64_u32 %0, vcc, %3, %3, %0\n\t"
                       "v_lshlrev_b32_e32 %1, 1, %1"
                       : "+v"(acc[k]), "+v"(a[k]) : "v"(b[k]), "v"(b[(k + 1) & 7]) : "vcc");
        } else if constexpr (OP == 36) {  // 4 mads + 1 doubling add
          asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_mad_u64_u32 %0, vcc, %3, %2, %0\n\t"
                       "v_mad_u64_u32 %0, vcc, %2, %2, %0\n\tv_mad_u64_u32 %0, vcc, %3, %3, %0\n\t"
                       "v_add_u32_e32 %1, %1, %1"
                       : "+v"(acc[k]), "+v"(a[k]) : "v"(b[k]), "v"(b[(k + 1) & 7]) : "vcc");
        }
      }
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= a[i] ^ b[i] ^ (uint32_t)acc[i] ^ (uint32_t)(acc[i] >> 32) ^ (uint32_t)(uint64_t)f[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
static void run(const char* name, int instrs_per_op, int blocks, uint32_t* d) {
  int iters = 2000;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, d, 10, 1u);
  CHK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; rep++) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(bench<OP>, dim3(blocks), dim3(256), 0, 0, d, iters, 1u + rep);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double lane_ops = (double)blocks * 256 * iters * 16 * 8 * instrs_per_op;
  double rate = lane_ops / (best * 1e-3);
  // lanes-per-CU-per-cycle at 2.4 GHz (full-rate VALU = 128)
  double per_cu_cyc = rate / (256.0 * 2.4e9);
  printf("%-28s %8.3f ms  %10.3f Tlane-op/s  %7.2f lane-op/CU/cyc@2.4GHz\n", name, best, rate * 1e-12, per_cu_cyc);
  CHK(hipEventDestroy(e0));
  CHK(hipEventDestroy(e1));
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  printf("device %s  CUs %d  clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  int blocks = p.multiProcessorCount * 8;
  uint32_t* d;
  CHK(hipMalloc(&d, (size_t)blocks * 256 * 4));
  run<4>("v_add_u32", 1, blocks, d);
  run<8>("v_add3_u32", 1, blocks, d);
  run<10>("v_alignbit_b32", 1, blocks, d);
  run<3>("v_add_co+v_addc_co (2 ins)", 2, blocks, d);
  run<9>("v_addc_co_u32_e64 sgpr cin", 1, blocks, d);
  run<11>("v_lshl_add_u64", 1, blocks, d);
  run<0>("v_mad_u64_u32", 1, blocks, d);
  run<1>("v_mul_lo_u32", 1, blocks, d);
  run<2>("v_mul_hi_u32", 1, blocks, d);
  run<6>("v_mad_u32_u24", 1, blocks, d);
  run<7>("v_mul_hi_u32_u24", 1, blocks, d);
  run<5>("v_fma_f64", 1, blocks, d);
  // encodings: a VOP2 op with a literal, with an SGPR, in VOP3 form; mixes
  run<12>("v_and_b32 literal (8 B)", 1, blocks, d);
  run<13>("v_and_b32 sgpr (4 B)", 1, blocks, d);
  run<14>("v_and_b32_e64 (8 B)", 1, blocks, d);
  run<15>("v_sub_u32 literal (8 B)", 1, blocks, d);
  run<16>("v_sub_u32 sgpr (4 B)", 1, blocks, d);
  run<17>("v_lshrrev_b64", 1, blocks, d);
  run<18>("mad + and literal (2 ins)", 2, blocks, d);
  run<19>("mad + and sgpr (2 ins)", 2, blocks, d);
  run<20>("4 mad + and literal (5 ins)", 5, blocks, d);
  run<21>("4 mad + and sgpr (5 ins)", 5, blocks, d);
  run<22>("4 mad (4 ins)", 4, blocks, d);
  run<23>("v_mad_u64_u32 sgpr operand", 1, blocks, d);
  run<24>("v_mad_u64_u32 inline const", 1, blocks, d);
  run<25>("v_add_u32_e64 (8 B)", 1, blocks, d);
  run<26>("v_lshlrev_b32 inline (4 B)", 1, blocks, d);
  run<27>("v_add_u32 x, x (doubling)", 1, blocks, d);
  run<28>("v_and_b32 inline const", 1, blocks, d);
  run<29>("v_lshrrev_b32 inline", 1, blocks, d);
  run<30>("v_add_u32 literal", 1, blocks, d);
  run<31>("v_lshlrev_b32 vgpr amount", 1, blocks, d);
  run<32>("v_mov_b32 vgpr", 1, blocks, d);
  run<33>("v_and_b32 vgpr, vgpr", 1, blocks, d);
  run<34>("v_sub_u32 vgpr, vgpr", 1, blocks, d);
  run<35>("4 mad + lshl inline (5 ins)", 5, blocks, d);
  run<36>("4 mad + add x,x (5 ins)", 5, blocks, d);
  CHK(hipFree(d));
  return 0;
}
