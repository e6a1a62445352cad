// Instruction-count probes: one field/group operation per kernel, on data
// loaded from and stored to global memory, so the ISA listing of each kernel
// is (almost only) that operation.  Built by tools/isa/isa_count.py.
#include "../../duckdb-cudasp-extension_amd/csrc/secp256k1_group.hpp"
using namespace cudasp;

__device__ __forceinline__ void ld(fe& a, const uint32_t* p) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) a.n[i] = p[i * 65536 + threadIdx.x];
}
__device__ __forceinline__ void st(uint32_t* p, const fe& a) {
#pragma unroll
  for (int i = 0; i < FE_LIMBS; i++) p[i * 65536 + threadIdx.x] = a.n[i];
}
extern "C" __global__ __launch_bounds__(256, 2) void probe_mul(const uint32_t* in, uint32_t* out) {
  fe a, b, r; ld(a, in); ld(b, in + 655360); fe_mul(r, a, b); st(out, r);
}
extern "C" __global__ __launch_bounds__(256, 2) void probe_sqr(const uint32_t* in, uint32_t* out) {
  fe a, r; ld(a, in); fe_sqr(r, a); st(out, r);
}
extern "C" __global__ __launch_bounds__(256, 2) void probe_dbl(const uint32_t* in, uint32_t* out) {
  gej p, r; ld(p.x, in); ld(p.y, in + 655360); ld(p.z, in + 2 * 655360);
  gej_double(r, p); st(out, r.x); st(out + 655360, r.y); st(out + 2 * 655360, r.z);
}
extern "C" __global__ __launch_bounds__(256, 2) void probe_madd(const uint32_t* in, uint32_t* out) {
  gej p, r; ge q; ld(p.x, in); ld(p.y, in + 655360); ld(p.z, in + 2 * 655360);
  ld(q.x, in + 3 * 655360); ld(q.y, in + 4 * 655360);
  gej_add_ge(r, p, q, nullptr); st(out, r.x); st(out + 655360, r.y); st(out + 2 * 655360, r.z);
}
extern "C" __global__ __launch_bounds__(256, 2) void probe_inv(const uint32_t* in, uint32_t* out) {
  fe a, r; ld(a, in); fe_inv(r, a); st(out, r);
}
extern "C" __global__ __launch_bounds__(256, 2) void probe_loadstore(const uint32_t* in, uint32_t* out) {
  fe a; ld(a, in); st(out, a);
}
extern "C" __global__ __launch_bounds__(256, 2) void probe_ydbl(const uint32_t* in, uint32_t* out) {
  gej p, r; ld(p.x, in); ld(p.y, in + 655360); ld(p.z, in + 2 * 655360);
  gej_double_neg_yh(r, p); st(out, r.x); st(out + 655360, r.y); st(out + 2 * 655360, r.z);
}
extern "C" __global__ __launch_bounds__(256, 2) void probe_yadd(const uint32_t* in, uint32_t* out) {
  gej p, r; ge q; ld(p.x, in); ld(p.y, in + 655360); ld(p.z, in + 2 * 655360);
  ld(q.x, in + 3 * 655360); ld(q.y, in + 4 * 655360);
  gej_add_ge_yh(r, p, q); st(out, r.x); st(out + 655360, r.y); st(out + 2 * 655360, r.z);
}
