// SHA-256 compression for the BIP-352 shared-secret tagged hash.
//
// The reference hashes tag || tag || ser per thread, recomputing SHA256(tag)
// each time (src/cudasp_gpu.cu:288-314, gECC hash::tagged_hash).  Here the
// 64-byte block SHA256(tag) || SHA256(tag) is constant, so the host compresses
// it once (sha256_midstate) and each row runs exactly one compression over
//   ser (37 B) || 0x80 || zeros || bitlen(64 + 37 = 101 bytes = 808 bits).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace cudasp {

#define CUDASP_SHA_HD __host__ __device__ __forceinline__

CUDASP_SHA_HD uint32_t sha_rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

struct sha256_k {
  static constexpr uint32_t k[64] = {
      0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
      0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
      0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
      0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
      0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
      0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
      0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
      0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u};
};

// state <- compress(state, w[0..15]); w is consumed (used as the schedule ring).
CUDASP_SHA_HD void sha256_compress(uint32_t state[8], uint32_t w[16]) {
  uint32_t a = state[0], b = state[1], c = state[2], d = state[3];
  uint32_t e = state[4], f = state[5], g = state[6], h = state[7];
#pragma unroll
  for (int i = 0; i < 64; i++) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i + 1) & 15], w2 = w[(i + 14) & 15];
      uint32_t s0 = sha_rotr(w15, 7) ^ sha_rotr(w15, 18) ^ (w15 >> 3);
      uint32_t s1 = sha_rotr(w2, 17) ^ sha_rotr(w2, 19) ^ (w2 >> 10);
      wi = w[i & 15] + s0 + w[(i + 9) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = sha_rotr(e, 6) ^ sha_rotr(e, 11) ^ sha_rotr(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = h + S1 + ch + sha256_k::k[i] + wi;
    uint32_t S0 = sha_rotr(a, 2) ^ sha_rotr(a, 13) ^ sha_rotr(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    h = g; g = f; f = e; e = d + t1;
    d = c; c = b; b = a; a = t1 + t2;
  }
  state[0] += a; state[1] += b; state[2] += c; state[3] += d;
  state[4] += e; state[5] += f; state[6] += g; state[7] += h;
}

CUDASP_SHA_HD void sha256_init(uint32_t s[8]) {
  s[0] = 0x6a09e667u; s[1] = 0xbb67ae85u; s[2] = 0x3c6ef372u; s[3] = 0xa54ff53au;
  s[4] = 0x510e527fu; s[5] = 0x9b05688cu; s[6] = 0x1f83d9abu; s[7] = 0x5be0cd19u;
}

// One BIP-352 shared-secret hash.  mid = state after the constant first block,
// x = shared secret x as 8 little-endian u32 limbs (fully reduced), y_odd = parity
// of y.  Output t as 8 little-endian u32 limbs of the big-endian digest read as
// an integer (the reference's host conversion, src/cudasp_gpu.cu:862-877:
// limb j = digest bytes [31-4j-3 .. 31-4j] big-endian = digest word 7-j).
// k: the output index serialized after x as ser32(k) (BIP-352); the reference
// always hashes k = 0 (src/cudasp_gpu.cu:278-282).
CUDASP_SHA_HD void bip352_shared_secret_hash(uint32_t t[8], const uint32_t mid[8], const uint32_t x[8],
                                             uint32_t y_odd, uint32_t k = 0) {
  // ser = (0x02 | y_odd) || BE(x) || ser32(k)   (src/cudasp_gpu.cu:261-282, k = 0 there)
  // x BE bytes: word k of BE(x) = x limb (7-k).  The message starts one byte in.
  uint32_t w[16];
  uint32_t prefix = 0x02u | (y_odd & 1u);
  w[0] = (prefix << 24) | (x[7] >> 8);
#pragma unroll
  for (int k = 1; k < 8; k++) w[k] = (x[8 - k] << 24) | (x[7 - k] >> 8);
  w[8] = (x[0] << 24) | (k >> 8);       // last x byte, then ser32(k) bytes 0..2
  w[9] = (k << 24) | 0x00800000u;       // ser32(k) byte 3, then the 0x80 pad byte
  w[10] = 0; w[11] = 0; w[12] = 0; w[13] = 0; w[14] = 0;
  w[15] = (64u + 37u) * 8u;
  uint32_t s[8];
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = mid[i];
  sha256_compress(s, w);
#pragma unroll
  for (int j = 0; j < 8; j++) t[j] = s[7 - j];
}

}  // namespace cudasp
