// Copies of executor-thread chunks into the batch slots (cudasp_host.cpp).
//
// The slots are write-once for the CPU: a slot's tweak blobs, outputs, txids
// and CSR words are written by the thread that reserved them and then read by
// the GPU (over PCIe, in place) or, for matching rows only, by the emit.
// Ordinary stores pull every destination line into the cache first (a read
// for ownership) and evict it later: 2x the bytes written in memory traffic,
// for data the CPU never reads back.  Non-temporal stores write the lines
// without reading them.  The host's per-row cost is memory traffic (the
// host ceiling), so the copies here use them; the
// writer issues an sfence before it commits the chunk (slot_copy_fence), so
// the stores are globally visible before the slot can be published.
#pragma once
#include <stdint.h>
#include <string.h>

#include <immintrin.h>

namespace cudasp_host {

// 64 bytes to a 16-byte aligned destination.
inline void nt_copy64(void* dst, const void* src) {
  const __m128i* s = static_cast<const __m128i*>(src);
  __m128i* d = static_cast<__m128i*>(dst);
  const __m128i a = _mm_loadu_si128(s), b = _mm_loadu_si128(s + 1), c = _mm_loadu_si128(s + 2),
                e = _mm_loadu_si128(s + 3);
  _mm_stream_si128(d, a);
  _mm_stream_si128(d + 1, b);
  _mm_stream_si128(d + 2, c);
  _mm_stream_si128(d + 3, e);
}

// 32 bytes to a 16-byte aligned destination.
inline void nt_copy32(void* dst, const void* src) {
  const __m128i* s = static_cast<const __m128i*>(src);
  __m128i* d = static_cast<__m128i*>(dst);
  const __m128i a = _mm_loadu_si128(s), b = _mm_loadu_si128(s + 1);
  _mm_stream_si128(d, a);
  _mm_stream_si128(d + 1, b);
}

// Any length and alignment: ordinary stores up to a 16-byte boundary and for
// the tail, non-temporal ones in between.
inline void nt_copy(void* dst, const void* src, size_t bytes) {
  uint8_t* d = static_cast<uint8_t*>(dst);
  const uint8_t* s = static_cast<const uint8_t*>(src);
  const size_t head = (16 - ((uintptr_t)d & 15)) & 15;
  if (bytes < head + 64) {
    memcpy(d, s, bytes);
    return;
  }
  memcpy(d, s, head);
  d += head;
  s += head;
  bytes -= head;
  for (; bytes >= 64; bytes -= 64, d += 64, s += 64) nt_copy64(d, s);
  for (; bytes >= 16; bytes -= 16, d += 16, s += 16)
    _mm_stream_si128(reinterpret_cast<__m128i*>(d), _mm_loadu_si128(reinterpret_cast<const __m128i*>(s)));
  memcpy(d, s, bytes);
}

// Before the chunk's commit: its non-temporal stores are globally visible.
inline void slot_copy_fence() { _mm_sfence(); }

}  // namespace cudasp_host
