/* cudasp_oracle.h -- CPU restatement of the reference cudasp_scan algorithm.
 * TEST INFRASTRUCTURE ONLY (parity checker and CPU baseline); see
 * cudasp_oracle.c for the reference lines each step follows. */
#ifndef CUDASP_ORACLE_H
#define CUDASP_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CUDASP_ORACLE_LABEL_INFINITY ((int64_t)0x8000000000000000ULL)

/* One row: t (the 32-byte BE digest) and values[0] = base compare value,
 * values[1 + j] = value of label j (INT64_MIN if F + L_j is infinity).
 * Returns 0, or -1 if d*T or F is the point at infinity. */
int cudasp_oracle_row(const uint8_t scan_key_le[32], const uint8_t spend_key_le[64], const uint8_t* label_keys_le,
                      uint32_t label_count, const uint8_t tweak_le[64], uint8_t t_be_out[32], int64_t* values_out);

/* n rows with pthreads: flags_out[n] (may be NULL), values_out[n * (1+L)] (may be NULL). */
int cudasp_oracle_scan(const uint8_t scan_key_le[32], const uint8_t spend_key_le[64], const uint8_t* label_keys_le,
                       uint32_t label_count, const uint8_t* tweaks_le, uint32_t n, const int64_t* outputs,
                       const uint32_t* offsets, const uint32_t* lengths, uint8_t* flags_out, int64_t* values_out,
                       int threads);

/* Protocol variants (cudasp_scan_options of include/cudasp_abi.h). */
typedef struct {
  uint32_t output_count;   /* K >= 1 output indices per row (ser32(k)) */
  uint32_t label_negation; /* also F - L_j, after all F + L_j */
  uint32_t full_x;         /* outputs: 32-byte BE x-only keys */
} cudasp_oracle_options;

/* values_out[k * (1 + L') + c] (L' = L, or 2 L with label_negation); xs_out
 * (may be NULL) the same entries as 32-byte BE x (zeros at infinity);
 * t_be_out (may be NULL) K digests. */
int cudasp_oracle_row_ex(const uint8_t scan_key_le[32], const uint8_t spend_key_le[64], const uint8_t* label_keys_le,
                         uint32_t label_count, const uint8_t tweak_le[64], const cudasp_oracle_options* opt,
                         uint8_t* t_be_out, uint8_t* xs_out, int64_t* values_out);
/* outputs: int64 values, or 32-byte BE x per output with full_x;
 * values_out[n * K * (1 + L')]. */
int cudasp_oracle_scan_ex(const uint8_t scan_key_le[32], const uint8_t spend_key_le[64], const uint8_t* label_keys_le,
                          uint32_t label_count, const uint8_t* tweaks_le, uint32_t n, const cudasp_oracle_options* opt,
                          const void* outputs, const uint32_t* offsets, const uint32_t* lengths, uint8_t* flags_out,
                          int64_t* values_out, int threads);

int cudasp_oracle_synth_tweak(const uint8_t s0_le[32], uint64_t index, uint8_t out_le[64]);
void cudasp_oracle_sha256(uint8_t out[32], const uint8_t* msg, size_t len);
void cudasp_oracle_fp_mul(const uint8_t a[32], const uint8_t b[32], uint8_t out[32]);

#ifdef __cplusplus
}
#endif
#endif
