/*
 * cudasp_abi.h -- C ABI of the MI355X (gfx950) cudasp_scan hot path.
 *
 * Two layers, both plain C (pointers and sizes only, no HIP or torch types):
 *
 * 1. The reference's own three-phase batch ABI, same names, argument order and
 *    meaning, so the reference host (src/cudasp_extension.cu:21-52, which
 *    forward-declares these) links against this library unchanged:
 *      LaunchBatchScan      replaces src/cudasp_gpu.cu:445-669
 *      RunBatchScanKernels  replaces src/cudasp_gpu.cu:673-966
 *      FreeBatchScanState   replaces src/cudasp_gpu.cu:969-1023
 *    plus FreeBatchScanManaged, the replacement for the host's cudaFree of the
 *    three managed buffers (src/cudasp_extension.cu:395-397).
 *
 * 2. The scanner API the rebuilt host uses: one scanner per (query, device),
 *    created once with the query's keys (the bind-time data of
 *    CudaspScanBindData, src/cudasp_extension.cu:87-104), then any number of
 *    batches, either device-resident and asynchronous on a caller stream, or
 *    from host memory (synchronous, the ProcessBatch contract of
 *    src/cudasp_extension.cu:226-410).
 *
 * Byte conventions are the reference's (src/cudasp_extension.cu:59-85):
 * scan key 32 bytes little-endian; spend, label and tweak keys 64 bytes =
 * x (32 B LE) || y (32 B LE).  Limb arrays are u32, limb 0 least significant;
 * device tweak columns are column-major: limb j of row i at [j * n + i].
 *
 * A row matches when int64(upper 64 bits of (t*G + B).x), or of
 * (t*G + B + L_j).x for some label j, is in the row's outputs list, with
 * t = SHA256(SHA256("BIP0352/SharedSecret")^2 || ser(d*T) || 00000000)
 * (src/cudasp_gpu.cu:74-178, :236-354).
 *
 * Errors: functions return CUDASP_OK (0) or a negative code; the message of
 * the last failure on the calling thread is available from cudasp_last_error().
 */
#ifndef CUDASP_ABI_H
#define CUDASP_ABI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CUDASP_OK 0
#define CUDASP_ERR_INVALID_ARG (-2)
#define CUDASP_ERR_HIP (-3)
#define CUDASP_ERR_NO_DEVICE (-4)
#define CUDASP_ERR_CAPACITY (-5)

/* Thread-local message of the last failure ("" if none). */
const char* cudasp_last_error(void);
/* Library version string. */
const char* cudasp_version(void);
/* Number of visible HIP devices (0 if none). */
int cudasp_device_count(void);

/* ---------------------------------------------------------------- scanner */
typedef struct cudasp_scanner cudasp_scanner;

/* Create a scanner on `device` for one query's keys.  label_keys holds
 * label_count 64-byte keys back to back (may be NULL when label_count is 0).
 * max_rows bounds the rows of any later batch.  The first scanner on a device
 * also builds that device's fixed-base table for the default window width
 * (cudasp_default_fixed_base_bits: 26-bit windows, 21.5 GB, on devices with
 * >= 128 GiB such as MI355X, else 22-bit, 1.5 GiB; CUDASP_FB_BITS=22|26 in the
 * environment overrides), kept for the process; tables of different devices
 * build in parallel.  Device memory of a scanner: the key constants, plus the
 * scratch of the launches it runs (k_scan_multi: ~2 KB + 216 B per label per
 * launched thread; the stage kernels' buffers only once a stage-kernel path
 * runs -- the protocol variants, the values/stage entry points, the LDS width).
 * Fails with CUDASP_ERR_INVALID_ARG for a scan key that is 0 mod n. */
int cudasp_scanner_create(int device, const uint8_t scan_private_key[32], const uint8_t spend_public_key[64],
                          const uint8_t* label_keys, uint32_t label_count, uint32_t max_rows,
                          cudasp_scanner** out);
void cudasp_scanner_destroy(cudasp_scanner* s);
/* Rebind an existing scanner (its device buffers, streams and capacity kept)
 * to another query's keys: same validation and errors as create.  Must not be
 * called while a batch of the scanner is in flight.  Lets a host keep scanners
 * across queries instead of reallocating them (the reference allocates its
 * solver state per batch, src/cudasp_gpu.cu:445-669). */
int cudasp_scanner_set_keys(cudasp_scanner* s, const uint8_t scan_private_key[32],
                            const uint8_t spend_public_key[64], const uint8_t* label_keys, uint32_t label_count);

/* Fixed-base window width of stage B's t*G (the reference's gECC d_mul_table,
 * src/cudasp_gpu.cu:317-354).  Prebuilt widths: 22 bits (12 windows, 1.5 GiB
 * table per device in HBM), 26 bits (10 windows, 21.5 GB in HBM; two mixed
 * additions fewer per row, ~1.5% faster end to end) and 7 bits (37 windows,
 * 151.5 KB, staged into each workgroup's LDS -- measured slower: 36 mixed
 * additions per row).  Same results at every width.  The process default is
 * CUDASP_FB_BITS from the environment (22 or 26), else 26 on a device with
 * >= 128 GiB, else 22.  set_fixed_base_bits (0 = the default) switches a scanner's
 * table, building it on first use; not concurrent with work in flight on the
 * scanner.  table_bytes returns 0 for an unsupported width. */
int cudasp_default_fixed_base_bits(void);
uint64_t cudasp_fixed_base_table_bytes(int bits);
int cudasp_scanner_set_fixed_base_bits(cudasp_scanner* s, int bits);
int cudasp_scanner_fixed_base_bits(const cudasp_scanner* s);

/* The spend key folded into the fixed-base table's top window: the table's
 * reachable top-window entries P become P + B and P - B (a per-(device,
 * width, key) table shared by the scanners holding that key: 268 MB at 26
 * bits, 1 MB at 22), so stage B's F = t*G + B costs one mixed addition fewer.
 * Used only for a spend key on the curve (the group law makes the result the
 * reference's chord addition P0 + B; an off-curve key, which the reference's
 * formulas also take, is added on its own) and an HBM width.  On by default;
 * CUDASP_FB_FOLD=0 turns it off process-wide, set_spend_fold(s, 0) for one
 * scanner (not concurrent with work in flight on it).  spend_folded returns 1
 * when the scanner's launches use the fold.  Results never depend on it. */
int cudasp_scanner_set_spend_fold(cudasp_scanner* s, int on);
int cudasp_scanner_spend_folded(const cudasp_scanner* s);

/* Launch shape of the scanner's next launches: rows per thread of stage A
 * (1, 2 or 4) and stage B (2 or 6); 0 = automatic (the default: 4 and 6, or
 * fewer for launches too small to fill the device).  Rows of a thread run in
 * sequence and share one inversion, so fewer rows per thread shorten a launch
 * at a few percent more instructions per row: a host that knows a launch is
 * the tail of its work (the last batches of a rank or executor thread) can
 * trade that for a shorter drain.  Results do not depend on it. */
int cudasp_scanner_set_rows_per_thread(cudasp_scanner* s, int rows_a, int rows_b);

/* Protocol variants, off by default.  With the
 * defaults a scanner computes exactly the reference's flags.
 *   output_count   K >= 1: each row is tested for the output indices
 *                  k = 0 .. K-1, t_k = SHA256(H(tag)||H(tag)||ser(S)||ser32(k))
 *                  (BIP-352); the reference hashes k = 0 only
 *                  (src/cudasp_gpu.cu:278-282).  A row matches if any k does.
 *   label_negation nonzero: every label is also tested negated, F - L_j after
 *                  the F + L_j of all labels (the "(and negated)" of
 *                  src/cudasp_gpu.cu:938-939, which the reference kernel does
 *                  not do).
 *   full_x         nonzero: outputs are 32-byte big-endian x-only keys (on-chain
 *                  taproot output keys), compared with all of F.x instead of
 *                  the signed int64 of its upper 64 bits.  Device and host
 *                  output arrays then hold 32 bytes per output (an int64_t*
 *                  argument points at them; offsets and lengths count outputs).
 * Device-path buffer sizes scale with K: stage t arrays are 8 x (K n) words
 * and the diagnostic values (1 + L') x (K n), virtual row k * n + row, where
 * L' = label_count (x2 with label_negation). */
#define CUDASP_MAX_OUTPUT_COUNT 64
typedef struct {
  uint32_t output_count;
  uint32_t label_negation;
  uint32_t full_x;
} cudasp_scan_options;

/* Set a scanner's options (the keys are kept; buffers grow as needed).
 * Not concurrent with work in flight on the scanner. */
int cudasp_scanner_set_options(cudasp_scanner* s, const cudasp_scan_options* options);

/* Concurrency: a scanner's launches share its scratch and staging buffers, so
 * two launches of ONE scanner must not run at the same time -- issue them on
 * one stream (or order them).  Use one scanner per stream for concurrent
 * batches (the table-function host keeps one per executor thread; bench.py
 * one per stream).  Scanners of one device share only the read-only
 * fixed-base table.
 *
 * Stream arguments: a hipStream_t; NULL = the scanner's own stream (for the
 * entry points without a scanner: the null stream); CUDASP_STREAM_DEFAULT =
 * the device's null stream, for callers whose current stream is the default
 * stream (its handle is 0, which would otherwise select the scanner's stream
 * and lose the ordering with the caller's work). */
#define CUDASP_STREAM_DEFAULT ((void*)1)

/* Device-resident batch, asynchronous on `stream`.  Inputs: tweak x and y columns (8 x n each,
 * column-major), the outputs CSR (values, per-row u32 offset and length).
 * Outputs: d_match_flags[n] (0/1, required); if d_match_rows and
 * d_match_count are both non-NULL, *d_match_count (which the caller zeroes)
 * receives the number of matches and d_match_rows their row indices, in no
 * particular order. */
int cudasp_scan_device(cudasp_scanner* s, const uint32_t* d_tweak_x, const uint32_t* d_tweak_y,
                       const int64_t* d_outputs, const uint32_t* d_output_offsets,
                       const uint32_t* d_output_lengths, uint32_t n, uint8_t* d_match_flags,
                       uint32_t* d_match_rows, uint32_t* d_match_count, void* stream);

/* Several device-resident batches in one call (e.g. a rank's share of a
 * resident table): the same flags, and the same match rows and counts per
 * batch, as cudasp_scan_device on each batch in turn.  With the default
 * options (output_count 1) and an HBM fixed-base width (22 or 26 bits) one
 * persistent kernel runs both stages over all rows of all batches: every
 * wavefront takes 64-row pieces from a device work counter, up to 6 per thread
 * (sharing one inversion) while much work remains and 2, then 1 as it runs out,
 * so the GPU stays full to the end and t never leaves the thread.  Otherwise
 * the batches go through cudasp_scan_device one after the other.  Batch sizes
 * are not bounded by the scanner's capacity on the persistent path (the
 * per-batch path needs n <= capacity).  Asynchronous on `stream`; the
 * descriptor array is read before the call returns.  match_count words are
 * added to (the caller zeroes them). */
typedef struct {
  const uint32_t* tweak_x;          /* 8 x n, column-major */
  const uint32_t* tweak_y;
  const int64_t* outputs;
  const uint32_t* output_offsets;   /* n */
  const uint32_t* output_lengths;   /* n */
  uint32_t n;
  uint8_t* match_flags;             /* n, required */
  uint32_t* match_rows;             /* optional, with match_count */
  uint32_t* match_count;
} cudasp_device_batch;
int cudasp_scan_device_batches(cudasp_scanner* s, const cudasp_device_batch* batches, uint32_t count, void* stream);

/* Streaming scan (the table-function host's device feeds; no reference
 * counterpart: it replaces the per-batch H2D copy + launch + D2H of
 * ProcessBatch, src/cudasp_extension.cu:226-410, for batches that arrive
 * while the query runs).  ONE persistent kernel per stream scans every batch
 * published into it, reading the batch straight from pinned host memory (the
 * 64-byte tweak blobs as the table holds them, the outputs CSR) and writing
 * its results back there: one flag per row and/or the indices of the
 * matching rows; the host polls for each batch's completion.  Needs a
 * scanner with an HBM fixed-base width (22 or 26 bits), any output_count
 * (up to 6 indices per row ride the pipelined schedule; more are taken one
 * row per piece, in groups of 6 indices); the scanner must not run other
 * launches while a stream on it is open.
 *   cudasp_host_alloc   coherent pinned host memory, device-addressable at
 *                       the same address: every host buffer of a published
 *                       batch must lie in such an allocation (checked at
 *                       publish: the kernel's system-scope result stores
 *                       need coherent memory).  The GPU may still cache
 *                       lines of it: the kernel acquires at system scope
 *                       before each piece's reads, so a buffer rewritten for
 *                       a later batch is read fresh.
 *   cudasp_stream_supported  1 when the scanner's current keys and options
 *                       allow a stream (an HBM fixed-base width, a label
 *                       count whose scratch fits), else 0.
 *   cudasp_stream_create  blocks = 0: the whole device (3 waves per SIMD).
 *   cudasp_stream_publish_batch  a batch of n >= 1 rows (cudasp_stream_batch):
 *                       d_mirror is a device buffer as large as the batch's
 *                       outputs (>= 1 word; the kernel copies each row's
 *                       outputs there once); match_flags (n bytes) and/or
 *                       match_rows (room for n indices).  The buffers must
 *                       stay untouched until the batch is done; then any of
 *                       them, d_mirror included, may carry a later batch
 *                       (the kernel writes mirrors through).  *seq
 *                       receives the batch's sequence number.  At most 64
 *                       batches may be published and not yet done
 *                       (CUDASP_ERR_CAPACITY otherwise).  Launches the kernel
 *                       if none is running: a kernel that finds nothing to do
 *                       for CUDASP_STREAM_IDLE_MS (default 20 ms) ends, so a
 *                       stalled host never holds the GPU; publish and wait
 *                       relaunch it.
 *   cudasp_stream_publish  the same with match_flags only (no match_rows).
 *   cudasp_stream_close  no batch follows: the kernel ends as soon as every
 *                       published batch is done (finish still waits and resets).
 *   cudasp_stream_query  1: batch seq done (results written), 0: not yet, < 0: error.
 *   cudasp_stream_wait   blocks until batch seq is done; CUDASP_ERR_HIP when
 *                       no batch completed for the stream's timeout
 *                       (cudasp_stream_set_timeout, CUDASP_STREAM_TIMEOUT_MS,
 *                       default 60000 ms).
 *   cudasp_stream_matches  matching rows of a done batch (its match_rows
 *                       entries, in no particular order); valid until 64 more
 *                       batches are published.
 *   cudasp_stream_finish  end of input: closes, waits for every batch and for
 *                       the kernel (bounded by the timeout), then resets the
 *                       stream for reuse (sequence numbers start again at 0).
 *   cudasp_stream_abandoned  1 when finish timed out with the kernel still
 *                       running: nothing the kernel may touch (the stream, its
 *                       scanner, the batch buffers) may be freed.
 *   cudasp_stream_stats  kernel launches so far and grid blocks.
 *   cudasp_stream_counters  the kernel's counters of the last finished
 *                       query (queued by finish; reading them while the
 *                       kernel runs could wait for it), summed over its
 *                       launches: pieces, wave-rows, polls with nothing to
 *                       claim, pipeline drains, (unused), worker exits,
 *                       idle exits, poller polls, workers' busy and lifetime
 *                       ticks (100 MHz). */
typedef struct cudasp_stream cudasp_stream;
#define CUDASP_STREAM_MAX_OUTPUT_COUNT CUDASP_MAX_OUTPUT_COUNT
typedef struct {
  const uint8_t* tweak_keys;      /* n x 64 bytes (x then y, little-endian words) */
  const int64_t* outputs;         /* outputs CSR values (4 words per output with full_x) */
  const uint32_t* output_offsets; /* n, in outputs; n + 1 when output_lengths is NULL */
  const uint32_t* output_lengths; /* n, or NULL: output_offsets are Arrow list offsets (row r's list is
                                     outputs[offsets[r] .. offsets[r + 1]), e.g. a pinned Arrow column's) */
  uint32_t n;
  uint8_t* match_flags;           /* n flags, or NULL */
  uint32_t* match_rows;           /* room for n row indices, or NULL */
  int64_t* d_mirror;              /* device memory, the batch's outputs words (>= 1) */
} cudasp_stream_batch;
int cudasp_host_alloc(void** p, size_t bytes);
void cudasp_host_free(void* p);
int cudasp_stream_supported(const cudasp_scanner* s);
int cudasp_stream_create(cudasp_scanner* s, uint32_t blocks, cudasp_stream** out);
int cudasp_stream_publish_batch(cudasp_stream* st, const cudasp_stream_batch* batch, uint64_t* seq);
int cudasp_stream_publish(cudasp_stream* st, const uint8_t* h_tweak_keys, const int64_t* h_outputs,
                          const uint32_t* h_output_offsets, const uint32_t* h_output_lengths, uint32_t n,
                          uint8_t* h_match_flags, int64_t* d_mirror, uint64_t* seq);
int cudasp_stream_close(cudasp_stream* st);
int cudasp_stream_query(cudasp_stream* st, uint64_t seq);
int cudasp_stream_wait(cudasp_stream* st, uint64_t seq);
int cudasp_stream_set_timeout(cudasp_stream* st, uint32_t ms);
int cudasp_stream_matches(cudasp_stream* st, uint64_t seq, uint32_t* count);
int cudasp_stream_finish(cudasp_stream* st);
int cudasp_stream_abandoned(const cudasp_stream* st);
int cudasp_stream_stats(const cudasp_stream* st, uint64_t* launches, uint32_t* blocks);
int cudasp_stream_counters(cudasp_stream* st, uint64_t* out, uint32_t count);
void cudasp_stream_destroy(cudasp_stream* st);

/* Host batch, synchronous: tweak keys as n 64-byte blobs back to back, the
 * outputs CSR in host memory; writes h_match_flags[n]. */
int cudasp_scan_host(cudasp_scanner* s, const uint8_t* h_tweak_keys, const int64_t* h_outputs,
                     size_t outputs_size, const uint32_t* h_output_offsets, const uint32_t* h_output_lengths,
                     uint32_t n, uint8_t* h_match_flags);

/* Diagnostic stage outputs for parity tests, asynchronous on `stream`:
 * d_t (8 x n column-major) receives the shared-secret hash scalar t;
 * d_values ((1 + label_count) x n column-major) the int64 compare values of
 * the base output and of each label (INT64_MIN for a label sum at infinity). */
int cudasp_row_values_device(cudasp_scanner* s, const uint32_t* d_tweak_x, const uint32_t* d_tweak_y,
                             uint32_t n, uint32_t* d_t, int64_t* d_values, void* stream);

/* Wait for the scanner's own stream. */
int cudasp_scanner_sync(cudasp_scanner* s);

/* Transpose n row-major 64-byte tweak blobs (device memory) into x and y
 * columns (8 x n each), asynchronous on `stream`. */
int cudasp_tweaks_to_columns(const uint8_t* d_tweak_rows, uint32_t n, uint32_t* d_tweak_x, uint32_t* d_tweak_y,
                             void* stream);

/* Stage-level launches (the two kernels of cudasp_scan_device, separately;
 * used to time each kernel).  Asynchronous on `stream`. */
int cudasp_stage_shared_secret_device(cudasp_scanner* s, const uint32_t* d_tweak_x, const uint32_t* d_tweak_y,
                                      uint32_t n, uint32_t* d_t, void* stream);
int cudasp_stage_match_device(cudasp_scanner* s, const uint32_t* d_t, const int64_t* d_outputs,
                              const uint32_t* d_output_offsets, const uint32_t* d_output_lengths, uint32_t n,
                              uint8_t* d_match_flags, uint32_t* d_match_rows, uint32_t* d_match_count, void* stream);

/* The fixed-base table of `device` at window width `bits` (22, 26 or 7; 0 =
 * the device's default), built now unless it exists: a scanner created later
 * finds it ready.  A host that knows its devices calls this at load time (the
 * DuckDB extension's Load, in the background) so the first query does not
 * pay the build.  *build_seconds (may be NULL): the build's wall time, 0 when
 * the table already existed.  Thread-safe (one build per device and width). */
int cudasp_fixed_base_prepare(int device, int bits, double* build_seconds);
/* Test hook: every stride-th entry of that table recomputed on its own (a
 * double-and-add and an inversion per entry) and compared with the built
 * one; *checked entries, *mismatched of them differ.  Synchronous. */
int cudasp_debug_fb_check(int device, int bits, uint32_t stride, uint64_t* checked, uint64_t* mismatched);
/* Test hook: the spend-key fold table of `spend_public_key` (64 bytes, an
 * on-curve key) at 22 or 26 bits, built as a scanner builds it, and every
 * stride-th entry (its + B and - B halves) recomputed on its own (one
 * inversion per entry) and compared.  Synchronous. */
int cudasp_debug_fold_check(int device, int bits, const uint8_t spend_public_key[64], uint32_t stride,
                            uint64_t* checked, uint64_t* mismatched);

/* Shader clock of the last k_scan_multi launch on `device` (measurement
 * only): s_memtime ticks over s_memrealtime time of the grid's first wave,
 * in MHz, and that wave's life in seconds (may be NULL).  Synchronizes the
 * device.  Boxes of one pool differ by a few percent in this clock. */
int cudasp_debug_multi_clock(int device, double* mhz, double* seconds);

/* Layout probe (measurement only): reads the algorithmic bytes of n rows
 * (tweak columns, offsets, lengths, outputs) and writes a flag per row, with
 * stage A's thread-to-row mapping and no arithmetic, so rocprof / HIP events
 * show the HBM cost of the column-major layout on its own.  Asynchronous on
 * `stream` (NULL = the null stream).  The flags carry no meaning. */
int cudasp_layout_probe(const uint32_t* d_tweak_x, const uint32_t* d_tweak_y, uint32_t n, const int64_t* d_outputs,
                        const uint32_t* d_output_offsets, const uint32_t* d_output_lengths, uint8_t* d_flags,
                        void* stream);

/* Synthetic benchmark tables, generated on `device`:
 * tweak rows T_i = (s0 + first_index + i) G as x/y columns (8 x n each), and
 * k splitmix64 outputs per row: outputs[i*k + j] = splitmix64(seed ^ ((first_index + i)*k + j)),
 * offsets[i] = i*k, lengths[i] = k. */
int cudasp_synth_tweak_columns(int device, const uint8_t s0_le[32], uint64_t first_index, uint32_t n,
                               uint32_t* d_x, uint32_t* d_y, void* stream);
int cudasp_synth_outputs(uint64_t seed, uint64_t first_index, uint32_t n, uint32_t k, int64_t* d_outputs,
                         uint32_t* d_offsets, uint32_t* d_lengths, void* stream);
/* Variable-length lists (mean (kmax+1)/2 outputs per row): lengths uniform in
 * [1, kmax]; the caller exclusive-scans them into offsets, then the values. */
int cudasp_synth_output_lengths(uint64_t seed, uint64_t first_index, uint32_t n, uint32_t kmax, uint32_t* d_lengths,
                                void* stream);
int cudasp_synth_output_values(uint64_t seed, uint64_t first_index, uint32_t n, const uint32_t* d_offsets,
                               const uint32_t* d_lengths, int64_t* d_outputs, void* stream);

/* Test hooks (field arithmetic of the kernels, on the device).
 * cudasp_field_layout: the build's limb layout (10 x 26 or 9 x 29 bits, top
 * limb 22 / 24 bits) and its multiplication magnitude limits.
 * cudasp_debug_field_ops: for i < n, out[i] = a[i] * b[i] (op 0) or a[i]^2
 * (op 1) mod p, operands `limbs` u32 limbs each (row-major, any magnitude the
 * kernels accept); the result has magnitude 1, not fully reduced.  The 9 x 29
 * layout adds its fused forms, reading d_b as three n-element arrays b, c, e:
 * op 2 a*b + c*e, op 3 a*b + c^2, op 4 a*b + c, op 5 a^2 + c, op 6 3*a^2.
 * op 7: out[i] = a[i]^-1 mod p, fully reduced (0 for a[i] = 0 mod p; d_b is
 * not read).  Device buffers; synchronous. */
int cudasp_field_layout(int* limbs, int* bits, int* mul_mag_max, int* sqr_mag_max, int* limb_mag_max);
int cudasp_debug_field_ops(int op, const uint32_t* d_a, const uint32_t* d_b, uint32_t* d_out, uint32_t n);

/* -------------------------------------------- reference three-phase ABI */
void* LaunchBatchScan(uint32_t** managed_points_x, uint32_t** managed_points_y, const uint32_t* h_scalar,
                      const uint32_t* h_spend_pubkey_x, const uint32_t* h_spend_pubkey_y,
                      const uint32_t* h_label_keys_x, const uint32_t* h_label_keys_y, uint32_t label_count,
                      const int64_t* h_outputs, const uint32_t* h_output_offsets,
                      const uint32_t* h_output_lengths, uint8_t** managed_match_flags, uint32_t count,
                      size_t outputs_size);

int RunBatchScanKernels(void* state_handle, uint32_t* managed_points_x, uint32_t* managed_points_y,
                        const uint32_t* h_scalar, const uint32_t* h_spend_pubkey_x,
                        const uint32_t* h_spend_pubkey_y, const uint32_t* h_label_keys_x,
                        const uint32_t* h_label_keys_y, uint32_t label_count, uint8_t* managed_match_flags,
                        uint32_t count);

void FreeBatchScanState(void* state_handle);

/* Frees one of the managed buffers LaunchBatchScan allocated. */
void FreeBatchScanManaged(void* ptr);

#ifdef __cplusplus
}
#endif

#endif /* CUDASP_ABI_H */
