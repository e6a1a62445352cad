/*
 * cudasp_host.h -- C ABI of the rebuilt cudasp_scan table-function host.
 *
 * This is the DuckDB-independent core of the reference's host plumbing
 * (src/cudasp_extension.cu:87-659): bind-time validation, per-thread row
 * accumulation, batch trigger, round-robin GPU assignment, batch processing
 * through the kernel ABI of cudasp_abi.h, the mutex-guarded global match list
 * and the single-thread emit in chunks of at most 2048 rows.  A DuckDB
 * extension (duckdb_ext/cudasp_extension.cpp) maps DuckDB's TableFunction
 * callbacks 1:1 onto these calls; the tests drive the same calls directly.
 *
 *   reference                        this ABI
 *   CudaspScanBind        :420-509   cudasp_tf_bind
 *   CudaspScanInit        :511-514   cudasp_tf_init
 *   CudaspScanLocalInit   :516-532   cudasp_tf_local_init
 *   CudaspScanFunction    :534-552   cudasp_tf_function
 *   CudaspScanFinalFunction :554-624 cudasp_tf_final
 *
 * Every function is thread-safe in the way DuckDB calls the reference's: one
 * local state per executor thread, shared bind data and global state.
 * Failure messages of cudasp_tf_function / cudasp_tf_final are available from
 * cudasp_last_error() (cudasp_abi.h) on the calling thread.
 */
#ifndef CUDASP_HOST_H
#define CUDASP_HOST_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CUDASP_TF_NEED_MORE_INPUT 0 /* OperatorResultType::NEED_MORE_INPUT */
#define CUDASP_TF_FINISHED 0        /* OperatorFinalizeResultType::FINISHED */
#define CUDASP_TF_HAVE_MORE_OUTPUT 1 /* OperatorFinalizeResultType::HAVE_MORE_OUTPUT */
#define CUDASP_TF_VECTOR_SIZE 2048  /* STANDARD_VECTOR_SIZE */
#define CUDASP_TF_DEFAULT_BATCH 300000

typedef struct cudasp_tf_bind_data cudasp_tf_bind_data;
typedef struct cudasp_tf_global cudasp_tf_global;
typedef struct cudasp_tf_local cudasp_tf_local;

/* One bind-time argument as DuckDB hands it over: is_blob = the value's
 * logical type is BLOB. */
typedef struct {
  const uint8_t* data;
  uint64_t size;
  int is_blob;
} cudasp_tf_blob_arg;

/* Bind.  arg_count = number of positional arguments (4 expected);
 * label_keys_is_list = the 4th argument is a LIST; has_batch_size /
 * batch_size_is_integer / batch_size as for the named parameter.  On failure
 * returns a negative code and writes the reference's InvalidInputException
 * message (NUL-terminated, truncated to err_cap) into err. */
int cudasp_tf_bind(uint32_t arg_count, cudasp_tf_blob_arg scan_private_key, cudasp_tf_blob_arg spend_public_key,
                   int label_keys_is_list, const cudasp_tf_blob_arg* label_keys, uint32_t label_count,
                   int has_batch_size, int batch_size_is_integer, int64_t batch_size, cudasp_tf_bind_data** out,
                   char* err, size_t err_cap);
/* Named parameters of the protocol variants (SURVEY.md 8(f) row 4;
 * cudasp_scan_options of cudasp_abi.h), applied after cudasp_tf_bind:
 *   output_count := INTEGER    (1 .. CUDASP_MAX_OUTPUT_COUNT, default 1)
 *   label_negation := BOOLEAN  (default false)
 *   full_x := BOOLEAN          (default false; the outputs column is then
 *                               BLOB[] of 32-byte big-endian x-only keys, fed
 *                               through the child_blob_* members below)
 * has_* = 0 keeps the default.  The defaults are the reference's semantics.
 * On failure returns a negative code and writes the message into err. */
int cudasp_tf_bind_options(cudasp_tf_bind_data* b, int has_output_count, int64_t output_count,
                           int has_label_negation, int label_negation, int has_full_x, int full_x, char* err,
                           size_t err_cap);
void cudasp_tf_bind_free(cudasp_tf_bind_data* b);
uint64_t cudasp_tf_bind_batch_size(const cudasp_tf_bind_data* b);

/* Global state (one per query): detects the devices.
 *
 * Batching: every GPU (logical GPU, see below) gets one *device feed* per
 * query -- a ring of pinned batch slots that all executor threads fill
 * together, and 1..4 streams, each with its own scanner, that run the closed
 * slots (H2D, transpose, one fused k_scan_multi launch, D2H of the flags): as
 * many as fill the GPU, within the hardware queues HIP leaves the feed beside
 * the null stream's (3 at the default GPU_MAX_HW_QUEUES = 4).  A
 * slot closes once it holds >= batch_size rows (the reference's trigger,
 * src/cudasp_extension.cu:416-418, applied to a device's rows instead of one
 * thread's) or runs out of output/txid space, and is launched by the last
 * thread still copying into it.  The last thread to finish launches the
 * partial slots, waits for all batches and emits the matches.  Batch
 * composition therefore differs from the reference's per-thread batches; the
 * emitted multiset of rows does not.
 *
 * A warning goes to stderr (once per process) when a query's streams on one
 * device exceed GPU_MAX_HW_QUEUES - 1 (read from the environment; HIP's
 * default is 4; only possible with the CUDASP_TF_STREAMS override): streams
 * sharing a hardware queue serialize their kernels. */
int cudasp_tf_init(const cudasp_tf_bind_data* b, cudasp_tf_global** out);
void cudasp_tf_global_free(cudasp_tf_global* g);
int cudasp_tf_num_gpus(const cudasp_tf_global* g);

/* What a query's host did (for benchmarks and diagnostics; read after the
 * last cudasp_tf_final, before cudasp_tf_global_free). */
typedef struct {
  uint32_t feeds;                  /* logical GPUs that received rows */
  uint32_t streams_per_feed;       /* streams (= scanners) per device feed */
  uint32_t max_streams_per_device; /* streams on the busiest HIP device */
  uint32_t hw_queues;              /* GPU_MAX_HW_QUEUES seen at cudasp_tf_init (4 if unset) */
  uint64_t launches;               /* batches launched, all feeds */
  uint64_t rows;                   /* rows launched, all feeds */
  double harvest_wait_s;           /* executor-thread time blocked on GPU completion */
  double reserve_s;                /* executor-thread time getting room in a slot (harvests and waits included) */
  double copy_s;                   /* executor-thread time copying rows into the slots */
  double launch_s;                 /* executor-thread time issuing the batches' copies and kernels */
  uint32_t streaming_feeds;        /* feeds that ran the streaming scan (cudasp_stream_*: one
                                      persistent kernel reading the slots in place) */
} cudasp_tf_stats;
int cudasp_tf_get_stats(cudasp_tf_global* g, cudasp_tf_stats* out);

/* Local state (one per executor thread).  local_gpu is the logical GPU index
 * (0 .. num_gpus-1) assigned round-robin over threads
 * (src/cudasp_extension.cu:523-529): the GPU of the thread's first chunk; its
 * later chunks continue round-robin over the logical GPUs, so any number of
 * threads feeds any number of GPUs.  local_device is the HIP device of
 * local_gpu (the same unless the test hook CUDASP_TF_DEVICE_MAP="d0,d1,..."
 * maps the logical GPUs to devices, e.g. "0,0,0,0" for four logical GPUs on
 * one card, each with its own feed). */
int cudasp_tf_local_init(cudasp_tf_global* g, cudasp_tf_local** out);
void cudasp_tf_local_free(cudasp_tf_local* l);
int cudasp_tf_local_gpu(const cudasp_tf_local* l);
int cudasp_tf_local_device(const cudasp_tf_local* l);
/* The work assignment used for multi-GPU sharding: unit `ordinal` (an
 * executor thread in the host, src/cudasp_extension.cu:523-529; a batch of
 * the table in bench.py) goes to GPU ordinal mod num_gpus.  Host-only. */
uint32_t cudasp_assign_gpu(uint64_t ordinal, uint32_t num_gpus);
/* The GPU resources of a finished query's device feeds (scanners, streams,
 * pinned and device batch slots) are kept in a process-wide pool (at most 64
 * entries) and reused by later queries with the same device, batch capacity
 * and stream count; a later query only rebinds the keys.
 * cudasp_tf_release_pool frees every pooled entry; cudasp_tf_pool_size
 * reports how many are parked. */
void cudasp_tf_release_pool(void);
uint32_t cudasp_tf_pool_size(void);
/* Cold start (no reference counterpart: the reference initialises each
 * device inside the first batch, src/cudasp_gpu.cu:474-484): builds every
 * logical GPU's fixed-base table and parks one ready streaming feed per
 * logical GPU -- scanner, persistent-kernel stream, all batch slots pinned --
 * in the pool for queries of this batch_size (0 = 300000), so the first query
 * of the process only rebinds keys.  The DuckDB extension calls it from a
 * background thread at LOAD.  Feeds already pooled are kept; *seconds (may
 * be NULL) receives the wall time.  Streaming-feed configurations only (one
 * feed per device); otherwise CUDASP_ERR_INVALID_ARG. */
int cudasp_tf_prewarm(uint64_t batch_size, double* seconds);

/* One input chunk (<= CUDASP_TF_VECTOR_SIZE = 2048 rows; a larger count is
 * rejected with CUDASP_ERR_INVALID_ARG) of the input table, columns by position:
 * 0 txid BLOB, 1 height INTEGER, 2 tweak_key BLOB, 3 outputs BIGINT[]
 * (src/cudasp_extension.cu:159-163), in DuckDB's unified form.  Validity
 * arrays may be NULL (= all valid).  outputs: per-row list entries
 * (offset/length into child_values), list validity, child validity. */
typedef struct {
  uint32_t count;
  const uint8_t* const* txid_data;
  const uint32_t* txid_size;
  const uint8_t* txid_valid;
  const int32_t* height;
  const uint8_t* height_valid;
  const uint8_t* const* tweak_data;
  const uint32_t* tweak_size;
  const uint8_t* tweak_valid;
  const uint64_t* list_offset;
  const uint64_t* list_length;
  const uint8_t* list_valid;
  const int64_t* child_values;
  const uint8_t* child_valid;
  /* full_x: the outputs child vector as BLOBs (32 bytes each) */
  const uint8_t* const* child_blob_data;
  const uint32_t* child_blob_size;
} cudasp_tf_chunk;

/* in_out_function: copy the chunk's rows into a device feed (the next
 * logical GPU of this thread's round-robin); a slot that reaches batch_size
 * rows is launched.  May block while every slot of the feed is in flight.
 * Returns CUDASP_TF_NEED_MORE_INPUT or a negative error code (message via
 * cudasp_last_error()). */
int cudasp_tf_function(const cudasp_tf_bind_data* b, cudasp_tf_global* g, cudasp_tf_local* l,
                       const cudasp_tf_chunk* chunk);

/* DuckDB's vectors as they are (the extension's pass-through form; replaces
 * the per-row marshalling of the reference's CudaspScanFunction,
 * src/cudasp_extension.cu:154-224, and of a cudasp_tf_chunk): each column is
 * its UnifiedVectorFormat -- the data array, the selection vector (NULL =
 * identity) and the validity mask's 64-bit words (NULL = all valid, bit i of
 * word i / 64 LSB-first, indexed through the selection like the data) -- so
 * CudaspScanFunction passes pointers only.  Element types:
 *   txid, tweak_key:  string_t (16 bytes: length, then the bytes inline when
 *                     length <= 12, else a 4-byte prefix and a pointer)
 *   height:           int32_t
 *   outputs:          list_entry_t {offset, length} into the child vector
 *   child:            int64_t, or string_t with full_x (32-byte x-only keys);
 *                     element k = list offset + position, through the
 *                     child's own selection vector and validity
 * Row semantics equal cudasp_tf_function's; count <= CUDASP_TF_VECTOR_SIZE. */
#define CUDASP_TF_STRING_INLINE 12 /* string_t::INLINE_LENGTH */
typedef struct {
  uint32_t length;
  uint8_t prefix[4];  /* inline strings continue over ptr's 8 bytes */
  const uint8_t* ptr; /* length > CUDASP_TF_STRING_INLINE */
} cudasp_tf_string;
typedef struct {
  uint64_t offset;
  uint64_t length;
} cudasp_tf_list_entry;
typedef struct {
  const void* data;         /* UnifiedVectorFormat::data */
  const uint32_t* sel;      /* SelectionVector::data() (sel_t), NULL = identity */
  const uint64_t* validity; /* ValidityMask::GetData(), NULL = all valid */
} cudasp_tf_vector;
typedef struct {
  uint32_t count;
  cudasp_tf_vector txid;
  cudasp_tf_vector height;
  cudasp_tf_vector tweak;
  cudasp_tf_vector outputs;
  cudasp_tf_vector child; /* ListVector::GetEntry(outputs) over ListVector::GetListSize rows */
} cudasp_tf_vectors;

int cudasp_tf_function_vectors(const cudasp_tf_bind_data* b, cudasp_tf_global* g, cudasp_tf_local* l,
                               const cudasp_tf_vectors* vectors);

/* Columnar input: a run of rows of the same four
 * columns as Arrow arrays, so Parquet/Arrow data (or DuckDB's Arrow export)
 * feeds the batch buffers with bulk copies instead of per-row pointers.
 * Buffers follow the Arrow C data layout; each column carries its Arrow array
 * offset (element offset into its buffers); validity bitmaps are LSB-first and
 * may be NULL (= all valid).
 *   txid:    binary (int32 offsets[count+1], data)
 *   height:  int32 values
 *   tweak:   binary (int32 offsets) or, when tweak_offsets is NULL,
 *            fixed_size_binary of tweak_fixed_width bytes
 *   outputs: list<int64> (int32 offsets[count+1] into the child array, which
 *            has its own offset and validity)
 * Row semantics are those of cudasp_tf_function (NULL txid/height/tweak rows
 * skipped, tweak length 64 enforced, NULL list = no outputs, NULL elements
 * dropped); rows are consumed in 2048-row pieces, each fed like one DuckDB
 * chunk, so the results equal feeding the same rows through
 * cudasp_tf_function. */
typedef struct {
  uint64_t count;
  const int32_t* txid_offsets;
  const uint8_t* txid_data;
  const uint8_t* txid_validity;
  uint64_t txid_offset;
  const int32_t* height;
  const uint8_t* height_validity;
  uint64_t height_offset;
  const int32_t* tweak_offsets;
  const uint8_t* tweak_data;
  const uint8_t* tweak_validity;
  uint64_t tweak_offset;
  int32_t tweak_fixed_width;
  const int32_t* list_offsets;
  const uint8_t* list_validity;
  uint64_t list_offset;
  const int64_t* child_values;
  const uint8_t* child_validity;
  uint64_t child_offset;
  /* full_x: the child array as binary (int32 child_blob_offsets) or, when
   * child_blob_offsets is NULL, fixed_size_binary(child_blob_fixed_width) */
  const int32_t* child_blob_offsets;
  const uint8_t* child_blob_data;
  int32_t child_blob_fixed_width;
} cudasp_tf_columns;

int cudasp_tf_function_columns(const cudasp_tf_bind_data* b, cudasp_tf_global* g, cudasp_tf_local* l,
                               const cudasp_tf_columns* cols);

/* One output chunk: up to 2048 matching rows (txid, height, tweak_key).  The
 * pointers stay valid until the global state is freed. */
typedef struct {
  uint32_t count;
  const uint8_t* txid_data[CUDASP_TF_VECTOR_SIZE];
  uint32_t txid_size[CUDASP_TF_VECTOR_SIZE];
  int32_t height[CUDASP_TF_VECTOR_SIZE];
  const uint8_t* tweak_data[CUDASP_TF_VECTOR_SIZE];
  uint32_t tweak_size[CUDASP_TF_VECTOR_SIZE];
} cudasp_tf_output;

/* in_out_function_final: the last thread to finish launches the feeds'
 * partial slots, waits for every batch and emits all matches.  Returns
 * CUDASP_TF_FINISHED (0) or
 * CUDASP_TF_HAVE_MORE_OUTPUT (1), or a negative error code. */
int cudasp_tf_final(const cudasp_tf_bind_data* b, cudasp_tf_global* g, cudasp_tf_local* l, cudasp_tf_output* out);

/* Pinned tables (no reference counterpart: the reference copies every row of
 * every query into per-thread strings and managed buffers,
 * src/cudasp_extension.cu:188-223, 327-337).  A tweak table is static while
 * wallets come and go: a pinned table copies its rows ONCE into coherent
 * pinned host memory (cudasp_host_alloc), batched and laid out as the
 * streaming kernel reads them (64-byte tweak blobs, int64 outputs with Arrow
 * list offsets), and every scan publishes those batches in place to one
 * persistent k_scan_stream per GPU -- no host copy per query.
 *
 *   cudasp_pinned_create  batch_size rows per batch (0 = 300000; at most
 *                        10,000,000, CUDASP_ERR_INVALID_ARG otherwise);
 *                        devices: the HIP device of each logical GPU (NULL =
 *                        {0}); batch k goes to logical GPU k mod
 *                        device_count, round-robin like the reference's
 *                        threads over its GPUs (src/cudasp_extension.cu:523-529);
 *                        a device listed m times runs m streaming kernels on
 *                        1/m of its wave slots each.
 *   cudasp_pinned_create_placed  the same with a placement:
 *                        CUDASP_TABLE_PINNED (cudasp_pinned_create's): the
 *                        rows in pinned host memory, read over PCIe by each
 *                        scan's streaming kernels;
 *                        CUDASP_TABLE_HBM: the rows resident in device memory
 *                        in k_scan_multi's layout (~93 B per row with 2
 *                        outputs), each scan one cudasp_scan_device_batches
 *                        launch per logical GPU over all of its batches (the
 *                        device-resident rate; any label count).
 *   cudasp_pinned_append  one run of rows (cudasp_tf_columns, int64 outputs;
 *                        not full_x), numbered after the rows appended before
 *                        (skipped rows keep their numbers).  The rows'
 *                        semantics are cudasp_tf_function_columns's: a NULL
 *                        txid, height or tweak skips the row, a tweak of
 *                        another size than 64 bytes fails the whole run
 *                        (nothing of it is kept), a NULL list has no outputs,
 *                        NULL elements are dropped.  A batch is closed (copied
 *                        into pinned memory) at batch_size rows, or earlier
 *                        when its outputs would pass 2^32 words.  Not while a
 *                        scan of the same table runs.
 *   cudasp_pinned_scan   cudasp_scan over every appended row with the bound
 *                        keys and options of b (cudasp_tf_bind and
 *                        cudasp_tf_bind_options; full_x is
 *                        CUDASP_ERR_INVALID_ARG, as are label counts the
 *                        streaming scan cannot hold in the pinned
 *                        placement).  *rows receives the
 *                        numbers of the matching rows, ascending (free with
 *                        cudasp_pinned_free_rows), *count their count.  Scans
 *                        of one table run one at a time (a lock); scanners and
 *                        streaming kernels are kept and rebound between scans.
 *   cudasp_pinned_info   rows appended, rows pinned (non-skipped), batches,
 *                        pinned and device bytes, the placement, and the last
 *                        scan's seconds.
 *   cudasp_pinned_free   frees the table (a table whose last scan timed out
 *                        with a kernel still running keeps its memory).
 * Test hooks (environment, read at create): CUDASP_TF_NULL_DEVICE=1 keeps the
 * batches in plain host memory with no device call (scans fail with
 * CUDASP_ERR_NO_DEVICE); CUDASP_PINNED_TEST_MAX_WORDS lowers the 2^32 - 1
 * words at which a batch closes early. 
 * Errors: negative CUDASP_ERR_* codes with the message in cudasp_last_error(). */
typedef struct cudasp_pinned_table cudasp_pinned_table;
typedef struct {
  uint64_t rows_appended;
  uint64_t rows_pinned;
  uint64_t batches;
  uint64_t pinned_bytes;
  uint64_t last_matches;
  double last_scan_s;    /* the whole cudasp_pinned_scan call */
  double last_publish_s; /* until every batch was published */
  int32_t placement;     /* CUDASP_TABLE_PINNED or CUDASP_TABLE_HBM */
  uint64_t device_bytes; /* device memory of the batches (HBM: all of them; pinned: the outputs mirrors) */
} cudasp_pinned_info_t;
#define CUDASP_TABLE_PINNED 0
#define CUDASP_TABLE_HBM 1
int cudasp_pinned_create(uint64_t batch_size, const int* devices, uint32_t device_count, cudasp_pinned_table** out);
int cudasp_pinned_create_placed(uint64_t batch_size, const int* devices, uint32_t device_count, int placement,
                                cudasp_pinned_table** out);
int cudasp_pinned_append(cudasp_pinned_table* t, const cudasp_tf_columns* cols);
int cudasp_pinned_scan(cudasp_pinned_table* t, const cudasp_tf_bind_data* b, uint64_t** rows, uint64_t* count);
void cudasp_pinned_free_rows(uint64_t* rows);
int cudasp_pinned_info(const cudasp_pinned_table* t, cudasp_pinned_info_t* out);
void cudasp_pinned_free(cudasp_pinned_table* t);

#ifdef __cplusplus
}
#endif

#endif /* CUDASP_HOST_H */
