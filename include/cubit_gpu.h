/*
 * cubit_gpu.h — C ABI of the MI355X bitmap-indexed table-scan filter (libcubitgpu.so).
 *
 * The reference (DuckDB v1.1.2, /root/reference) has no C ABI for this path: its drop-in
 * boundary is the C++ `TableFunction` callback struct
 * (src/include/duckdb/function/table_function.hpp:184-301) whose `seq_scan` implementation
 * (src/function/table/table_scan.cpp:119-146, 405-442) drives
 * RowGroup::TemplatedScan (src/storage/table/row_group.cpp:447-604). The entry points below
 * are what a C++ DuckDB extension calls from its replacement table
 * function; each cites the reference function whose work it takes over.
 *
 * Conventions: every call returns an int status (CUBIT_OK = 0), never
 * throws across the ABI, and records a message readable with cubit_last_error() (thread
 * local). Output buffers are caller-owned device buffers. A context owns one HIP stream
 * (cubit_ctx_set_stream), a claim ticket and a tile directory; every call on a context or on
 * its tables holds the context's mutex, so DuckDB's pipeline threads may share it (calls
 * serialise; GPU work stays asynchronous on the stream). Results named "last" belong to the
 * context's most recent call: threads that need their own give themselves a context each.
 * Row ids are int64 (DuckDB ROW_TYPE). Bitvectors are LSB-first 64-bit words, the layout
 * of DuckDB's ValidityMask (src/include/duckdb/common/types/validity_mask.hpp:22,164-168).
 */
#ifndef CUBIT_GPU_H
#define CUBIT_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes */
#define CUBIT_OK 0
#define CUBIT_ERR_INVALID 1      /* bad argument */
#define CUBIT_ERR_HIP 2          /* HIP runtime error */
#define CUBIT_ERR_OOM 3          /* device allocation failed */
#define CUBIT_ERR_UNSUPPORTED 4  /* predicate shape / type not supported */
#define CUBIT_ERR_CAPACITY 5     /* output buffer too small (count still reported) */
#define CUBIT_ERR_DEVICE 6       /* device-side failure (stream event creation, …) */

/* ---- physical types (DuckDB PhysicalType subset on the path: DATE = INT32,
 *      DECIMAL(15,2) = INT64, BIGINT = INT64, INTEGER = INT32). A column holds INT32 or INT64
 *      values; the narrower and unsigned codes name the T of BITPACKING segments
 *      (cubit_table_add_bitpacked_column; bitpacking.cpp:953-977 GetFunction: BOOL and INT8
 *      as int8_t, …, UINT64 and LIST offsets as uint64_t), unpacked into an INT32 column
 *      (INT8, INT16, UINT8, UINT16) or an INT64 column (UINT32). A UINT64 (UBIGINT) column
 *      holds the unsigned values' 64 bits and compares them unsigned, through the key
 *      v ^ 2^63 (cubit_fp_key): its constants, keys, update values, statistics and probed values
 *      are those bits in an int64. */
#define CUBIT_TYPE_INT32 0
#define CUBIT_TYPE_INT64 1
#define CUBIT_TYPE_INT8 2
#define CUBIT_TYPE_INT16 3
#define CUBIT_TYPE_UINT8 4
#define CUBIT_TYPE_UINT16 5
#define CUBIT_TYPE_UINT32 6
#define CUBIT_TYPE_UINT64 7
/* FLOAT / DOUBLE (PhysicalType::FLOAT / DOUBLE): the column holds the IEEE bit patterns as DuckDB's
 * vectors do, and every value crossing the ABI — filter constants, index keys, update values,
 * statistics, probed values — is a bit pattern carried in an int64 (FLOAT: the 32-bit pattern,
 * zero-extended). Comparisons follow DuckDB's floating-point operators
 * (src/common/vector_operations/comparison_operators.cpp:17-88, src/include/duckdb/common/
 * operator/comparison_operators.hpp:100-146): NaN equals NaN and is greater than every other value,
 * -0.0 equals +0.0. The library compares through cubit_fp_key below, an order-preserving map of the
 * patterns onto signed integers under which those operators are plain integer comparisons. */
#define CUBIT_TYPE_FLOAT 8
#define CUBIT_TYPE_DOUBLE 9
/* VARCHAR (PhysicalType::VARCHAR, string_t): the column holds int32 codes of an order-preserving
 * dictionary (cubit_dict: the distinct strings sorted as DuckDB compares them —
 * src/include/duckdb/common/types/string_type.hpp:143-206: the bytes as unsigned, then the length),
 * so a code comparison is the string comparison and every index, zonemap and kernel works on the
 * codes. A CONSTANT filter node on a VARCHAR column carries the ADDRESS of a cubit_string in
 * `constant` (the planner maps it to a code bound; strings absent from the dictionary included);
 * index keys (cubit_table_build_index `values`) likewise. Update values, appended values, probed
 * values and statistics are codes. */
#define CUBIT_TYPE_VARCHAR 10
/* HUGEINT / UHUGEINT (PhysicalType::INT128 / UINT128: hugeint_t / uhugeint_t, {lower, upper}) have
 * no column storage of their own: such a column is a dictionary column (cubit_table_add_dict_column)
 * over its values' 16-byte ORDER KEYS (cubit_key128: the 128 bits big-endian, HUGEINT's sign bit
 * flipped), whose unsigned byte order — the dictionary's order — is the values' order (hugeint_t's
 * and uhugeint_t's comparison operators). Its codes are the values' ranks, so every index, zonemap
 * and kernel works on them as on a VARCHAR column's; filter constants and index keys cross as
 * cubit_strings over their keys, probed codes map back through cubit_dict_entry + cubit_value128.
 * The type codes name the key encoding only (a column of more than 2^31 - 1 distinct values does
 * not fit the INT32 codes and stays on the caller's CPU path). */
#define CUBIT_TYPE_INT128 11
#define CUBIT_TYPE_UINT128 12
static inline void cubit_key128(int type, uint64_t lower, uint64_t upper, unsigned char key[16]) {
    if (type == CUBIT_TYPE_INT128) upper ^= 0x8000000000000000ull; /* signed order as unsigned bytes */
    for (int i = 0; i < 8; i++) {
        key[i] = (unsigned char)(upper >> (56 - 8 * i));
        key[8 + i] = (unsigned char)(lower >> (56 - 8 * i));
    }
}
static inline void cubit_value128(int type, const unsigned char key[16], uint64_t *lower, uint64_t *upper) {
    uint64_t hi = 0, lo = 0;
    for (int i = 0; i < 8; i++) {
        hi = (hi << 8) | key[i];
        lo = (lo << 8) | key[8 + i];
    }
    *lower = lo;
    *upper = type == CUBIT_TYPE_INT128 ? hi ^ 0x8000000000000000ull : hi;
}

/* The comparison key of a FLOAT / DOUBLE bit pattern or UINT64 value (any other type: the value
 * itself): UINT64 → v ^ 2^63; FLOAT / DOUBLE: every
 * NaN → one key above +inf's, -x → -(pattern of x) (so -0.0 and +0.0 share key 0), +x → its pattern.
 * cubit_fp_value is its inverse on keys (a NaN key → the positive quiet NaN, key 0 → +0.0). */
static inline int64_t cubit_fp_key(int type, int64_t bits) {
    if (type == CUBIT_TYPE_UINT64) return (int64_t)((uint64_t)bits ^ 0x8000000000000000ull);  /* unsigned order */
    if (type == CUBIT_TYPE_FLOAT) {
        const uint32_t u = (uint32_t)bits, mag = u & 0x7fffffffu;
        if (mag > 0x7f800000u) return 0x7fc00000;
        return (u >> 31) ? -(int64_t)mag : (int64_t)mag;
    }
    if (type == CUBIT_TYPE_DOUBLE) {
        const uint64_t u = (uint64_t)bits, mag = u & 0x7fffffffffffffffull;
        if (mag > 0x7ff0000000000000ull) return (int64_t)0x7ff8000000000000ull;
        return (u >> 63) ? -(int64_t)mag : (int64_t)mag;
    }
    return bits;
}
static inline int64_t cubit_fp_value(int type, int64_t key) {
    if (type == CUBIT_TYPE_UINT64) return (int64_t)((uint64_t)key ^ 0x8000000000000000ull);
    if (type == CUBIT_TYPE_FLOAT) return key < 0 ? (int64_t)(0x80000000u | (uint32_t)(-key)) : key;
    if (type == CUBIT_TYPE_DOUBLE) return key < 0 ? (int64_t)(0x8000000000000000ull | (uint64_t)(-key)) : key;
    return key;
}

/* ---- comparison (ExpressionType COMPARE_* used by ConstantFilter,
 *      src/planner/filter/constant_filter.cpp) */
#define CUBIT_CMP_EQ 0
#define CUBIT_CMP_NE 1
#define CUBIT_CMP_LT 2
#define CUBIT_CMP_LE 3
#define CUBIT_CMP_GT 4
#define CUBIT_CMP_GE 5

/* ---- filter node kinds: mirror TableFilterType (src/include/duckdb/planner/table_filter.hpp:20-27) */
#define CUBIT_FILTER_CONSTANT 0    /* ConstantFilter(cmp, constant) on `column` */
#define CUBIT_FILTER_IS_NULL 1
#define CUBIT_FILTER_IS_NOT_NULL 2
#define CUBIT_FILTER_OR 3          /* ConjunctionOrFilter, n_children follow (prefix order) */
#define CUBIT_FILTER_AND 4         /* ConjunctionAndFilter */

/* ---- bitmap index encodings */
#define CUBIT_INDEX_RANGE 0     /* L_j = {valid rows with v < edge_j}; exact for constants on edges */
#define CUBIT_INDEX_EQUALITY 1  /* E_k = {rows with v == value_k} (CUBIT's equality encoding) */
#define CUBIT_INDEX_BINS 2      /* B_i = {valid rows with edge_i <= v < edge_i+1}: kept beside a range or
                                   equality index on the same column; a range whose bounds are bin
                                   edges reads its bins instead of two range bitvectors when fewer */

/* ---- bitvector program opcodes (operands >= 0 are leaf indices, postfix order) */
#define CUBIT_OP_AND (-1)
#define CUBIT_OP_OR (-2)
#define CUBIT_OP_ANDNOT (-3) /* a AND NOT b */

/* ---- scan flags
 * Default output order ("tile runs"): the row ids of each 131,072-row tile form one
 * ascending run, and runs appear in the order tiles finished — the shape of DuckDB's
 * parallel table scan, whose morsels reach the sink in nondeterministic order with a batch
 * index (src/function/table/table_scan.cpp:179-189). cubit_ctx_last_tiles() returns the
 * tile directory ({start, length} per tile) that restores row order for free.
 * CUBIT_SCAN_ORDERED lays the runs out ascending: the look-back decode places each tile's run at
 * the sum of the earlier tiles' counts, so no extra pass (partitions up to 4,608 tiles = 6.0e8
 * rows; larger ones take one extra device pass). The small partitions that AUTO decodes with the
 * look-back kernel are ascending without the flag, too.
 * Capacity: *d_count is always the full number of qualifying rows. When it exceeds
 * `capacity` the calls still return CUBIT_OK (they do not wait for the kernel) and the
 * buffer holds an unspecified subset of the ids (runs are claimed in nondeterministic order;
 * with CUBIT_SCAN_ORDERED the ordered array has holes) — compare *d_count with capacity, or
 * pass CUBIT_SCAN_CHECK_CAPACITY, which waits for the scan and returns CUBIT_ERR_CAPACITY. */
#define CUBIT_SCAN_COUNT_ONLY 1u     /* do not materialise row ids */
#define CUBIT_SCAN_ORDERED 2u        /* one globally ascending array */
#define CUBIT_SCAN_CHECK_CAPACITY 4u /* synchronise; CUBIT_ERR_CAPACITY when *d_count > capacity */
/* Zonemaps (RowGroup::CheckZonemap / CheckZonemapSegments, src/storage/table/row_group.cpp:361-371,
 * 407-445): every index and validity bitvector carries, per zone of 131,072 rows, whether no row
 * or every row of the zone is set. A scan evaluates its filter over these classes (three-valued
 * logic) and skips the zones where it is false on every row — as the reference skips row groups
 * whose min/max statistics fail a filter. Results are identical either way; this flag turns the
 * skip off. */
#define CUBIT_SCAN_NO_ZONEMAP 8u

typedef struct cubit_ctx cubit_ctx;
typedef struct cubit_table cubit_table;
typedef struct cubit_dict cubit_dict;

/* a string constant or key of a VARCHAR column (string_t's data and size) */
typedef struct {
    const char *data;
    uint64_t size;
} cubit_string;

/* One node of a predicate tree in prefix order. A TableFilterSet (per-column AND,
 * table_filter.hpp:67-101) is an AND root whose children each reference one column; a
 * cross-column OR tree (the residual PhysicalFilter, execute_conjunction.cpp:56-142) uses
 * the same nodes. */
typedef struct {
    int32_t kind;       /* CUBIT_FILTER_* */
    int32_t cmp;        /* CUBIT_CMP_* (CONSTANT only) */
    int32_t column;     /* table column index (leaf kinds) */
    int32_t n_children; /* AND / OR */
    int64_t constant;   /* CONSTANT: value in the column's physical representation */
} cubit_filter_node;

/* DuckDB TransactionData{start_time, transaction_id} (src/include/duckdb/transaction/transaction_data.hpp) */
typedef struct {
    uint64_t start_time;
    uint64_t transaction_id;
} cubit_txn;

/* ------------------------------------------------------------------ context */
/* devices visible to the process (one context per device for a table held as partitions) */
int cubit_device_count(int *n);
int cubit_ctx_create(int device, cubit_ctx **out);
int cubit_ctx_destroy(cubit_ctx *ctx);
/* stream is a hipStream_t (NULL = the null stream). */
int cubit_ctx_set_stream(cubit_ctx *ctx, void *stream);
const char *cubit_last_error(void);
/* Which evaluate + decode kernel the context's scans launch: AUTO (the measured policy: the
 * look-back kernel — one workgroup per 131,072-row tile, output offsets by look-back over the
 * earlier tiles' counts — when the partition's tiles fit the co-resident grid; else the
 * run-claimed kernel when a workgroup walks three or more tiles, else the pair-claimed one),
 * or one of them always (tests and benchmarks; LOOKBACK up to 4,608 tiles). Results are
 * identical. Under AUTO a CUBIT_SCAN_ORDERED scan takes the look-back kernel at any size up to
 * 4,608 tiles (its runs land in tile order). */
#define CUBIT_DECODE_AUTO 0
#define CUBIT_DECODE_PAIRS 1
#define CUBIT_DECODE_RUNS 2
#define CUBIT_DECODE_LOOKBACK 3
/* reported by cubit_ctx_last_decode_kernel only: a program of one index bitvector as it stands
 * decodes with its offsets known up front (the bitvector's per-zone counts, kept with its zone
 * map): the look-back kernel without its walk, at any tile count; taken under AUTO and LOOKBACK */
#define CUBIT_DECODE_PREFIXED 4
int cubit_ctx_set_decode_kernel(cubit_ctx *ctx, int kernel);
/* Look-back decode: polls of an earlier tile's flag before the polling thread counts that tile
 * from its bitvectors itself (0 = the library default, 2^22). The expiry path is part of every
 * launch — no workgroup waits without bound and the count is always exact — and a small limit
 * forces it (tests). */
int cubit_ctx_set_lookback_spins(cubit_ctx *ctx, uint32_t spins);
/* The kernel the context's last decode launched (CUBIT_DECODE_PAIRS, _RUNS, _LOOKBACK or _PREFIXED; 0 when
 * the partition had no row and nothing was launched). */
int cubit_ctx_last_decode_kernel(cubit_ctx *ctx, int *kernel);
/* Filter-kernel durations measured with HIP events recorded around each launch on the
 * context stream (ms); requires cubit_ctx_enable_timing(ctx, 1). */
int cubit_ctx_enable_timing(cubit_ctx *ctx, int on);
int cubit_last_kernel_ms(cubit_ctx *ctx, float *ms);
/* Every timed filter-kernel launch since the last reset: ms[i] for i < min(cap, *n). */
int cubit_ctx_timing_reset(cubit_ctx *ctx);
int cubit_ctx_kernel_times(cubit_ctx *ctx, float *ms, uint32_t cap, uint32_t *n);
/* Steady-state decode time: the context's next decode launch is issued `reps` times back to
 * back on its stream between two stream events (reps <= 100000; 0 disarms). Every repeat
 * rewrites the same outputs from the same inputs, so results are unchanged. Afterwards
 * cubit_ctx_repeat_time gives the mean ms per launch and the number of launches bracketed.
 * A dispatch-stamped pair (cubit_ctx_enable_timing) puts a marker and its gap inside each
 * sample, which matters for kernels of a few microseconds. */
int cubit_ctx_set_repeat(cubit_ctx *ctx, uint32_t reps);
int cubit_ctx_repeat_time(cubit_ctx *ctx, double *ms_per_launch, uint32_t *launches);
/* Compile-time contract checks (vector 2048 = 32 words, row group 122880 = 1920 words). */
int cubit_abi_version(void);
int cubit_vector_size(void);
int cubit_row_group_size(void);

/* ------------------------------------------------------------------ device memory helpers */
int cubit_dev_alloc(cubit_ctx *ctx, uint64_t bytes, void **dptr);
int cubit_dev_free(cubit_ctx *ctx, void *dptr);
/* Page-locked host memory: device ↔ host copies into it run at the link's rate (the
 * table-function mirror stages its DataChunk columns here). cubit_host_free accepts a NULL
 * context (the memory outlives contexts). */
int cubit_host_alloc(cubit_ctx *ctx, uint64_t bytes, void **hptr);
int cubit_host_free(cubit_ctx *ctx, void *hptr);
int cubit_memcpy_h2d(cubit_ctx *ctx, void *dst, const void *src, uint64_t bytes);
int cubit_memcpy_d2h(cubit_ctx *ctx, void *dst, const void *src, uint64_t bytes);
int cubit_memset_d(cubit_ctx *ctx, void *dst, int value, uint64_t bytes);
/* Device → device copy enqueued on the context stream (not waited for): the table-function
 * mirror packs a group's 8-byte row ids into its staging block with it. */
int cubit_memcpy_d2d(cubit_ctx *ctx, void *dst, const void *src, uint64_t bytes);
int cubit_sync(cubit_ctx *ctx);
/* Copy streams: a stream of the context's device whose work starts after everything enqueued
 * on the context stream before the call (one pipeline task of the table-function mirror copies
 * its windows on its own, so the tasks' copies overlap instead of queueing on one stream).
 * cubit_memcpy_d2h_stream copies on it and waits for the copy; cubit_memcpy_d2h_async only
 * enqueues it, and cubit_copy_stream_sync waits for everything enqueued on the stream (the
 * copies of one window's columns, one wait). Destroyed streams go back to a pool of the context
 * (creating a HIP stream costs milliseconds) and are freed with it. */
int cubit_copy_stream_create(cubit_ctx *ctx, void **stream);
int cubit_copy_stream_destroy(cubit_ctx *ctx, void *stream);
int cubit_memcpy_d2h_stream(cubit_ctx *ctx, void *stream, void *dst, const void *src, uint64_t bytes);
int cubit_memcpy_d2h_async(cubit_ctx *ctx, void *stream, void *dst, const void *src, uint64_t bytes);
int cubit_copy_stream_sync(cubit_ctx *ctx, void *stream);
/* An event marking everything enqueued so far on a copy stream, or on the context stream when
 * `stream` is NULL (pooled per context): cubit_copy_event_sync waits for it on the host — a
 * consumer thread waits for one staged group of copies, not for the whole stream;
 * cubit_copy_stream_wait_event makes a copy stream wait for it on the device — the copies of a
 * group start when that group's probes are done; cubit_copy_event_destroy waits too and returns
 * it to the pool. */
int cubit_copy_event_record(cubit_ctx *ctx, void *stream, void **event);
int cubit_copy_event_sync(cubit_ctx *ctx, void *event);
int cubit_copy_stream_wait_event(cubit_ctx *ctx, void *stream, void *event);
int cubit_copy_event_destroy(cubit_ctx *ctx, void *event);
/* Synchronise the context stream and report any pending HIP error. */
int cubit_ctx_check(cubit_ctx *ctx);
/* Tile directory of the last row-id materialisation on this context (device pointer, valid
 * until the next scan): d_dir[2i] = start of tile i's run in the output, d_dir[2i+1] = its
 * length; tile i covers rows [i*rows_per_tile, (i+1)*rows_per_tile) of the partition. */
int cubit_ctx_last_tiles(cubit_ctx *ctx, const uint64_t **d_dir, uint32_t *n_tiles, uint64_t *rows_per_tile);

/* ------------------------------------------------------------------ low level (kernels) */

/* K0 — predicate → bitvector over a raw column (TemplatedFilterSelection compare,
 * column_segment.cpp:261-349; NULL never passes). words must hold
 * cubit_padded_words(n_rows) words; padding is zeroed. */
int cubit_build_bitvector(cubit_ctx *ctx, const void *d_col, int type, const uint64_t *d_validity, uint64_t n_rows,
                          int cmp, int64_t constant, uint64_t *d_words);
/* words per bitvector including tile padding */
uint64_t cubit_padded_words(uint64_t n_rows);

/* K1+K2 — evaluate a postfix program over `n_leaves` device bitvectors (each
 * cubit_padded_words(n_rows) words; leaf_negate bit k complements leaf k before use) and
 * write the int64 row ids row_base + r of the set rows into d_rowids (capacity `capacity`;
 * tile-run order unless CUBIT_SCAN_ORDERED), the count into *d_count (device). d_rowids may be NULL with
 * CUBIT_SCAN_COUNT_ONLY; d_result_words (optional) receives the evaluated bitvector.
 * Replaces the per-vector sel narrowing + row-id synthesis of RowGroup::TemplatedScan
 * (row_group.cpp:537-580). */
int cubit_bitvector_eval(cubit_ctx *ctx, const uint64_t *const *d_leaves, uint32_t n_leaves, uint32_t leaf_negate,
                         const int32_t *prog, uint32_t n_prog, uint64_t n_rows, int64_t row_base, int64_t *d_rowids,
                         uint64_t capacity, uint64_t *d_count, uint64_t *d_result_words, uint32_t flags);

/* K3 — gather a column at row ids: out[i] = col[rowids[i] - row_base] as int64
 * (ColumnData::FetchRow / FilterScan+Slice, column_data.cpp:305-309, 452-461). The number
 * of ids is read from *d_count (device), at most max_n. */
int cubit_gather(cubit_ctx *ctx, const void *d_col, int type, const int64_t *d_rowids, const uint64_t *d_count,
                 uint64_t max_n, int64_t row_base, int64_t *d_out);
/* Transfer compaction of a DataChunk column: d_out[i] = (int32)(d_in[i] - offset) for
 * i < min(*d_count, max_n). A caller whose column values all lie within [offset - 2^31,
 * offset + 2^31) (row ids of a partition below 2^31 rows with offset = row_base; DATE, or
 * DECIMAL / BIGINT whose statistics fit) moves 4 instead of 8 bytes per row to the host and
 * widens while it fills the vector (the table-function mirror's windows). */
int cubit_narrow_i32(cubit_ctx *ctx, const int64_t *d_in, const uint64_t *d_count, uint64_t max_n, int64_t offset,
                     int32_t *d_out);
/* cubit_narrow_i32 that checks the bound instead of trusting it: *d_overflow (device; the caller
 * zeroes it) becomes 1 when some value lies outside [offset - 2^31, offset + 2^31), and the
 * compacted copy must then not be used. */
int cubit_narrow_i32_checked(cubit_ctx *ctx, const int64_t *d_in, const uint64_t *d_count, uint64_t max_n,
                             int64_t offset, int32_t *d_out, uint32_t *d_overflow);
/* Transfer compaction to the width a column's statistics allow: d_out[i] = (unsigned, `width` =
 * 1, 2, 3 or 4 bytes, little-endian, packed)(d_in[i] - offset) for i < min(*d_count, max_n), for
 * values in [offset, offset + 2^(8·width)) — e.g. l_discount's 0 … 10 as one byte,
 * l_extendedprice's cents as three, a partition's row ids as four. *d_overflow
 * (device; the caller zeroes it) becomes 1 when a value lies outside, and the copy must then not
 * be used. */
int cubit_narrow_checked(cubit_ctx *ctx, const int64_t *d_in, const uint64_t *d_count, uint64_t max_n, int64_t offset,
                         int width, void *d_out, uint32_t *d_overflow);
/* Fused probe + reduce: sum over ids of a[r]*b[r] as a 128-bit integer (lo, hi int64 at
 * d_out[0..1]) — Q6's sum(l_extendedprice*l_discount) (DECIMAL(38,4) storage). */
int cubit_gather_sum_product(cubit_ctx *ctx, const int64_t *d_a, const int64_t *d_b, const int64_t *d_rowids,
                             const uint64_t *d_count, uint64_t max_n, int64_t row_base, int64_t *d_out);

/* ------------------------------------------------------------------ table partition API */

/* A row-range partition of a table resident on one device: rows [row_base, row_base+n_rows). */
int cubit_table_create(cubit_ctx *ctx, uint64_t n_rows, int64_t row_base, cubit_table **out);
int cubit_table_destroy(cubit_table *t);
/* rows, row base and owning context of a partition */
int cubit_table_info(cubit_table *t, uint64_t *n_rows, int64_t *row_base, cubit_ctx **ctx);
/* Device pointer (read-only, owned by the table or the caller that registered it) and type
 * of column `col`'s values — e.g. a column unpacked by K5 (ColumnData's decoded vectors,
 * src/storage/table/column_data.cpp:135-188). */
int cubit_table_column_data(cubit_table *t, int col, const void **data, int *type);
/* Register column `col`. data/validity are host pointers unless on_device = 1 (then the
 * table only references them). validity may be NULL (no NULLs). A caller-owned (on_device = 1)
 * buffer must not change while registered unless the caller says so with
 * cubit_table_column_changed: the table caches per-zone statistics of the values (zonemaps,
 * column statistics, selectivity estimates) and would otherwise skip zones by stale bounds.
 * Index bitvectors are not rebuilt by it (rebuild with cubit_table_build_index). `type` may be
 * any CUBIT_TYPE_* code: an 8- / 16-bit or unsigned column is widened on the device into an
 * owned INT32 / INT64 column (even from on_device data) — TINYINT … UINTEGER vectors as DuckDB
 * holds them; a UINT64 (UBIGINT) column keeps its values' bits and compares them unsigned; a FLOAT
 * or DOUBLE column is copied into the table (even from on_device data) as its bit patterns plus
 * their comparison keys (see the type codes) — widened and FP copies are the table's own, so a
 * later change to the caller's buffer is not seen: register the column again; a VARCHAR column is registered with its dictionary
 * (cubit_table_add_dict_column). Appends, updates and probes then use the stored values
 * (cubit_table_column_data reports the type held). */
int cubit_table_add_column(cubit_table *t, int col, int type, const void *data, const uint64_t *validity,
                           int on_device);
/* ---- VARCHAR dictionaries. A dictionary is built once per table (every partition of a table
 * encodes its rows against the same one, so codes are global) from any list of strings: n strings,
 * string i = bytes[offsets[i], offsets[i+1]) — duplicates and order do not matter; it keeps the
 * distinct ones sorted in DuckDB's string order (at most 2^31 - 1). Immutable once built: a table
 * that gains a string its dictionary lacks is re-registered with a new one (cubit_dict_encode
 * says so). cubit_dict_destroy drops the caller's reference; columns registered with the
 * dictionary hold their own until they go. Host-only: no context, no device memory. */
int cubit_dict_create(const char *bytes, const uint64_t *offsets, uint64_t n, cubit_dict **out);
int cubit_dict_destroy(cubit_dict *d);
int cubit_dict_size(const cubit_dict *d, uint64_t *n);
/* the string of a code (pointers into the dictionary, valid while it lives) */
int cubit_dict_entry(const cubit_dict *d, uint64_t code, const char **data, uint64_t *size);
/* codes[i] = the code of string i (layout as cubit_dict_create); a row whose validity bit is 0
 * (validity may be NULL) gets code 0 and its string is not read. CUBIT_ERR_UNSUPPORTED when a
 * valid string is not in the dictionary (codes are then unspecified). */
int cubit_dict_encode(const cubit_dict *d, const char *bytes, const uint64_t *offsets, uint64_t n,
                      const uint64_t *validity, int32_t *codes);
/* *lower_bound = the first code whose string is >= s (the size when none), *present = s is in it */
int cubit_dict_lookup(const cubit_dict *d, const char *data, uint64_t size, uint64_t *lower_bound, int *present);
/* cubit_dict_encode with every array in the context's device memory (the strings, their offsets,
 * the validity, the codes): one GPU lane per string searches the dictionary's entries (copied to
 * the device for the call). A valid string the dictionary lacks gets code -1 and makes the call
 * return CUBIT_ERR_UNSUPPORTED after the launch. */
int cubit_dict_encode_device(cubit_ctx *ctx, const cubit_dict *d, const char *d_bytes, const uint64_t *d_offsets,
                             uint64_t n, const uint64_t *d_validity, int32_t *d_codes);
/* Register a VARCHAR column: codes (host, or device with on_device = 1 as cubit_table_add_column)
 * of the table's rows against `d`, validity as for cubit_table_add_column. Every valid code must
 * lie in [0, size of d) (CUBIT_ERR_INVALID otherwise). The column holds a reference to d. */
int cubit_table_add_dict_column(cubit_table *t, int col, cubit_dict *d, const int32_t *codes, const uint64_t *validity,
                                int on_device);

/* The values of a caller-owned column changed: drop what the table derived from them. */
int cubit_table_column_changed(cubit_table *t, int col);
/* Register a column given as DuckDB BITPACKING segments (K5; the reference's persistent
 * integer storage, src/storage/compression/bitpacking.cpp): `bytes` holds the segment images
 * (each: 8-byte header = end of its metadata words, group data, metadata words of the
 * 2,048-row groups growing down), segment i at seg_offsets[i] (8-aligned) with seg_rows[i]
 * rows; the segments cover the partition in row order. The GPU unpacks every group
 * (CONSTANT, CONSTANT_DELTA, FOR, DELTA_FOR) into the column; NULLs come from `validity`
 * (host words; DuckDB keeps them in a separate validity segment). `type` is the segments' T,
 * any CUBIT_TYPE_* (header fields of T's size, T's wrap-around arithmetic); the column holds
 * the values widened to INT32 or INT64, or (UINT64) as their 64 bits, compared unsigned (see the
 * type codes). Malformed segments are
 * refused before anything is launched. With timing on, the unpack kernel is a timed launch
 * (cubit_last_kernel_ms). */
int cubit_table_add_bitpacked_column(cubit_table *t, int col, int type, const uint8_t *bytes, uint64_t n_bytes,
                                     const uint64_t *seg_offsets, const uint64_t *seg_rows, uint32_t n_segments,
                                     const uint64_t *validity);
/* Register a column given as DuckDB RLE segments (src/storage/compression/rle.cpp, the
 * reference's run-length codec for numeric columns): segment i at seg_offsets[i] with seg_rows[i]
 * rows, each as RLECompressState::FlushSegment writes it (8-byte header = offset of the uint16
 * run lengths, the run values as T from byte 8, the lengths after them; runs of at most 65,535
 * rows, zero-length runs allowed); the segments cover the partition in row order. The host reads
 * the runs (a segment whose runs do not cover its rows is refused before anything is launched),
 * only the runs cross to the device, and the GPU expands them into the column. `type` and the
 * column held are as for cubit_table_add_bitpacked_column; NULLs come from `validity` (a NULL
 * row's run value is whatever run it fell in, as in the reference). With timing on, the expand
 * kernel is a timed launch. */
int cubit_table_add_rle_column(cubit_table *t, int col, int type, const uint8_t *bytes, uint64_t n_bytes,
                               const uint64_t *seg_offsets, const uint64_t *seg_rows, uint32_t n_segments,
                               const uint64_t *validity);
/* Register a column given as DuckDB segments whose codecs differ from row group to row group, as
 * DuckDB's checkpoint picks one per segment (ColumnDataCheckpointer): seg_codecs[i] is
 * CUBIT_CODEC_UNCOMPRESSED (rows × T, the segment as FixedSizeAppend writes it),
 * CUBIT_CODEC_CONSTANT (no bytes; every row is seg_constants[i], the value as T widened to int64 —
 * a CONSTANT segment's value lives in its statistics), CUBIT_CODEC_RLE or CUBIT_CODEC_BITPACKING
 * (the layouts above); seg_offsets[i] is ignored for CONSTANT segments and seg_constants may be
 * NULL when there are none. The GPU writes every segment's rows; `type`, the column held and
 * `validity` as for cubit_table_add_bitpacked_column (the packed segments are not kept: the
 * packed filter does not apply). */
#define CUBIT_CODEC_UNCOMPRESSED 0
#define CUBIT_CODEC_CONSTANT 1
#define CUBIT_CODEC_RLE 2
#define CUBIT_CODEC_BITPACKING 3
int cubit_table_add_segment_column(cubit_table *t, int col, int type, const uint8_t *bytes, uint64_t n_bytes,
                                   const uint64_t *seg_offsets, const uint64_t *seg_rows, const int32_t *seg_codecs,
                                   const int64_t *seg_constants, uint32_t n_segments, const uint64_t *validity);
/* A column registered with cubit_table_add_bitpacked_column keeps its segments on the device:
 * a constant comparison the index cannot answer (K0) then unpacks and compares in one pass over
 * the packed bytes (w/8 bytes per row — the reference's ColumnSegment::Scan →
 * BitpackingScanPartial → FilterSelection, column_segment.cpp:378-522) instead of reading the
 * plain column. Off by default: on MI355X it measured 0.41–0.45 ms against K0's 0.43–0.44 ms
 * for a 600 M-row 12-bit date column (2.6x fewer bytes, but the unpack is instruction-bound, so
 * it does not win). Results are identical either way. Appends and merges drop the segments (the
 * plain column stays). cubit_table_last_packed: leaves the last scan built so. */
int cubit_table_use_packed_filter(cubit_table *t, int on);
int cubit_table_last_packed(cubit_table *t, uint32_t *n_leaves);
/* Selection narrowing (on by default): in a conjunction, a constant comparison on a column the
 * index cannot answer (K0) reads its column only at the rows the rest of the conjunction keeps,
 * when that is at most one row in 32 — the reference's filter loop reading each later filter
 * column through the selection of the earlier ones (RowGroup::TemplatedScan, row_group.cpp:
 * 537-550). Results are identical either way. cubit_table_last_narrowed: K0 leaves the last
 * scan built so. */
int cubit_table_use_narrowing(cubit_table *t, int on);
int cubit_table_last_narrowed(cubit_table *t, uint32_t *n_leaves);
/* The columns of the K0 comparisons the last scan built, in build order (cols[i] for i <
 * min(cap, *n)). Narrowing orders them by estimated selectivity — every literal's fraction of
 * kept rows from its column's per-zone min / max, the reference's AdaptiveFilter ordering
 * (src/execution/adaptive_filter.cpp:21-88) decided up front — most selective first, so the
 * order does not depend on the order of the filters; the estimate also decides whether to
 * narrow, without waiting for the device. */
int cubit_table_last_k0_order(cubit_table *t, int32_t *cols, uint32_t cap, uint32_t *n);
/* Build a bitmap index on `col` (K0). edges/values sorted ascending; n = 0 means "all
 * distinct values of the column" (exact for every constant). RANGE / EQUALITY replace the
 * column's primary index; BINS (n >= 2 edges) adds a secondary binned index. */
int cubit_table_build_index(cubit_table *t, int col, int encoding, const int64_t *values, uint32_t n);
/* Number of bitvectors and bytes held by the indexes on col, all encodings (0 if none). */
int cubit_table_index_info(cubit_table *t, int col, uint32_t *n_bitvectors, uint64_t *bytes);
/* Index persistence (the reference persists index state through IndexStorageInfo,
 * bound_index.hpp:117-118): write a column's RANGE / EQUALITY / BINS index (keys,
 * statistics, bitvectors) to one file, and load it back into a partition of the same size
 * (it replaces that encoding's index on the column). The file does not carry the column
 * data: load it only beside the column it was built from. It names the column's type and, for a
 * dictionary column (VARCHAR, HUGEINT / UHUGEINT), its dictionary (a fingerprint of the entries):
 * a load onto a column of another type or against another dictionary is refused
 * (CUBIT_ERR_INVALID). */
int cubit_table_save_index(cubit_table *t, int col, int encoding, const char *path);
int cubit_table_load_index(cubit_table *t, int col, const char *path);

/* MVCC delta. Deletes: rows with their delete ids (ChunkVectorInfo::deleted,
 * chunk_info.cpp:181-202). Updates on `col`: rows, new values and version ids
 * (UpdateSegment::Update, update_segment.cpp:1074-1199), chronological. Host arrays. */
int cubit_table_set_deletes(cubit_table *t, const int64_t *rows, const uint64_t *ids, uint64_t n);
int cubit_table_set_updates(cubit_table *t, int col, const int64_t *rows, const int64_t *values,
                            const uint64_t *versions, uint64_t n);
/* Updates that may set NULL (UPDATE … SET x = NULL, or a NULL row given a value): as
 * cubit_table_set_updates, plus valid[i] (1 = values[i], 0 = NULL; valid = NULL: every record
 * carries its value). DuckDB keeps these as the validity column's update chain beside the value
 * chain (InitializeUpdateValidity, src/storage/table/update_segment.cpp:588-600) and merges the
 * newest visible record into the vector's mask (UpdateMergeValidity :94-99, FetchRowValidity
 * :357-370). A reader that sees a SET NULL record finds the row in IS NULL and in no comparison,
 * and its probe reports NULL; cubit_table_column_statistics reports has_null. A column
 * registered without validity gets an all-valid one on the first SET NULL record. */
int cubit_table_set_updates_nullable(cubit_table *t, int col, const int64_t *rows, const int64_t *values,
                                     const uint8_t *valid, const uint64_t *versions, uint64_t n);
/* Inserts: n disjoint row ranges [row_begin[i], row_end[i]) appended by one transaction each,
 * with its insert id (ChunkConstantInfo::insert_id / ChunkVectorInfo::inserted,
 * src/storage/table/chunk_info.cpp:36-53, 123-161); a reader sees a range when
 * UseInsertedVersion(start_time, transaction_id, id) holds (chunk_info.cpp:11-19). Rows
 * outside every range were inserted before any snapshot. Replaces the previous set. */
int cubit_table_set_inserts(cubit_table *t, const int64_t *row_begin, const int64_t *row_end, const uint64_t *ids,
                            uint64_t n);

/* Index maintenance. Append n_new rows to the partition
 * (RowGroupCollection::Append, src/storage/table/row_group_collection.cpp, with every index's
 * BoundIndex::Append, src/include/duckdb/execution/index/bound_index.hpp:67-70): data[i] /
 * validity[i] are host arrays for column cols[i], one entry per registered column; validity[i]
 * = NULL (or validity = NULL) means all valid, else LSB-first words with bit 0 = the first
 * appended row. The new rows get local ids n_rows … n_rows+n_new-1; every index on every column
 * is maintained in place (bitvectors of the appended slice spliced in at bit n_rows; statistics
 * widened; an every-distinct-value index gains keys for values it has not seen). insert_id != 0
 * records [n_rows, n_rows+n_new) as an insert range of that transaction (see set_inserts);
 * 0 = visible to every snapshot. Storage grows geometrically when the padding runs out.
 * Columns registered as caller-owned device memory (add_column on_device = 1) are copied into
 * table-owned storage on the first append or merge; the caller's buffer is no longer read.
 * On an error the partition keeps its previous rows: scans and counts are those of the state
 * before the call (a later append overwrites the slice). What the failed call already did to
 * the indexes stays but never changes a result: bits spliced past the last row (masked by every
 * scan), statistics widened (bounds the values still lie within) and keys added to an
 * every-distinct-value index (exact leaves of values no row holds). */
int cubit_table_append(cubit_table *t, uint64_t n_new, const int *cols, const void *const *data,
                       const uint64_t *const *validity, uint32_t n_cols, uint64_t insert_id);
/* Merge the update records of `col` with version < horizon into the base values and the
 * column's indexes (the checkpoint of update chains, UpdateSegment, update_segment.cpp;
 * CUBIT's merge of its update bitvectors): each row takes its newest merged record — its value
 * (the row becomes valid) or NULL (the row's validity bit clears and it leaves every index
 * bitvector) — and the index bitvectors flip the rows whose predicate changed. Only snapshots with
 * start_time >= horizon may be served afterwards (as the reference folds versions only below
 * the lowest active start). Records at or past horizon stay. *n_merged = rows merged. */
int cubit_table_merge_updates(cubit_table *t, int col, uint64_t horizon, uint64_t *n_merged);

/* The scan: evaluate a predicate tree (prefix nodes) for transaction `txn` (NULL = see
 * every committed row, no MVCC delta applied) and write the qualifying row ids into
 * d_rowids (tile runs, or ascending with CUBIT_SCAN_ORDERED), the count into *d_count. Replaces TableScanFunc → DataTable::Scan →
 * RowGroup::TemplatedScan's filter + row-id materialisation (table_scan.cpp:119-146). */
int cubit_table_scan(cubit_table *t, const cubit_filter_node *nodes, uint32_t n_nodes, const cubit_txn *txn,
                     int64_t *d_rowids, uint64_t capacity, uint64_t *d_count, uint32_t flags);
/* cubit_table_scan plus this scan's tile directory (as cubit_ctx_last_tiles describes it),
 * copied into d_dir (room for dir_cap tiles, 2 words each) on the context's stream within the
 * same call: safe when several threads scan on one context, where a cubit_ctx_last_tiles read
 * after the scan may already describe another thread's scan. *n_tiles = 0: no run (the filter
 * folded away or nothing to decode). Not with CUBIT_SCAN_COUNT_ONLY; CUBIT_ERR_CAPACITY when
 * dir_cap is too small (a partition has ⌈n_rows / 131,072⌉ tiles). */
int cubit_table_scan_tiles(cubit_table *t, const cubit_filter_node *nodes, uint32_t n_nodes, const cubit_txn *txn,
                           int64_t *d_rowids, uint64_t capacity, uint64_t *d_count, uint32_t flags, uint64_t *d_dir,
                           uint32_t dir_cap, uint32_t *n_tiles, uint64_t *rows_per_tile);
/* Probe column `col` at the scan's row ids (visible values for txn; a NULL row's slot as stored). */
int cubit_table_probe(cubit_table *t, int col, const cubit_txn *txn, const int64_t *d_rowids, const uint64_t *d_count,
                      uint64_t max_n, int64_t *d_out);
/* The probe with NULL-ness — ColumnData::FilterScan + Vector::Slice (column_data.cpp:305-309,
 * vector.cpp:223-258) and FetchRow (column_data.cpp:452-461) hand back the vector's validity with
 * its values: d_out[i] = the visible value of row d_rowids[i], 0 when it is NULL, and bit i of
 * d_validity (LSB-first 64-bit words, DuckDB's ValidityMask layout; room for ⌈max_n / 64⌉ words,
 * the first ⌈min(*d_count, max_n) / 64⌉ written, bits past the count 0) = the row is valid for
 * txn, with its visible SET NULL / value records applied. */
int cubit_table_probe_validity(cubit_table *t, int col, const cubit_txn *txn, const int64_t *d_rowids,
                               const uint64_t *d_count, uint64_t max_n, int64_t *d_out, uint64_t *d_validity);
/* Estimated qualifying rows of a filter tree (the nodes cubit_table_scan takes), from the
 * per-zone min / max statistics the zonemaps use (values uniform within a zone, columns
 * independent) — the cardinality estimate a caller sizes its row-id buffer by, as DuckDB's
 * TableScanInitGlobal sizes nothing but the planner estimates a filtered scan's rows from column
 * statistics (table_scan.cpp:88-106, TableFilter::CheckStatistics). No kernel beyond the zone
 * statistics (computed once per table version); exactness never depends on it. */
int cubit_table_estimate_rows(cubit_table *t, const cubit_filter_node *nodes, uint32_t n_nodes, uint64_t *rows);
/* Bitvectors the last cubit_table_scan read per 64-row word (K) — for roofline bytes. */
int cubit_table_last_plan(cubit_table *t, uint32_t *n_leaves, uint32_t *n_passes);
/* Column statistics — DataTable::GetStatistics behind seq_scan's `statistics` callback
 * (TableScanStatistics, src/function/table/table_scan.cpp:108-117): min / max of the valid
 * values (widened by the column's update records, as UpdateSegment merges updates into the
 * segment statistics) and whether any row is NULL / non-NULL. min = max = 0 when no row is
 * valid. */
int cubit_table_column_statistics(cubit_table *t, int col, int64_t *min, int64_t *max, int *has_null,
                                  int *has_no_null);
/* Zones (131,072 rows each) the last scan or sum_product evaluated, out of the partition's
 * zones; fewer when the zonemaps skipped some (0 when the filter folded to FALSE). */
int cubit_table_last_zones(cubit_table *t, uint32_t *evaluated, uint32_t *zones);

/* SELECT sum(a * b) WHERE <filter> as one fused pass (K1 + K3): evaluate the program,
 * gather a (and b) for the qualifying rows only, accumulate in 128 bits — no row ids are
 * materialised. Replaces the scan → FilterScan/Slice probe (column_data.cpp:305-309) → SUM
 * chain of a query like TPC-H Q6 (sum(l_extendedprice * l_discount)). a and b are INT64
 * columns (DECIMAL storage); rows where a or b is NULL do not contribute. When the filter
 * pins b to at most 4 values of an exact range index, b is decoded from that index instead
 * of gathered (CUBIT_SUM_GATHER_B forces the gather). d_out[0..1] = {lo, hi} of the 128-bit
 * sum; d_count (optional) = qualifying rows. Visible MVCC updates on a or b fall back to
 * scan + probe (with validity when a column is nullable: NULL rows add nothing) + sum. */
#define CUBIT_SUM_GATHER_B 1u
#define CUBIT_SUM_NO_ZONEMAP 2u /* as CUBIT_SCAN_NO_ZONEMAP */
/* When a was registered as DuckDB BITPACKING segments (cubit_table_add_bitpacked_column), the
 * fused pass reads it at the qualifying rows straight from them: BitpackingScanPartial +
 * ColumnData::FilterScan (src/storage/compression/bitpacking.cpp:779-868, column_data.cpp:305-309)
 * as one pass that touches only the packed lines holding a qualifying row (a FOR value is its
 * group's base + w bits at bit i·w; rows of DELTA_FOR groups come from the unpacked column). The
 * gathers move whole 128-byte lines, so w-bit values touch fewer lines than 8-byte ones (SF100 Q6,
 * 24-bit l_extendedprice: 0.223 vs 0.245 ms). CUBIT_SUM_PLAIN_A reads the unpacked column instead;
 * CUBIT_SUM_PACKED_A names the default. */
#define CUBIT_SUM_PACKED_A 4u
#define CUBIT_SUM_PLAIN_A 8u
int cubit_table_sum_product(cubit_table *t, const cubit_filter_node *nodes, uint32_t n_nodes, const cubit_txn *txn,
                            int col_a, int col_b, int64_t *d_out, uint64_t *d_count, uint32_t flags);
/* How the last sum_product read b: number of values decoded from the index (0 = gathered). */
int cubit_table_last_sum_decode(cubit_table *t, uint32_t *n_values);
/* Whether the last sum_product read a from its BITPACKING segments. */
int cubit_table_last_sum_packed(cubit_table *t, int *packed);

#ifdef __cplusplus
}
#endif
#endif /* CUBIT_GPU_H */
