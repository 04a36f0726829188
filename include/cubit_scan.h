/*
 * cubit_scan.h — C surface of libcubit_scan.so, the host-side mirror of DuckDB's
 * TableFunction callbacks for the bitmap-indexed scan (duckdb-cubit_amd/host/).
 *
 * Each entry point replaces one seq_scan callback (src/function/table/table_scan.cpp) and
 * keeps its contract:
 *   cubit_scan_init_global  ← TableScanInitGlobal   (table_scan.cpp:88-106)
 *                             (bind data = table partition + TransactionData): runs the GPU
 *                             scan (one ordered decode + the probes, on the device) and copies
 *                             only the count and tile directory to the host
 *   (the ids and probed values reach the host window by window — consecutive non-empty tiles,
 *    about 262,144 rows — when a local state claims the window, as seq_scan materialises a row
 *    group only when a thread takes its morsel)
 *   cubit_scan_max_threads  ← GlobalTableFunctionState::MaxThreads (DataTable::MaxThreads,
 *                             data_table.cpp:247-254)
 *   cubit_scan_init_local   ← TableScanInitLocal    (table_scan.cpp:67-86)
 *   cubit_scan_function     ← TableScanFunc         (table_scan.cpp:119-146): ≤ 2,048 rows per
 *                             call, 0 rows = finished (PhysicalTableScan::GetData,
 *                             physical_table_scan.cpp:82-103)
 *   cubit_scan_batch_index  ← TableScanGetBatchIndex (table_scan.cpp:179-189)
 *   cubit_scan_progress     ← TableScanProgress     (table_scan.cpp:158-177)
 *   cubit_scan_cardinality  ← TableScanCardinality  (table_scan.cpp:201-208): NodeStatistics of
 *                             the partition (bind time, no scan state)
 *   cubit_scan_statistics   ← TableScanStatistics   (table_scan.cpp:108-117): min / max /
 *                             has_null / has_no_null of a storage column; CUBIT_ERR_UNSUPPORTED
 *                             for the row id (the reference returns no statistics)
 * column_ids / projection_ids / filters mean what TableFunctionInitInput's members mean
 * (table_function.hpp:103-126): column_ids are storage columns (UINT64_MAX = row id), the
 * output holds column_ids[projection_ids[i]] (or every column_id when projection_ids is
 * empty), and filter columns need not be projected (filter_prune). Errors are status codes
 * with a message from cubit_scan_last_error(). cubit_scan_function may be called
 * concurrently with distinct local states (one per pipeline task).
 */
#ifndef CUBIT_SCAN_H
#define CUBIT_SCAN_H

#include <stdint.h>

#include "cubit_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define CUBIT_COLUMN_ROW_ID UINT64_MAX /* COLUMN_IDENTIFIER_ROW_ID */

typedef struct cubit_scan cubit_scan;
typedef struct cubit_scan_local cubit_scan_local;

const char *cubit_scan_last_error(void);
int cubit_scan_init_global(cubit_table *table, const uint64_t *column_ids, uint32_t n_column_ids,
                           const uint64_t *projection_ids, uint32_t n_projection_ids, const cubit_filter_node *nodes,
                           uint32_t n_nodes, const cubit_txn *txn, cubit_scan **out);
/* One scan over a table held as n_tables partitions (cubit_table_create row ranges: disjoint and
 * ascending in row order, CUBIT_ERR_INVALID otherwise), each on its own context — one device per
 * partition, or several partitions per device. DuckDB scans a table through one cursor over all
 * of its row groups (RowGroupCollection::InitializeParallelScan / NextParallelScan,
 * src/storage/table/row_group_collection.cpp:174-224): here every partition decodes and probes
 * on its own device (launched before any count is read, so the devices work side by side), the
 * windows of all partitions form one cursor in row order, each window is copied device-to-host
 * from its own partition, and batch index = the partition's first tile (the tiles of the earlier
 * partitions, ⌈n_rows / 131,072⌉ each) + its tile. No device-to-device exchange. */
int cubit_scan_init_global_multi(cubit_table *const *tables, uint32_t n_tables, const uint64_t *column_ids,
                                 uint32_t n_column_ids, const uint64_t *projection_ids, uint32_t n_projection_ids,
                                 const cubit_filter_node *nodes, uint32_t n_nodes, const cubit_txn *txn,
                                 cubit_scan **out);
int cubit_scan_max_threads(cubit_scan *scan, uint64_t *out);
int cubit_scan_init_local(cubit_scan *scan, cubit_scan_local **out);
/* out_columns[i] receives output column i (capacity 2,048 int64 each); *out_count the rows */
int cubit_scan_function(cubit_scan *scan, cubit_scan_local *local, int64_t *const *out_columns, uint64_t *out_count);
/* cubit_scan_function with each output column's validity: out_validity[i] (NULL, or either array
 * NULL, to skip) receives 32 LSB-first words — the chunk's FlatVector::Validity
 * (validity_mask.hpp:22,164-168), bit r = row r of the chunk valid, rows past *out_count set —
 * and a NULL row's value is 0. The reference's scan hands the vector's mask out with its values
 * (ColumnData::FilterScan + Vector::Slice, column_data.cpp:305-309, vector.cpp:223-258); the
 * values-only call drops it. */
int cubit_scan_function_validity(cubit_scan *scan, cubit_scan_local *local, int64_t *const *out_columns,
                                 uint64_t *const *out_validity, uint64_t *out_count);
int cubit_scan_batch_index(cubit_scan *scan, cubit_scan_local *local, uint64_t *out);
int cubit_scan_progress(cubit_scan *scan, double *out);
/* Decode launches init_global made, summed over the partitions: one per partition unless a
 * filter kept more than twice the rows cubit_table_estimate_rows predicted (then one more with
 * the exact count). Diagnostic: the reference's scan has no second pass to count. */
int cubit_scan_decodes(cubit_scan *scan, uint32_t *out);
int cubit_scan_cardinality(cubit_table *table, uint64_t *estimated, uint64_t *max);
int cubit_scan_statistics(cubit_table *table, uint64_t column_id, int64_t *min, int64_t *max, int *has_null,
                          int *has_no_null);
/* the same over the partitions of one table: rows summed; statistics merged (min of the
 * partitions' minima and max of their maxima over those holding a valid value, either NULL flag) */
int cubit_scan_cardinality_multi(cubit_table *const *tables, uint32_t n_tables, uint64_t *estimated, uint64_t *max);
int cubit_scan_statistics_multi(cubit_table *const *tables, uint32_t n_tables, uint64_t column_id, int64_t *min,
                                int64_t *max, int *has_null, int *has_no_null);
/* Buffers of finished scans are kept for the next one (page-locked host windows and device
 * result buffers; at most CUBIT_SCAN_CACHE_MB MiB pinned — default 1024 — and 16x that on the
 * device). This frees every cached buffer and reports what was cached (either pointer may be
 * NULL); call it before destroying a context whose scans are done. */
int cubit_scan_release_cached(uint64_t *pinned_bytes, uint64_t *device_bytes);
int cubit_scan_local_destroy(cubit_scan_local *local);
int cubit_scan_destroy(cubit_scan *scan);

#ifdef __cplusplus
}
#endif
#endif /* CUBIT_SCAN_H */
