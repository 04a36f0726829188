// Host-side mirror of DuckDB's TableFunction interface for the bitmap-indexed scan.
//
// DuckDB v1.1.2 drives a table scan through the callback struct TableFunction
// (src/include/duckdb/function/table_function.hpp:184-301): bind → init_global →
// init_local (per pipeline task) → function (one DataChunk of ≤ STANDARD_VECTOR_SIZE rows per
// call, size 0 = finished; PhysicalTableScan::GetData, physical_table_scan.cpp:82-103), with
// get_batch_index for order-preserving sinks (table_scan.cpp:179-189) and
// table_scan_progress. `seq_scan` sets projection_pushdown / filter_pushdown /
// filter_prune (table_scan.cpp:422-442).
//
// cubit_scan is the drop-in replacement of seq_scan's callbacks for a table partition held
// by libcubitgpu (include/cubit_gpu.h): init_global runs the GPU scan once (fused evaluate +
// decode, then the probe of every projected column, K1–K3) — the way index_scan
// materialises its row-id list at plan time (table_scan.cpp:296-370) — and `function` hands
// the result out as DataChunks, one 131,072-row tile per morsel, so N pipeline tasks drain
// it concurrently and batch index = tile index restores row order.
//
// The types below reproduce the shape of the DuckDB ones this path touches, without the
// DuckDB headers (the shim in INTEGRATION.md maps them 1:1 onto the real classes).
#pragma once

#include <atomic>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/cubit_gpu.h"

namespace cubit {
namespace duck {

using idx_t = uint64_t;
using column_t = uint64_t;
constexpr column_t COLUMN_IDENTIFIER_ROW_ID = (column_t)-1;  // src/include/duckdb/common/constants.hpp
constexpr idx_t STANDARD_VECTOR_SIZE = 2048;                  // common/vector_size.hpp:16-20

// ValidityMask of one flat vector (src/include/duckdb/common/types/validity_mask.hpp:22,164-168):
// LSB-first 64-bit words, bit i = row i valid; no words allocated (all_valid) = every row valid,
// the state FlatVector::Validity starts in and a scan leaves for a column without NULLs.
struct ValidityMask {
    bool all_valid = true;
    uint64_t words[STANDARD_VECTOR_SIZE / 64];
    void SetAllValid() { all_valid = true; }
    bool RowIsValid(idx_t i) const { return all_valid || ((words[i >> 6] >> (i & 63)) & 1ull); }
};

// DataChunk with flat int64 vectors (ROW_TYPE row ids; DATE / DECIMAL(15,2) physical values
// widened to int64) and their validity masks. size() == 0 signals the end of the scan.
struct DataChunk {
    std::vector<std::vector<int64_t>> data;
    std::vector<ValidityMask> validity;
    idx_t count = 0;
    // caller-owned vectors of STANDARD_VECTOR_SIZE values per column (null entries: `data`), so a
    // chunk is filled where its consumer reads it instead of being copied there afterwards
    int64_t* const* external = nullptr;
    int64_t* Column(idx_t c) { return external && external[c] ? external[c] : data[c].data(); }
    void Initialize(idx_t n_columns) {
        data.assign(n_columns, std::vector<int64_t>(STANDARD_VECTOR_SIZE));
        validity.assign(n_columns, ValidityMask{});
        count = 0;
    }
    void Reset() {
        count = 0;
        for (auto& v : validity) v.SetAllValid();
    }
    idx_t size() const { return count; }
    void SetCardinality(idx_t n) { count = n; }
};

struct FunctionData {
    virtual ~FunctionData() = default;
};
struct GlobalTableFunctionState {
    virtual ~GlobalTableFunctionState() = default;
    virtual idx_t MaxThreads() const { return 1; }
};
struct LocalTableFunctionState {
    virtual ~LocalTableFunctionState() = default;
};

// TableFilterSet as prefix-order cubit_filter_node trees (kind/cmp/column/constant mirror
// ConstantFilter / IsNull / IsNotNull / ConjunctionAnd / ConjunctionOr); the root ANDs the
// per-column filters exactly like TableFilterSet::filters (table_filter.hpp:67-101).
struct TableFilterSet {
    std::vector<cubit_filter_node> nodes;
};

struct TableFunctionInitInput {
    const FunctionData* bind_data = nullptr;
    std::vector<column_t> column_ids;   // storage columns to scan (or ROW_ID)
    std::vector<idx_t> projection_ids;  // positions of column_ids to emit (filter_prune)
    const TableFilterSet* filters = nullptr;
    bool CanRemoveFilterColumns() const { return !projection_ids.empty(); }
};

struct TableFunctionInput {
    const FunctionData* bind_data;
    LocalTableFunctionState* local_state;
    GlobalTableFunctionState* global_state;
};

using table_function_init_global_t = std::unique_ptr<GlobalTableFunctionState> (*)(TableFunctionInitInput& input);
using table_function_init_local_t = std::unique_ptr<LocalTableFunctionState> (*)(TableFunctionInitInput& input,
                                                                                  GlobalTableFunctionState* gstate);
using table_function_t = void (*)(TableFunctionInput& data, DataChunk& output);
using table_function_get_batch_index_t = idx_t (*)(const FunctionData* bind_data, LocalTableFunctionState* lstate,
                                                   GlobalTableFunctionState* gstate);
using table_function_progress_t = double (*)(const FunctionData* bind_data, const GlobalTableFunctionState* gstate);

// NodeStatistics (src/include/duckdb/storage/statistics/node_statistics.hpp:16-33)
struct NodeStatistics {
    bool has_estimated_cardinality = false;
    idx_t estimated_cardinality = 0;
    bool has_max_cardinality = false;
    idx_t max_cardinality = 0;
};
// the numeric part of BaseStatistics (NumericStats min / max, has_null / has_no_null)
struct ColumnStatistics {
    int64_t min = 0, max = 0;
    bool has_null = false, has_no_null = false;
};
using table_function_cardinality_t = NodeStatistics (*)(const FunctionData* bind_data);
// false = no statistics (the reference returns nullptr, e.g. for the row-id column)
using table_statistics_t = bool (*)(const FunctionData* bind_data, column_t column_id, ColumnStatistics& out);

struct TableFunction {
    std::string name;
    table_function_t function = nullptr;
    table_function_init_global_t init_global = nullptr;
    table_function_init_local_t init_local = nullptr;
    table_function_get_batch_index_t get_batch_index = nullptr;
    table_function_progress_t table_scan_progress = nullptr;
    table_function_cardinality_t cardinality = nullptr;
    table_statistics_t statistics = nullptr;
    bool projection_pushdown = false;
    bool filter_pushdown = false;
    bool filter_prune = false;
};

// One row-range partition of the table as libcubitgpu holds it: rows [row_base, row_base +
// n_rows) on the device of `ctx`.
struct CubitPartition {
    cubit_table* table = nullptr;
    cubit_ctx* ctx = nullptr;
    idx_t n_rows = 0;
    int64_t row_base = 0;
};

// bind data: the table's partitions in row order (one per device, or several per device) and the
// reading transaction (TransactionData{start_time, id}). DuckDB scans one table through one
// cursor over every row group (RowGroupCollection::InitializeParallelScan / NextParallelScan,
// row_group_collection.cpp:174-224); the partitions play the row groups' part.
struct CubitScanBindData : public FunctionData {
    std::vector<CubitPartition> parts;
    idx_t n_rows = 0;  // all partitions
    bool has_txn = false;
    cubit_txn txn{};
};

TableFunction GetCubitScanFunction();

}  // namespace duck
}  // namespace cubit
