// DuckDB v1.1.2 loadable extension that routes table scans with pushed filters to the MI355X
// bitmap-indexed scan (include/cubit_gpu.h, include/cubit_scan.h).
//
// This file is the DuckDB-side binding a maintainer adds. It compiles
// against the DuckDB headers only: `make -C duckdb-cubit_amd shim-check DUCKDB_INCLUDE=…`
// runs a full semantic check (g++ -fsyntax-only) against a DuckDB v1.1.2 source tree.
// Linking it needs libduckdb, which this repository does not build.
//
//   PRAGMA cubit_attach('lineitem', 'l_shipdate,l_discount,l_quantity,l_extendedprice'
//                       [, 'l_shipdate=range:1994-01-01,1995-01-01;l_discount=range;…' [, devices]]);
//     copies those columns to the GPU (every column from one snapshot; one row-range partition
//     per device, `devices` of them — 1 by default, 0 = every visible device) and builds the
//     named bitmap indexes;
//   PRAGMA cubit_sync('lineitem');
//     brings the partition to the table's committed state (appended rows, committed deletes;
//     every column again after an UPDATE of an attached one).
//   The optimizer swaps seq_scan for cubit_scan when every pushed filter of the scan is
//   supported, every scanned column is attached, and the partition is exactly the state the
//   scanning transaction sees (CubitPartitionIsCurrent); otherwise seq_scan runs as before.
//   The swapped scan checks again when it runs (CubitInitGlobal, in the executing transaction)
//   and hands the whole scan to seq_scan's own callbacks when the partition is not current —
//   a prepared statement keeps its plan across EXECUTEs (prepared_statement_data.cpp:64 re-plans
//   only on a catalog change), so the plan-time check alone would not do.
//
// Reference interfaces used (src/include/duckdb/…):
//   OptimizerExtension::optimize_function          optimizer/optimizer_extension.hpp:31-41
//     run after the built-in optimizers, i.e. after filter pushdown (optimizer.cpp:222-227)
//   LogicalGet::{function, bind_data, column_ids, projection_ids, table_filters}
//                                                  planner/operator/logical_get.hpp:38-60
//   TableFunction callbacks                        function/table_function.hpp:187-215
//   TableFilterSet / ConstantFilter / Conjunction* / Is[Not]NullFilter
//                                                  planner/table_filter.hpp:20-101, planner/filter/*.hpp
//   DuckTransaction::{start_time, transaction_id}  transaction/duck_transaction.hpp:23-38
#include <deque>

#include "duckdb.hpp"
#include "duckdb/catalog/catalog_entry/duck_table_entry.hpp"
#include "duckdb/catalog/catalog_entry/table_catalog_entry.hpp"
#include "duckdb/common/unordered_set.hpp"
#include "duckdb/function/function_set.hpp"
#include "duckdb/function/pragma_function.hpp"
#include "duckdb/function/table_function.hpp"
#include "duckdb/main/attached_database.hpp"
#include "duckdb/main/client_context_state.hpp"
#include "duckdb/main/extension_util.hpp"
#include "duckdb/planner/extension_callback.hpp"
#include "duckdb/transaction/meta_transaction.hpp"
#include "duckdb/optimizer/optimizer_extension.hpp"
#include "duckdb/parser/statement/insert_statement.hpp"
#include "duckdb/planner/filter/conjunction_filter.hpp"
#include "duckdb/planner/filter/constant_filter.hpp"
#include "duckdb/planner/filter/null_filter.hpp"
#include "duckdb/planner/operator/logical_delete.hpp"
#include "duckdb/planner/operator/logical_get.hpp"
#include "duckdb/planner/operator/logical_insert.hpp"
#include "duckdb/planner/operator/logical_update.hpp"
#include "duckdb/planner/table_filter.hpp"
#include "duckdb/common/enums/compression_type.hpp"
#include "duckdb/storage/block_manager.hpp"
#include "duckdb/storage/buffer_manager.hpp"
#include "duckdb/storage/data_table.hpp"
#include "duckdb/storage/table_io_manager.hpp"
#include "duckdb/storage/table_storage_info.hpp"
#include "duckdb/transaction/duck_transaction.hpp"
#include "duckdb/transaction/duck_transaction_manager.hpp"
#include "duckdb/transaction/local_storage.hpp"

#include "cubit_gpu.h"
#include "cubit_scan.h"

#include <memory>
#include <mutex>
#include <shared_mutex>

namespace duckdb {

// ------------------------------------------------------------------ registry

// A bitmap index the attach builds on one column (cubit_table_build_index): its encoding and
// keys (empty = every distinct value of the column).
struct CubitIndexSpec {
    column_t column;
    int encoding;  // CUBIT_INDEX_RANGE / _EQUALITY / _BINS
    vector<int64_t> keys;
    vector<string> str_keys;  // a VARCHAR column's keys (sorted, distinct)
};

// One GPU partition per attached table: the device context, the cubit_table, which storage
// columns it holds (with their physical width) and how current it is.
//
// Staleness is tracked per table, never through the database-wide last commit (every commit,
// read-only ones included, advances DuckTransactionManager::last_commit: GetCommitTimestamp,
// duck_transaction_manager.cpp:201-205, 248):
//  * appends: the table's row count (DataTable::GetTotalRows) against the partition's;
//  * deletes and updates: every DELETE, UPDATE and INSERT … ON CONFLICT DO UPDATE planned on
//    the table (CubitOptimize sees each plan) records its transaction id in `writers`. A sync
//    forgets a writer only once that transaction has finished before the sync's snapshot began
//    (transaction ids grow, so id < LowestActiveId() means finished), so whatever it committed
//    is in the snapshot the sync reads;
//  * the snapshot: `sync_start` is the start time of the transaction the last sync read the
//    table in (one transaction for every column). A scan may use the partition only if its own
//    snapshot includes that one (start_time >= sync_start).
//
// Lifetime: the contexts and the partitions are shared objects (CubitContexts,
// CubitPartitionSet). A scan holds its partition set from init_global until its global state
// goes away, and the bind-time callbacks hold it for their call, so an attach or a rebuilding sync
// that swaps a new set in under `lock` never frees a table or a context that a running scan still
// reads: the last holder does. Lock order: `lock`, then a set's `rw`.

// One context per device in use, destroyed with the last partition set built on them.
struct CubitContexts {
    vector<cubit_ctx *> ctxs;
    ~CubitContexts() {
        if (!ctxs.empty()) {
            cubit_scan_release_cached(nullptr, nullptr);  // pooled buffers of the contexts going away
        }
        for (auto c : ctxs) {
            cubit_ctx_destroy(c);
        }
    }
};

// The table as row-range partitions in row order, partition i on contexts->ctxs[i] (one partition
// per device: PRAGMA cubit_attach's `devices`), scanned through one cursor
// (cubit_scan_init_global_multi).
struct CubitPartitionSet {
    std::shared_ptr<CubitContexts> contexts;
    vector<cubit_table *> parts;
    vector<uint64_t> part_base;  // first row id of each partition
    // per dictionary column (VARCHAR; HUGEINT / UHUGEINT over their order keys): the
    // order-preserving dictionary every partition's codes index (one per table, so codes are
    // global); the chunks decode codes with it
    unordered_map<column_t, cubit_dict *> dicts;
    // a scan's init_global — the only part of a scan that reads the tables; its chunks come from
    // its own buffers — holds it shared; a sync's in-place appends and deletes hold it exclusive
    std::shared_mutex rw;
    ~CubitPartitionSet() {
        for (auto t : parts) {
            cubit_table_destroy(t);
        }
        for (auto &kv : dicts) {
            cubit_dict_destroy(kv.second);
        }
    }
};

struct CubitAttached {
    std::shared_ptr<CubitContexts> contexts;   // the contexts the next set is built on
    std::shared_ptr<CubitPartitionSet> set;    // the current partitions (under `lock`)
    int devices = 1;                           // devices the attach asked for (0 = every visible one)
    bool Attached() const {                    // under `lock`
        return set && !set->parts.empty();
    }
    std::shared_ptr<CubitPartitionSet> Current() {
        lock_guard<mutex> g(lock);
        return set;
    }
    unordered_map<column_t, PhysicalType> columns;
    vector<column_t> column_order;  // attached storage columns, in upload order
    vector<CubitIndexSpec> indexes; // the attach's index specification
    uint64_t gpu_rows = 0;          // rows of the GPU partition (row ids 0 … gpu_rows-1)
    transaction_t sync_start = 0;   // start time of the last sync's snapshot
    // writers not yet folded in by a sync: transaction id → whether it may change the values of
    // an attached column (then the sync re-reads every column). Recorded when a statement that
    // deleted or updated rows ends (CubitContextState::QueryEnd, every connection, prepared and
    // unoptimized statements included), when a DELETE / UPDATE is planned (NoteWriters), and at
    // attach for every still-active transaction that had already written (CubitRegistry::Dirty).
    unordered_map<transaction_t, bool> writers;
    mutex lock;  // scans, writers and syncs of different connections meet here
    mutex sync_lock;  // one attach or sync of the table at a time
};

class CubitRegistry {
public:
    static CubitAttached *Find(const TableCatalogEntry &t) {
        lock_guard<mutex> g(lock);
        auto it = map().find(&t);
        return it == map().end() ? nullptr : it->second.get();
    }
    // Every attached table of database `db` (a writer's changes cannot be attributed to a table
    // from the transaction's undo properties, so they count against all of them).
    static vector<std::pair<const TableCatalogEntry *, CubitAttached *>> InDatabase(const AttachedDatabase &db) {
        lock_guard<mutex> g(lock);
        vector<std::pair<const TableCatalogEntry *, CubitAttached *>> out;
        for (auto &kv : map()) {
            if (&kv.first->catalog.GetAttached() == &db) {
                out.emplace_back(kv.first, kv.second.get());
            }
        }
        return out;
    }
    // Transactions that deleted or updated rows, per database, whether or not a table was
    // attached then: an attach must not miss a writer that started before it and commits after
    // its snapshot. Entries of finished transactions (id < LowestActiveId) are dropped.
    static void NoteDirty(const AttachedDatabase &db, transaction_t id, bool values, transaction_t lowest_active) {
        lock_guard<mutex> g(lock);
        auto &m = dirty()[&db];
        for (auto it = m.begin(); it != m.end();) {  // finished writers: bounded however rare syncs are
            it = it->first < lowest_active ? m.erase(it) : std::next(it);
        }
        auto &w = m[id];
        w = w || values;
    }
    static unordered_map<transaction_t, bool> Dirty(const AttachedDatabase &db, transaction_t lowest_active) {
        lock_guard<mutex> g(lock);
        auto &m = dirty()[&db];
        for (auto it = m.begin(); it != m.end();) {
            it = it->first < lowest_active ? m.erase(it) : std::next(it);
        }
        return m;
    }
    static CubitAttached &Insert(const TableCatalogEntry &t) {
        lock_guard<mutex> g(lock);
        auto &slot = map()[&t];
        if (!slot) {
            slot = make_uniq<CubitAttached>();
        }
        return *slot;
    }

private:
    static unordered_map<const TableCatalogEntry *, unique_ptr<CubitAttached>> &map() {
        static unordered_map<const TableCatalogEntry *, unique_ptr<CubitAttached>> m;
        return m;
    }
    static unordered_map<const AttachedDatabase *, unordered_map<transaction_t, bool>> &dirty() {
        static unordered_map<const AttachedDatabase *, unordered_map<transaction_t, bool>> m;
        return m;
    }
    static mutex lock;
};
mutex CubitRegistry::lock;

static void Check(int rc) {
    if (rc != CUBIT_OK) {
        throw InvalidInputException("cubit: %s", cubit_last_error());
    }
}

// ------------------------------------------------------------------ filters

// Physical types whose values the GPU compares exactly, carried as int64: the signed integers up
// to 64 bits (DATE, TIME, TIMESTAMP*, DECIMAL(≤18) included), BOOLEAN, the unsigned integers up to
// 32 bits, and FLOAT / DOUBLE as their bit patterns (the library compares them with DuckDB's
// floating-point operators, include/cubit_gpu.h), UBIGINT as its bits (compared unsigned), and
// VARCHAR as int32 codes of the table's order-preserving dictionary (constants cross as
// cubit_strings), and HUGEINT / UHUGEINT as codes of a dictionary over their 16-byte order keys
// (cubit_key128: the codes are the values' ranks; constants cross as cubit_strings over keys).
static bool GpuPhysical(PhysicalType t) {
    switch (t) {
    case PhysicalType::BOOL:
    case PhysicalType::INT8:
    case PhysicalType::INT16:
    case PhysicalType::INT32:
    case PhysicalType::INT64:
    case PhysicalType::UINT8:
    case PhysicalType::UINT16:
    case PhysicalType::UINT32:
    case PhysicalType::UINT64:   // the bits, compared unsigned
    case PhysicalType::FLOAT:
    case PhysicalType::DOUBLE:
    case PhysicalType::VARCHAR:  // as codes of an order-preserving dictionary (cubit_dict)
    case PhysicalType::INT128:   // as codes of a dictionary over the values' order keys
    case PhysicalType::UINT128:
        return true;
    default:
        return false;
    }
}

// a column held as dictionary codes: VARCHAR (the strings), HUGEINT / UHUGEINT (their order keys)
static bool DictPhysical(PhysicalType t) {
    return t == PhysicalType::VARCHAR || t == PhysicalType::INT128 || t == PhysicalType::UINT128;
}

// a HUGEINT / UHUGEINT value as its 16-byte order key (cubit_key128), in a string for the
// dictionary's bytes + offsets layout
static string Key128(PhysicalType t, uint64_t lower, uint64_t upper) {
    unsigned char k[16];
    cubit_key128(t == PhysicalType::INT128 ? CUBIT_TYPE_INT128 : CUBIT_TYPE_UINT128, lower, upper, k);
    return string((const char *)k, 16);
}
static string Key128(const Value &v) {
    if (v.type().InternalType() == PhysicalType::INT128) {
        const auto h = v.GetValueUnsafe<hugeint_t>();
        return Key128(PhysicalType::INT128, h.lower, (uint64_t)h.upper);
    }
    const auto u = v.GetValueUnsafe<uhugeint_t>();
    return Key128(PhysicalType::UINT128, u.lower, u.upper);
}

// uploaded from 8-byte values (INT64, UINT32 widened, DOUBLE patterns; else from 4-byte ones)
static bool WidePhysical(PhysicalType t) {
    return t == PhysicalType::INT64 || t == PhysicalType::UINT32 || t == PhysicalType::UINT64 ||
           t == PhysicalType::DOUBLE;
}

// the CUBIT_TYPE_* a column is registered as
static int UploadType(PhysicalType t) {
    switch (t) {
    case PhysicalType::FLOAT:
        return CUBIT_TYPE_FLOAT;
    case PhysicalType::DOUBLE:
        return CUBIT_TYPE_DOUBLE;
    case PhysicalType::UINT64:
        return CUBIT_TYPE_UINT64;
    default:
        return WidePhysical(t) ? CUBIT_TYPE_INT64 : CUBIT_TYPE_INT32;
    }
}

static uint32_t FloatBits(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}
static int64_t DoubleBits(double d) {
    int64_t b;
    memcpy(&b, &d, 8);
    return b;
}

static bool Supported(const TableFilter &f) {
    switch (f.filter_type) {
    case TableFilterType::CONSTANT_COMPARISON: {
        auto &c = f.Cast<ConstantFilter>();
        if (!GpuPhysical(c.constant.type().InternalType())) {
            return false;
        }
        switch (c.comparison_type) {
        case ExpressionType::COMPARE_EQUAL:
        case ExpressionType::COMPARE_NOTEQUAL:
        case ExpressionType::COMPARE_LESSTHAN:
        case ExpressionType::COMPARE_LESSTHANOREQUALTO:
        case ExpressionType::COMPARE_GREATERTHAN:
        case ExpressionType::COMPARE_GREATERTHANOREQUALTO:
            return true;
        default:
            return false;
        }
    }
    case TableFilterType::IS_NULL:
    case TableFilterType::IS_NOT_NULL:
        return true;
    case TableFilterType::CONJUNCTION_OR:
        for (auto &ch : f.Cast<ConjunctionOrFilter>().child_filters) {
            if (!Supported(*ch)) {
                return false;
            }
        }
        return true;
    case TableFilterType::CONJUNCTION_AND:
        for (auto &ch : f.Cast<ConjunctionAndFilter>().child_filters) {
            if (!Supported(*ch)) {
                return false;
            }
        }
        return true;
    default:
        return false;  // STRUCT_EXTRACT and anything newer stay on seq_scan
    }
}

// one value of a flat vector of an integer-backed physical type, as int64
static int64_t PhysicalAsInt64(Vector &v, idx_t i) {
    switch (v.GetType().InternalType()) {
    case PhysicalType::BOOL:
        return FlatVector::GetData<bool>(v)[i] ? 1 : 0;
    case PhysicalType::UINT8:
        return FlatVector::GetData<uint8_t>(v)[i];
    case PhysicalType::UINT16:
        return FlatVector::GetData<uint16_t>(v)[i];
    case PhysicalType::UINT32:
        return FlatVector::GetData<uint32_t>(v)[i];
    case PhysicalType::INT8:
        return FlatVector::GetData<int8_t>(v)[i];
    case PhysicalType::INT16:
        return FlatVector::GetData<int16_t>(v)[i];
    case PhysicalType::INT32:
        return FlatVector::GetData<int32_t>(v)[i];
    case PhysicalType::FLOAT:
        return FloatBits(FlatVector::GetData<float>(v)[i]);  // the pattern, zero-extended
    case PhysicalType::DOUBLE:
        return DoubleBits(FlatVector::GetData<double>(v)[i]);
    default:
        return FlatVector::GetData<int64_t>(v)[i];
    }
}

static int64_t ConstantAsInt64(const Value &v) {
    switch (v.type().InternalType()) {
    case PhysicalType::BOOL:
        return v.GetValueUnsafe<bool>() ? 1 : 0;
    case PhysicalType::UINT8:
        return v.GetValueUnsafe<uint8_t>();
    case PhysicalType::UINT16:
        return v.GetValueUnsafe<uint16_t>();
    case PhysicalType::UINT32:
        return v.GetValueUnsafe<uint32_t>();
    case PhysicalType::INT8:
        return v.GetValueUnsafe<int8_t>();
    case PhysicalType::INT16:
        return v.GetValueUnsafe<int16_t>();
    case PhysicalType::INT32:
        return v.GetValueUnsafe<int32_t>();  // DATE days, INTEGER, DECIMAL(≤9)
    case PhysicalType::FLOAT:
        return FloatBits(v.GetValueUnsafe<float>());
    case PhysicalType::DOUBLE:
        return DoubleBits(v.GetValueUnsafe<double>());
    case PhysicalType::UINT64:
        return (int64_t)v.GetValueUnsafe<uint64_t>();  // the bits
    default:
        return v.GetValueUnsafe<int64_t>();  // BIGINT, DECIMAL(10..18) scaled
    }
}

// prefix-order cubit_filter_node tree of one column's TableFilter (kinds are numbered like
// TableFilterType, comparisons like the CUBIT_CMP_* of ExpressionType::COMPARE_*)
// A VARCHAR constant crosses as the address of a cubit_string over the Value's own bytes (the
// TableFilterSet outlives the scan's init_global, which plans it), a HUGEINT / UHUGEINT constant
// as one over its order key; the arena holds the structs and keys.
struct ConstantArena {
    std::deque<cubit_string> strings;
    std::deque<string> keys;
};
static void Emit(const TableFilter &f, int32_t column, vector<cubit_filter_node> &out, ConstantArena &arena) {
    cubit_filter_node n {};
    n.column = column;
    switch (f.filter_type) {
    case TableFilterType::CONSTANT_COMPARISON: {
        auto &c = f.Cast<ConstantFilter>();
        n.kind = CUBIT_FILTER_CONSTANT;
        switch (c.comparison_type) {
        case ExpressionType::COMPARE_EQUAL:
            n.cmp = CUBIT_CMP_EQ;
            break;
        case ExpressionType::COMPARE_NOTEQUAL:
            n.cmp = CUBIT_CMP_NE;
            break;
        case ExpressionType::COMPARE_LESSTHAN:
            n.cmp = CUBIT_CMP_LT;
            break;
        case ExpressionType::COMPARE_LESSTHANOREQUALTO:
            n.cmp = CUBIT_CMP_LE;
            break;
        case ExpressionType::COMPARE_GREATERTHAN:
            n.cmp = CUBIT_CMP_GT;
            break;
        default:
            n.cmp = CUBIT_CMP_GE;
            break;
        }
        const auto phys = c.constant.type().InternalType();
        if (phys == PhysicalType::VARCHAR) {
            const string &str = StringValue::Get(c.constant);
            arena.strings.push_back(cubit_string {str.data(), str.size()});
            n.constant = (int64_t)(intptr_t)&arena.strings.back();
        } else if (phys == PhysicalType::INT128 || phys == PhysicalType::UINT128) {
            arena.keys.push_back(Key128(c.constant));
            arena.strings.push_back(cubit_string {arena.keys.back().data(), 16});
            n.constant = (int64_t)(intptr_t)&arena.strings.back();
        } else {
            n.constant = ConstantAsInt64(c.constant);
        }
        out.push_back(n);
        return;
    }
    case TableFilterType::IS_NULL:
        n.kind = CUBIT_FILTER_IS_NULL;
        out.push_back(n);
        return;
    case TableFilterType::IS_NOT_NULL:
        n.kind = CUBIT_FILTER_IS_NOT_NULL;
        out.push_back(n);
        return;
    case TableFilterType::CONJUNCTION_OR:
    case TableFilterType::CONJUNCTION_AND: {
        const bool is_or = f.filter_type == TableFilterType::CONJUNCTION_OR;
        auto &children = is_or ? f.Cast<ConjunctionOrFilter>().child_filters
                               : f.Cast<ConjunctionAndFilter>().child_filters;
        n.kind = is_or ? CUBIT_FILTER_OR : CUBIT_FILTER_AND;
        n.n_children = (int32_t)children.size();
        out.push_back(n);
        for (auto &ch : children) {
            Emit(*ch, column, out, arena);
        }
        return;
    }
    default:
        throw InternalException("cubit: unsupported table filter reached Emit");
    }
}

// ------------------------------------------------------------------ table function

// The swapped scan keeps the seq_scan it replaced — TableScanFunction's callbacks and its
// TableScanBindData, as the binder made them (table_scan.cpp:405-442) — so that a scan whose
// partition is not current when it runs is seq_scan's, unchanged.
struct CubitBindData : public TableFunctionData {
    CubitBindData(DuckTableEntry &table_p, CubitAttached &attached_p, TableFunction seq_p,
                  unique_ptr<FunctionData> seq_bind_p)
        : table(table_p), attached(attached_p), seq(std::move(seq_p)), seq_bind(std::move(seq_bind_p)) {
    }
    DuckTableEntry &table;
    CubitAttached &attached;
    TableFunction seq;
    unique_ptr<FunctionData> seq_bind;
};

struct CubitGlobalState : public GlobalTableFunctionState {
    ~CubitGlobalState() override {
        if (scan) {
            cubit_scan_destroy(scan);
        }
    }
    idx_t MaxThreads() const override {
        return seq_global ? seq_global->MaxThreads() : max_threads;
    }
    cubit_scan *scan = nullptr;
    std::shared_ptr<CubitPartitionSet> set;  // released after the scan (member order)
    idx_t max_threads = 1;
    vector<LogicalType> out_types;  // output chunk column types, in output order
    vector<cubit_dict *> out_dicts;  // a dictionary output column's dictionary (held by `set`), else null
    ConstantArena constants;  // the VARCHAR / HUGEINT / UHUGEINT constants of the pushed filters
    // set when the scan runs as seq_scan (the partition was not current at init_global)
    unique_ptr<GlobalTableFunctionState> seq_global;
};

struct CubitLocalState : public LocalTableFunctionState {
    ~CubitLocalState() override {
        if (local) {
            cubit_scan_local_destroy(local);
        }
    }
    cubit_scan_local *local = nullptr;
    vector<vector<int64_t>> staging;  // one STANDARD_VECTOR_SIZE int64 buffer per output column
    vector<int64_t *> ptrs;
    vector<vector<uint64_t>> validity;  // one STANDARD_VECTOR_SIZE / 64-word mask per output column
    vector<uint64_t *> vptrs;
    unique_ptr<LocalTableFunctionState> seq_local;
};

static bool CubitPartitionIsCurrent(ClientContext &context, DuckTableEntry &table, CubitAttached &attached);
static bool PartitionCurrentLocked(ClientContext &context, DuckTableEntry &table, CubitAttached &attached);

// The partition set a scan may run on, taken with the freshness checks under one hold of the
// attached table's lock (a sync cannot land between the check and the set), and with the set's
// `rw` held shared until the scan's device work is launched: nullptr when the scan must be
// seq_scan's (stale, or a scanned column not on the GPU).
static std::shared_ptr<CubitPartitionSet> AcquireCurrent(ClientContext &context, DuckTableEntry &table,
                                                         CubitAttached &attached, const vector<column_t> &column_ids,
                                                         std::shared_lock<std::shared_mutex> &reading) {
    lock_guard<mutex> g(attached.lock);
    if (!PartitionCurrentLocked(context, table, attached)) {
        return nullptr;
    }
    for (auto c : column_ids) {  // a re-attach may have changed the column set
        if (c != COLUMN_IDENTIFIER_ROW_ID && !attached.columns.count(c)) {
            return nullptr;
        }
    }
    reading = std::shared_lock<std::shared_mutex>(attached.set->rw);
    return attached.set;
}

static unique_ptr<GlobalTableFunctionState> CubitInitGlobal(ClientContext &context, TableFunctionInitInput &input) {
    auto &bind = input.bind_data->Cast<CubitBindData>();
    // the plan may be older than the partition's state (a prepared statement, a write committed
    // since planning): check again in the executing transaction, and run as seq_scan if stale
    std::shared_lock<std::shared_mutex> reading;
    auto set = AcquireCurrent(context, bind.table, bind.attached, input.column_ids, reading);
    if (!set) {
        auto g = make_uniq<CubitGlobalState>();
        TableFunctionInitInput seq_input(bind.seq_bind.get(), input.column_ids, input.projection_ids, input.filters);
        g->seq_global = bind.seq.init_global(context, seq_input);
        return std::move(g);
    }
    auto g = make_uniq<CubitGlobalState>();
    vector<cubit_filter_node> nodes;
    if (input.filters && !input.filters->filters.empty()) {
        // the TableFilterSet is an AND over columns; its keys index column_ids
        nodes.push_back(cubit_filter_node {CUBIT_FILTER_AND, 0, 0, (int32_t)input.filters->filters.size(), 0});
        for (auto &kv : input.filters->filters) {
            Emit(*kv.second, (int32_t)input.column_ids[kv.first], nodes, g->constants);
        }
    }
    auto &tx = DuckTransaction::Get(context, bind.table.catalog);
    cubit_txn txn {tx.start_time, tx.transaction_id};
    vector<uint64_t> cols;
    for (auto c : input.column_ids) {
        cols.push_back(c == COLUMN_IDENTIFIER_ROW_ID ? CUBIT_COLUMN_ROW_ID : (uint64_t)c);
    }
    vector<uint64_t> proj(input.projection_ids.begin(), input.projection_ids.end());
    g->set = set;
    auto &parts = set->parts;
    if (cubit_scan_init_global_multi(parts.data(), (uint32_t)parts.size(), cols.data(), (uint32_t)cols.size(),
                                     proj.data(), (uint32_t)proj.size(), nodes.data(), (uint32_t)nodes.size(), &txn,
                                     &g->scan) != CUBIT_OK) {
        throw InvalidInputException("cubit_scan: %s", cubit_scan_last_error());
    }
    reading.unlock();  // the chunks come from the scan's own buffers
    uint64_t mt = 1;
    cubit_scan_max_threads(g->scan, &mt);
    g->max_threads = mt;
    const bool pruned = input.CanRemoveFilterColumns();
    const idx_t n_out = pruned ? input.projection_ids.size() : input.column_ids.size();
    for (idx_t i = 0; i < n_out; i++) {
        const column_t c = input.column_ids[pruned ? input.projection_ids[i] : i];
        g->out_types.push_back(c == COLUMN_IDENTIFIER_ROW_ID
                                   ? LogicalType(LogicalType::ROW_TYPE)
                                   : bind.table.GetColumn(LogicalIndex(c)).GetType());
        auto d = set->dicts.find(c);
        g->out_dicts.push_back(c != COLUMN_IDENTIFIER_ROW_ID && d != set->dicts.end() ? d->second : nullptr);
    }
    return std::move(g);
}

static unique_ptr<LocalTableFunctionState> CubitInitLocal(ExecutionContext &context, TableFunctionInitInput &input,
                                                          GlobalTableFunctionState *global_state) {
    auto &g = global_state->Cast<CubitGlobalState>();
    auto l = make_uniq<CubitLocalState>();
    if (g.seq_global) {
        auto &bind = input.bind_data->Cast<CubitBindData>();
        if (bind.seq.init_local) {
            TableFunctionInitInput seq_input(bind.seq_bind.get(), input.column_ids, input.projection_ids, input.filters);
            l->seq_local = bind.seq.init_local(context, seq_input, g.seq_global.get());
        }
        return std::move(l);
    }
    if (cubit_scan_init_local(g.scan, &l->local) != CUBIT_OK) {
        throw InternalException("cubit_scan: %s", cubit_scan_last_error());
    }
    l->staging.resize(g.out_types.size(), vector<int64_t>(STANDARD_VECTOR_SIZE));
    l->validity.resize(g.out_types.size(), vector<uint64_t>(STANDARD_VECTOR_SIZE / 64));
    for (idx_t c = 0; c < g.out_types.size(); c++) {
        l->ptrs.push_back(l->staging[c].data());
        l->vptrs.push_back(l->validity[c].data());
    }
    return std::move(l);
}

template <class T>
static void Narrow(const int64_t *src, Vector &dst, idx_t n) {
    auto d = FlatVector::GetData<T>(dst);
    for (idx_t i = 0; i < n; i++) {
        d[i] = (T)src[i];
    }
}

// int64 staging → the column's physical type (DATE/INTEGER narrow, BIGINT/DECIMAL copy; VARCHAR
// codes → the dictionary's strings, copied into the vector's string heap; a NULL row's code is 0
// and its slot is left as the validity mask says)
static void CopyOut(const int64_t *src, Vector &dst, idx_t n, const uint64_t *valid, cubit_dict *dict) {
    switch (dst.GetType().InternalType()) {
    case PhysicalType::VARCHAR: {
        auto d = FlatVector::GetData<string_t>(dst);
        for (idx_t i = 0; i < n; i++) {
            const char *p = nullptr;
            uint64_t len = 0;
            if (!((valid[i >> 6] >> (i & 63)) & 1) || !dict || cubit_dict_entry(dict, (uint64_t)src[i], &p, &len) != CUBIT_OK) {
                d[i] = string_t();
                continue;
            }
            d[i] = StringVector::AddString(dst, p, len);
        }
        break;
    }
    case PhysicalType::INT128:
    case PhysicalType::UINT128: {  // codes → order keys → the 128-bit values
        const bool is_signed = dst.GetType().InternalType() == PhysicalType::INT128;
        for (idx_t i = 0; i < n; i++) {
            const char *p = nullptr;
            uint64_t len = 0, lower = 0, upper = 0;
            if (((valid[i >> 6] >> (i & 63)) & 1) && dict && cubit_dict_entry(dict, (uint64_t)src[i], &p, &len) == CUBIT_OK &&
                len == 16) {
                cubit_value128(is_signed ? CUBIT_TYPE_INT128 : CUBIT_TYPE_UINT128, (const unsigned char *)p, &lower,
                               &upper);
            }
            if (is_signed) {
                FlatVector::GetData<hugeint_t>(dst)[i] = hugeint_t((int64_t)upper, lower);
            } else {
                FlatVector::GetData<uhugeint_t>(dst)[i] = uhugeint_t(upper, lower);
            }
        }
        break;
    }
    case PhysicalType::BOOL:
        Narrow<bool>(src, dst, n);
        break;
    case PhysicalType::UINT8:
        Narrow<uint8_t>(src, dst, n);
        break;
    case PhysicalType::UINT16:
        Narrow<uint16_t>(src, dst, n);
        break;
    case PhysicalType::UINT32:
        Narrow<uint32_t>(src, dst, n);
        break;
    case PhysicalType::INT8: {
        auto d = FlatVector::GetData<int8_t>(dst);
        for (idx_t i = 0; i < n; i++) {
            d[i] = (int8_t)src[i];
        }
        break;
    }
    case PhysicalType::INT16: {
        auto d = FlatVector::GetData<int16_t>(dst);
        for (idx_t i = 0; i < n; i++) {
            d[i] = (int16_t)src[i];
        }
        break;
    }
    case PhysicalType::INT32: {
        auto d = FlatVector::GetData<int32_t>(dst);
        for (idx_t i = 0; i < n; i++) {
            d[i] = (int32_t)src[i];
        }
        break;
    }
    case PhysicalType::FLOAT: {  // the 32-bit patterns back into the floats (DOUBLE: the 8-byte copy below)
        auto d = FlatVector::GetData<float>(dst);
        for (idx_t i = 0; i < n; i++) {
            const uint32_t u = (uint32_t)src[i];
            memcpy(d + i, &u, 4);
        }
        break;
    }
    default:
        memcpy(FlatVector::GetData<int64_t>(dst), src, n * sizeof(int64_t));
        break;
    }
}

// the chunk's mask for one column (FlatVector::Validity, validity_mask.hpp:22,164-168): left
// all-valid unless a row is NULL, as a vector read from a segment without NULLs
static void CopyValidity(const uint64_t *words, Vector &dst, idx_t n) {
    const idx_t nw = (n + 63) / 64;
    bool all = true;
    for (idx_t j = 0; j < nw; j++) {
        all = all && words[j] == ~0ull;
    }
    auto &mask = FlatVector::Validity(dst);
    if (all) {
        mask.Reset();  // no buffer = every row valid, whatever an earlier chunk left (validity_mask.hpp:139-143)
        return;
    }
    mask.Initialize(STANDARD_VECTOR_SIZE);
    auto data = mask.GetData();
    for (idx_t j = 0; j < nw; j++) {
        data[j] = words[j];
    }
}

static void CubitScanFunc(ClientContext &context, TableFunctionInput &data, DataChunk &output) {
    auto &g = data.global_state->Cast<CubitGlobalState>();
    auto &l = data.local_state->Cast<CubitLocalState>();
    if (g.seq_global) {
        auto &bind = data.bind_data->Cast<CubitBindData>();
        TableFunctionInput seq_data(bind.seq_bind.get(), l.seq_local.get(), g.seq_global.get());
        bind.seq.function(context, seq_data, output);
        return;
    }
    uint64_t n = 0;
    if (cubit_scan_function_validity(g.scan, l.local, l.ptrs.data(), l.vptrs.data(), &n) != CUBIT_OK) {
        throw InternalException("cubit_scan: %s", cubit_scan_last_error());
    }
    for (idx_t c = 0; c < output.ColumnCount(); c++) {
        CopyOut(l.ptrs[c], output.data[c], n, l.vptrs[c], g.out_dicts[c]);
        CopyValidity(l.vptrs[c], output.data[c], n);
    }
    output.SetCardinality(n);  // 0 rows = finished (PhysicalTableScan::GetData)
}

static idx_t CubitBatchIndex(ClientContext &context, const FunctionData *bind_data,
                             LocalTableFunctionState *local_state, GlobalTableFunctionState *global_state) {
    auto &g = global_state->Cast<CubitGlobalState>();
    auto &l = local_state->Cast<CubitLocalState>();
    if (g.seq_global) {
        auto &bind = bind_data->Cast<CubitBindData>();
        return bind.seq.get_batch_index(context, bind.seq_bind.get(), l.seq_local.get(), g.seq_global.get());
    }
    uint64_t b = 0;
    cubit_scan_batch_index(g.scan, l.local, &b);
    return b;
}

static double CubitProgress(ClientContext &context, const FunctionData *bind_data,
                            const GlobalTableFunctionState *global_state) {
    auto &g = global_state->Cast<CubitGlobalState>();
    if (g.seq_global) {
        auto &bind = bind_data->Cast<CubitBindData>();
        return bind.seq.table_scan_progress ? bind.seq.table_scan_progress(context, bind.seq_bind.get(), g.seq_global.get())
                                            : -1;
    }
    double p = 0;
    cubit_scan_progress(g.scan, &p);
    return p;
}

// TableScanCardinality (table_scan.cpp:201-208) over the attached partition
static unique_ptr<NodeStatistics> CubitCardinality(ClientContext &context, const FunctionData *bind_data) {
    auto &bind = bind_data->Cast<CubitBindData>();
    uint64_t estimated = 0, max = 0;
    auto set = bind.attached.Current();  // held for the call: a re-attach may swap it meanwhile
    if (!set) {
        return nullptr;
    }
    auto &parts = set->parts;
    if (cubit_scan_cardinality_multi(parts.data(), (uint32_t)parts.size(), &estimated, &max) != CUBIT_OK) {
        return nullptr;
    }
    return make_uniq<NodeStatistics>(estimated, max);
}

// TableScanStatistics (table_scan.cpp:108-117): the column's min / max / NULL flags from the
// GPU partition; none for the row id, as the reference
static unique_ptr<BaseStatistics> CubitStatistics(ClientContext &context, const FunctionData *bind_data,
                                                  column_t column_id) {
    auto &bind = bind_data->Cast<CubitBindData>();
    if (column_id == COLUMN_IDENTIFIER_ROW_ID) {
        return nullptr;
    }
    int64_t lo = 0, hi = 0;
    int has_null = 0, has_no_null = 0;
    auto set = bind.attached.Current();
    if (!set) {
        return nullptr;
    }
    auto &parts = set->parts;
    if (cubit_scan_statistics_multi(parts.data(), (uint32_t)parts.size(), column_id, &lo, &hi, &has_null,
                                    &has_no_null) != CUBIT_OK) {
        return nullptr;
    }
    const auto &type = bind.table.GetColumn(LogicalIndex(column_id)).GetType();
    auto stats = BaseStatistics::CreateEmpty(type);
    if (type.InternalType() == PhysicalType::VARCHAR) {
        // the codes' min / max are ranks: their dictionary entries are the column's min / max
        // strings (StringStats keeps their prefixes). Length and unicode are not tracked here:
        // left unknown / possible, as conservative statistics must be.
        auto d = set->dicts.find(column_id);
        if (d == set->dicts.end()) {
            return nullptr;
        }
        if (has_no_null) {
            for (int64_t code : {lo, hi}) {
                const char *p = nullptr;
                uint64_t len = 0;
                if (cubit_dict_entry(d->second, (uint64_t)code, &p, &len) != CUBIT_OK) {
                    return nullptr;
                }
                StringStats::Update(stats, string_t(p, (uint32_t)len));
            }
            StringStats::ResetMaxStringLength(stats);
            StringStats::SetContainsUnicode(stats);
            stats.SetHasNoNull();
        }
        if (has_null) {
            stats.SetHasNull();
        }
        return stats.ToUnique();
    }
    if (has_no_null) {
        const auto phys = type.InternalType();
        if (phys == PhysicalType::INT128 || phys == PhysicalType::UINT128) {
            // the codes' min / max are the values' (codes are ranks): their entries, decoded
            auto d = set->dicts.find(column_id);
            const char *p[2] = {nullptr, nullptr};
            uint64_t len[2] = {0, 0}, lower[2], upper[2];
            if (d == set->dicts.end() || cubit_dict_entry(d->second, (uint64_t)lo, &p[0], &len[0]) != CUBIT_OK ||
                cubit_dict_entry(d->second, (uint64_t)hi, &p[1], &len[1]) != CUBIT_OK || len[0] != 16 || len[1] != 16) {
                return nullptr;
            }
            const int kt = phys == PhysicalType::INT128 ? CUBIT_TYPE_INT128 : CUBIT_TYPE_UINT128;
            for (int k = 0; k < 2; k++) {
                cubit_value128(kt, (const unsigned char *)p[k], &lower[k], &upper[k]);
            }
            // as the column's logical type: HUGEINT, UHUGEINT, DECIMAL(19..38) or UUID storage values
            auto value_of = [&](int k) {
                const hugeint_t h((int64_t)upper[k], lower[k]);
                if (phys == PhysicalType::UINT128) return Value::UHUGEINT(uhugeint_t(upper[k], lower[k]));
                if (type.id() == LogicalTypeId::DECIMAL)
                    return Value::DECIMAL(h, DecimalType::GetWidth(type), DecimalType::GetScale(type));
                if (type.id() == LogicalTypeId::UUID) return Value::UUID(h);
                return Value::HUGEINT(h);
            };
            NumericStats::SetMin(stats, value_of(0));
            NumericStats::SetMax(stats, value_of(1));
        } else if (phys == PhysicalType::FLOAT || phys == PhysicalType::DOUBLE) {  // bit patterns
            float f[2];
            double d[2];
            const uint32_t u[2] = {(uint32_t)lo, (uint32_t)hi};
            memcpy(f, u, sizeof(f));
            memcpy(&d[0], &lo, 8);
            memcpy(&d[1], &hi, 8);
            NumericStats::SetMin(stats, phys == PhysicalType::FLOAT ? Value::FLOAT(f[0]) : Value::DOUBLE(d[0]));
            NumericStats::SetMax(stats, phys == PhysicalType::FLOAT ? Value::FLOAT(f[1]) : Value::DOUBLE(d[1]));
        } else if (phys == PhysicalType::UINT64) {
            NumericStats::SetMin(stats, Value::UBIGINT((uint64_t)lo));
            NumericStats::SetMax(stats, Value::UBIGINT((uint64_t)hi));
        } else {
            NumericStats::SetMin(stats, Value::Numeric(type, lo));  // DECIMAL: lo is the storage value
            NumericStats::SetMax(stats, Value::Numeric(type, hi));
        }
        stats.SetHasNoNull();
    }
    if (has_null) {
        stats.SetHasNull();
    }
    return stats.ToUnique();
}

TableFunction GetCubitScanFunction() {
    TableFunction f("cubit_scan", {}, CubitScanFunc);
    f.init_global = CubitInitGlobal;
    f.init_local = CubitInitLocal;
    f.get_batch_index = CubitBatchIndex;
    f.table_scan_progress = CubitProgress;
    f.cardinality = CubitCardinality;
    f.statistics = CubitStatistics;
    f.projection_pushdown = true;  // as seq_scan (table_scan.cpp:436-438)
    f.filter_pushdown = true;
    f.filter_prune = true;
    return f;
}

// ------------------------------------------------------------------ optimizer swap

// The GPU partition holds exactly what the scanning transaction's seq_scan would read:
//  * the transaction has changed nothing (DuckTransaction::ChangesMade, duck_transaction.hpp:59):
//    its own deletes of persistent rows go to the row groups' version info
//    (DataTable::Delete → RowGroupCollection::Delete, data_table.cpp:1181-1189) and its appends
//    to its LocalStorage, which DataTable::Scan reads after the persistent rows
//    (data_table.cpp:277-287, local_storage.cpp:326-341) — none of that is on the GPU;
//  * no writer of the table is outstanding (CubitAttached::writers: recorded when its statement
//    ends or when it is planned) and every committed append is synced;
//  * the transaction's snapshot includes the one the partition was read in.
static bool PartitionCurrentLocked(ClientContext &context, DuckTableEntry &table, CubitAttached &attached) {
    auto &tx = DuckTransaction::Get(context, table.catalog);
    auto &storage = table.GetStorage();
    if (tx.ChangesMade() || LocalStorage::Get(tx).Find(storage)) {
        return false;
    }
    return attached.Attached() && attached.writers.empty() && storage.GetTotalRows() == attached.gpu_rows &&
           tx.start_time >= attached.sync_start;
}

static bool CubitPartitionIsCurrent(ClientContext &context, DuckTableEntry &table, CubitAttached &attached) {
    lock_guard<mutex> g(attached.lock);
    return PartitionCurrentLocked(context, table, attached);
}

// DELETE / UPDATE / INSERT … ON CONFLICT DO UPDATE planned on an attached table: remember the
// writing transaction (see CubitAttached). Returns whether the plan writes any table.
static bool NoteWriters(ClientContext &context, LogicalOperator &op) {
    bool writes = false;
    for (auto &child : op.children) {
        writes |= NoteWriters(context, *child);
    }
    optional_ptr<TableCatalogEntry> table;
    bool changes_values = false;
    switch (op.type) {
    case LogicalOperatorType::LOGICAL_DELETE:
        table = &op.Cast<LogicalDelete>().table;
        break;
    case LogicalOperatorType::LOGICAL_UPDATE: {
        auto &u = op.Cast<LogicalUpdate>();
        table = &u.table;
        changes_values = true;  // refined below against the attached columns
        break;
    }
    case LogicalOperatorType::LOGICAL_INSERT: {
        auto &ins = op.Cast<LogicalInsert>();
        writes = true;  // appends reach the partition through the row count
        if (ins.action_type == OnConflictAction::UPDATE || ins.action_type == OnConflictAction::REPLACE) {
            table = &ins.table;
            changes_values = true;
        }
        break;
    }
    default:
        return writes;
    }
    writes = true;
    if (!table) {
        return writes;
    }
    auto attached = CubitRegistry::Find(*table);
    if (!attached) {
        return writes;
    }
    auto &tx = DuckTransaction::Get(context, table->catalog);
    lock_guard<mutex> g(attached->lock);
    if (changes_values && op.type == LogicalOperatorType::LOGICAL_UPDATE) {
        changes_values = false;
        for (auto &c : op.Cast<LogicalUpdate>().columns) {
            changes_values |= attached->columns.count(c.index) > 0;
        }
    }
    auto &w = attached->writers[tx.transaction_id];
    w = w || changes_values;
    return writes;
}

static void SwapScans(ClientContext &context, unique_ptr<LogicalOperator> &plan) {
    for (auto &child : plan->children) {
        SwapScans(context, child);
    }
    if (plan->type != LogicalOperatorType::LOGICAL_GET) {
        return;
    }
    auto &get = plan->Cast<LogicalGet>();
    if (get.function.name != "seq_scan" || get.table_filters.filters.empty()) {
        return;
    }
    auto table = get.GetTable();
    if (!table || !table->IsDuckTable()) {
        return;
    }
    auto attached = CubitRegistry::Find(*table);
    if (!attached) {
        return;
    }
    if (!CubitPartitionIsCurrent(context, table->Cast<DuckTableEntry>(), *attached)) {
        return;  // seq_scan reads what the GPU partition does not hold
    }
    for (auto c : get.column_ids) {
        if (c != COLUMN_IDENTIFIER_ROW_ID && !attached->columns.count(c)) {
            return;  // a scanned column is not on the GPU
        }
    }
    for (auto &kv : get.table_filters.filters) {
        if (!Supported(*kv.second)) {
            return;
        }
    }
    auto seq = get.function;
    auto seq_bind = std::move(get.bind_data);
    get.function = GetCubitScanFunction();
    get.bind_data = make_uniq<CubitBindData>(table->Cast<DuckTableEntry>(), *attached, std::move(seq), std::move(seq_bind));
}

// A writer recorded when its statement ends, whatever planned it: ClientContextState::QueryEnd
// (client_context_state.hpp:38-44) runs in ClientContext::EndQueryInternal before an autocommit
// commits (client_context.cpp:205-228), and for an explicit transaction after each of its
// statements, so a DELETE or UPDATE is known before any other transaction can see it — prepared
// statements run again with EXECUTE, statements planned with enable_optimizer off and writes of
// transactions that began before the attach included. The undo buffer says whether the
// transaction deleted or updated rows (UndoBufferProperties, undo_buffer.hpp:19-25) but not in
// which table, so the writer counts against every attached table of the database it modified
// (MetaTransaction::ModifiedDatabase, meta_transaction.hpp:59-62). Appends need no record: they
// reach the partition through the row count.
class CubitContextState : public ClientContextState {
public:
    void QueryEnd(ClientContext &context) override {
        if (!context.transaction.HasActiveTransaction()) {
            return;
        }
        auto &meta = context.ActiveTransaction();
        auto db = meta.ModifiedDatabase();
        if (!db || db->IsSystem() || db->IsTemporary()) {
            return;
        }
        auto tr = meta.TryGetTransaction(*db);
        if (!tr || !tr->IsDuckTransaction()) {
            return;
        }
        auto &tx = tr->Cast<DuckTransaction>();
        if (noted_db == db.get() && noted_id == tx.transaction_id && noted_values) {
            return;  // recorded with values changed: nothing the undo buffer says can add to it
        }
        if (!tx.ChangesMade()) {
            return;
        }
        auto props = tx.GetUndoProperties();  // walks the undo buffer: once per statement at most
        if (!props.has_deletes && !props.has_updates) {
            return;
        }
        noted_db = db.get();
        noted_id = tx.transaction_id;
        noted_values = props.has_updates;
        CubitRegistry::NoteDirty(*db, tx.transaction_id, props.has_updates,
                                 DuckTransactionManager::Get(*db).LowestActiveId());
        for (auto &kv : CubitRegistry::InDatabase(*db)) {
            lock_guard<mutex> g(kv.second->lock);
            auto &w = kv.second->writers[tx.transaction_id];
            w = w || props.has_updates;
        }
    }

private:
    const AttachedDatabase *noted_db = nullptr;  // the writer this connection recorded last
    transaction_t noted_id = 0;
    bool noted_values = false;
};

static void RegisterContextState(ClientContext &context) {
    if (!context.registered_state.count("cubit")) {
        context.registered_state["cubit"] = make_shared_ptr<CubitContextState>();
    }
}

// ExtensionCallback::OnConnectionOpened (extension_callback.hpp:22): every connection opened
// after the load carries the state (cubit_init registers it on the ones already open)
class CubitExtensionCallback : public ExtensionCallback {
public:
    void OnConnectionOpened(ClientContext &context) override {
        RegisterContextState(context);
    }
};

// OptimizerExtension::optimize_function (optimizer_extension.hpp:31-41), run after the built-in
// optimizers (optimizer.cpp:222-227). Scans inside a plan that writes keep seq_scan: the rows a
// DELETE / UPDATE reads are the rows it changes.
static void CubitOptimize(OptimizerExtensionInput &input, unique_ptr<LogicalOperator> &plan) {
    RegisterContextState(input.context);
    if (NoteWriters(input.context, *plan)) {
        return;
    }
    SwapScans(input.context, plan);
}

// ------------------------------------------------------------------ attach / sync

// The attached columns of one snapshot, in row-id order: values widened to int64 and DuckDB
// validity words per column, plus which row ids the snapshot holds (absent = deleted).
struct CubitSnapshot {
    uint64_t first = 0;  // row id of element 0
    uint64_t rows = 0;   // first … first+rows-1
    vector<vector<int64_t>> values;
    vector<vector<uint64_t>> validity;
    vector<vector<string>> strings;  // a dictionary column's values: strings, 128-bit order keys (`values` stay 0)
    vector<bool> present;
};

// One query over the table's row ids ≥ first in the connection's open transaction. The
// snapshot covers at least row ids [first, total_rows): rows the transaction does not see —
// deleted by a commit before it began — are absent (present = false), the tail included, so the
// partition's row count stays DataTable::GetTotalRows' (total_rows is read before the
// transaction begins: every row it counts was committed before the snapshot, since appends reach
// the row groups inside the commit, under the lock StartTransaction takes).
static void ReadRows(Connection &con, const string &table_name, DuckTableEntry &entry, const vector<column_t> &cols,
                     uint64_t first, uint64_t total_rows, CubitSnapshot &snap) {
    string sql = "SELECT rowid";
    for (auto c : cols) {
        sql += ", " + KeywordHelper::WriteOptionallyQuoted(entry.GetColumn(LogicalIndex(c)).Name());
    }
    sql += " FROM " + KeywordHelper::WriteOptionallyQuoted(table_name);
    if (first) {
        sql += " WHERE rowid >= " + to_string(first);
    }
    sql += " ORDER BY rowid";
    auto res = con.Query(sql);
    if (res->HasError()) {
        res->ThrowError();
    }
    snap.first = first;
    snap.rows = 0;
    snap.values.assign(cols.size(), {});
    snap.validity.assign(cols.size(), {});
    snap.strings.assign(cols.size(), {});
    snap.present.clear();
    vector<bool> is_str(cols.size());
    for (idx_t c = 0; c < cols.size(); c++) {
        is_str[c] = DictPhysical(entry.GetColumn(LogicalIndex(cols[c])).GetType().InternalType());
    }
    while (auto chunk = res->Fetch()) {
        chunk->Flatten();
        auto ids = FlatVector::GetData<int64_t>(chunk->data[0]);
        for (idx_t i = 0; i < chunk->size(); i++) {
            const uint64_t r = (uint64_t)ids[i] - first;
            if (r >= snap.rows) {
                snap.rows = r + 1;
                snap.present.resize(snap.rows, false);
                for (idx_t c = 0; c < cols.size(); c++) {
                    snap.values[c].resize(snap.rows, 0);
                    snap.validity[c].resize((snap.rows + 63) / 64, 0);
                    if (is_str[c]) {
                        snap.strings[c].resize(snap.rows);
                    }
                }
            }
            snap.present[r] = true;
            for (idx_t c = 0; c < cols.size(); c++) {
                auto &vec = chunk->data[c + 1];
                if (!FlatVector::Validity(vec).RowIsValid(i)) {
                    continue;
                }
                snap.validity[c][r >> 6] |= 1ull << (r & 63);
                const auto phys = vec.GetType().InternalType();
                if (phys == PhysicalType::INT128) {
                    const auto h = FlatVector::GetData<hugeint_t>(vec)[i];
                    snap.strings[c][r] = Key128(phys, h.lower, (uint64_t)h.upper);
                } else if (phys == PhysicalType::UINT128) {
                    const auto u = FlatVector::GetData<uhugeint_t>(vec)[i];
                    snap.strings[c][r] = Key128(phys, u.lower, u.upper);
                } else if (is_str[c]) {
                    snap.strings[c][r] = FlatVector::GetData<string_t>(vec)[i].GetString();
                } else {
                    snap.values[c][r] = PhysicalAsInt64(vec, i);
                }
            }
        }
    }
    if (total_rows > first && snap.rows < total_rows - first) {  // deleted tail rows
        snap.rows = total_rows - first;
        snap.present.resize(snap.rows, false);
        for (idx_t c = 0; c < cols.size(); c++) {
            snap.values[c].resize(snap.rows, 0);
            snap.validity[c].resize((snap.rows + 63) / 64, 0);
            if (is_str[c]) {
                snap.strings[c].resize(snap.rows);
            }
        }
    }
}

// Strings as the bytes + offsets layout cubit_dict_create / cubit_dict_encode read (string i =
// bytes[offsets[i], offsets[i+1]); an invalid row contributes an empty slot)
static void PackStrings(const vector<string> &strs, vector<char> &bytes, vector<uint64_t> &offsets) {
    bytes.clear();
    offsets.assign(1, 0);
    for (auto &x : strs) {
        bytes.insert(bytes.end(), x.begin(), x.end());
        offsets.push_back(bytes.size());
    }
}

// A VARCHAR column of a snapshot as its table-wide dictionary (its valid strings) and every row's
// code (NULL rows: 0); the caller owns the dictionary.
// The codes of packed strings on the GPU (cubit_dict_encode_device): the bytes, offsets and
// validity copied to `ctx`'s device, the codes copied back. False when a device step fails (the
// caller encodes on the host).
static bool EncodeOnDevice(cubit_ctx *ctx, cubit_dict *d, const vector<char> &bytes, const vector<uint64_t> &offsets,
                           const vector<uint64_t> &validity, vector<int32_t> &codes) {
    const uint64_t n = codes.size();
    void *db = nullptr, *doff = nullptr, *dv = nullptr, *dc = nullptr;
    bool ok = cubit_dev_alloc(ctx, std::max<uint64_t>(bytes.size(), 16), &db) == CUBIT_OK &&
              cubit_dev_alloc(ctx, offsets.size() * 8, &doff) == CUBIT_OK &&
              cubit_dev_alloc(ctx, std::max<uint64_t>(validity.size() * 8, 16), &dv) == CUBIT_OK &&
              cubit_dev_alloc(ctx, n * 4, &dc) == CUBIT_OK;
    ok = ok && (bytes.empty() || cubit_memcpy_h2d(ctx, db, bytes.data(), bytes.size()) == CUBIT_OK) &&
         cubit_memcpy_h2d(ctx, doff, offsets.data(), offsets.size() * 8) == CUBIT_OK &&
         cubit_memcpy_h2d(ctx, dv, validity.data(), validity.size() * 8) == CUBIT_OK &&
         cubit_dict_encode_device(ctx, d, static_cast<const char *>(db), static_cast<const uint64_t *>(doff), n,
                                  static_cast<const uint64_t *>(dv), static_cast<int32_t *>(dc)) == CUBIT_OK &&
         cubit_memcpy_d2h(ctx, codes.data(), dc, n * 4) == CUBIT_OK;
    for (void *p : {db, doff, dv, dc}) {
        if (p) {
            cubit_dev_free(ctx, p);
        }
    }
    return ok;
}

// Columns of at least this many rows are encoded on the GPU (a lane per string) when a context is
// at hand; smaller ones on the host.
static constexpr uint64_t kDeviceEncodeRows = 1 << 20;

static cubit_dict *EncodeStrings(const vector<string> &strs, const vector<uint64_t> &validity, vector<int32_t> &codes,
                                 cubit_ctx *ctx = nullptr) {
    vector<string> valid_strs;
    for (idx_t r = 0; r < strs.size(); r++) {
        if ((validity[r >> 6] >> (r & 63)) & 1) {
            valid_strs.push_back(strs[r]);
        }
    }
    vector<char> bytes;
    vector<uint64_t> offsets;
    PackStrings(valid_strs, bytes, offsets);
    cubit_dict *d = nullptr;
    Check(cubit_dict_create(bytes.data(), offsets.data(), valid_strs.size(), &d));
    PackStrings(strs, bytes, offsets);
    codes.assign(strs.size(), 0);
    if (ctx && strs.size() >= kDeviceEncodeRows && EncodeOnDevice(ctx, d, bytes, offsets, validity, codes)) {
        return d;  // every valid string is in d (it was built from them): the device encode cannot miss
    }
    const int rc = cubit_dict_encode(d, bytes.data(), offsets.data(), strs.size(), validity.data(), codes.data());
    if (rc != CUBIT_OK) {
        cubit_dict_destroy(d);
        Check(rc);
    }
    return d;
}

// Whether every valid string of a snapshot column is in `d` (an in-place append keeps the
// dictionary; a new string makes the sync rebuild with a new one)
static bool StringsInDict(cubit_dict *d, const vector<string> &strs, const vector<uint64_t> &validity) {
    for (idx_t r = 0; r < strs.size(); r++) {
        if (!((validity[r >> 6] >> (r & 63)) & 1)) {
            continue;
        }
        uint64_t lb = 0;
        int present = 0;
        if (cubit_dict_lookup(d, strs[r].data(), strs[r].size(), &lb, &present) != CUBIT_OK || !present) {
            return false;
        }
    }
    return true;
}

// Every distinct value when the column has at most this many (l_discount 11, l_quantity 50);
// a column with more gets no index unless the attach names one (l_shipdate's 2,526 distinct
// dates would take 2,526 bitvectors, 190 GB at SF100): its comparisons are built from the raw
// column at scan time (K0).
static constexpr idx_t kDefaultDistinctIndexMax = 256;

static bool FewDistinct(const vector<int64_t> &v, const vector<uint64_t> &valid) {
    unordered_set<int64_t> seen;
    for (idx_t r = 0; r < v.size(); r++) {
        if ((valid[r >> 6] >> (r & 63)) & 1) {
            seen.insert(v[r]);
            if (seen.size() > kDefaultDistinctIndexMax) {
                return false;
            }
        }
    }
    return true;
}

// The CUBIT_TYPE_* of a column's BITPACKING segments: the T DuckDB packs its physical type
// with (bitpacking.cpp:953-977, BOOL as int8_t); -1 for a type the partition does not hold.
static int SegmentType(PhysicalType t) {
    switch (t) {
    case PhysicalType::BOOL:
    case PhysicalType::INT8:
        return CUBIT_TYPE_INT8;
    case PhysicalType::INT16:
        return CUBIT_TYPE_INT16;
    case PhysicalType::INT32:
        return CUBIT_TYPE_INT32;
    case PhysicalType::INT64:
        return CUBIT_TYPE_INT64;
    case PhysicalType::UINT8:
        return CUBIT_TYPE_UINT8;
    case PhysicalType::UINT16:
        return CUBIT_TYPE_UINT16;
    case PhysicalType::UINT32:
        return CUBIT_TYPE_UINT32;
    case PhysicalType::UINT64:
        return CUBIT_TYPE_UINT64;
    default:
        return -1;
    }
}

// K5 from the database file: when every segment of column `col` is a persistent BITPACKING
// segment without in-memory updates and together they hold rows [0, n_rows) in order, the
// column is registered from those segment images as DuckDB wrote them
// (cubit_table_add_bitpacked_column: unpacked on the GPU, the packed filter and the packed
// probe reachable) and true is returned; otherwise false, and the caller uploads decoded values.
// The segments come from DataTable::GetColumnSegmentInfo (data_table.hpp:198 — the rows behind
// pragma_storage_info; ColumnData::GetColumnSegmentInfo, column_data.cpp:597-645: column_path
// "[c]" is the values, "[c, 0]" the validity, segment_start an absolute row) and are read from
// the row-data block manager (TableIOManager::GetBlockManagerForRowData, table_io_manager.hpp:30;
// BlockManager::RegisterBlock, block_manager.hpp:83; BufferManager::Pin, buffer_manager.hpp:41)
// at their block offset. A BITPACKING segment's first 8 bytes are the end of its metadata, i.e.
// its size (BitpackingCompressState::FlushSegment); an RLE segment's are the offset of its run
// lengths, which end it (RLECompressState::FlushSegment, rle.cpp:190-205); an UNCOMPRESSED one
// is its values; a CONSTANT one has no bytes, its value is its statistics' minimum. A column
// whose segments all use those codecs is taken from them (one codec: that codec's entry point;
// mixed: cubit_table_add_segment_column); any other codec (DICTIONARY, FSST, ALP, …) uses the
// snapshot's values. Deleted rows stay in the segments (visibility is the partition's delete
// list); updates make has_updates true and keep this path off.
static bool AttachSegmentColumn(DuckTableEntry &entry, column_t col, PhysicalType ptype, uint64_t n_rows,
                                cubit_table *t, const uint64_t *validity) {
    const int seg_type = SegmentType(ptype);
    if (seg_type < 0 || n_rows == 0) {
        return false;
    }
    auto &storage = entry.GetStorage();
    const string path = "[" + to_string(col) + "]";
    const string bitpacking = CompressionTypeToString(CompressionType::COMPRESSION_BITPACKING);
    const string rle = CompressionTypeToString(CompressionType::COMPRESSION_RLE);
    vector<ColumnSegmentInfo> segs;
    for (auto &info : storage.GetColumnSegmentInfo()) {
        if (info.column_id == col && info.column_path == path) {
            segs.push_back(info);
        }
    }
    std::sort(segs.begin(), segs.end(), [](const ColumnSegmentInfo &a, const ColumnSegmentInfo &b) {
        return a.segment_start < b.segment_start;
    });
    // the codecs the GPU reads: BITPACKING (unpacked), RLE (runs expanded), CONSTANT (one value,
    // from the segment's statistics), UNCOMPRESSED (the values); one codec for every segment keeps
    // its own entry point (a BITPACKING column keeps its segments for the packed filter)
    const string constant = CompressionTypeToString(CompressionType::COMPRESSION_CONSTANT);
    const string uncompressed = CompressionTypeToString(CompressionType::COMPRESSION_UNCOMPRESSED);
    const auto &ltype = entry.GetColumn(LogicalIndex(col)).GetType();
    vector<int32_t> codecs;
    vector<int64_t> constants;
    uint64_t next = 0;
    for (auto &sg : segs) {
        if (sg.has_updates || sg.segment_start != next) {
            return false;
        }
        const string &c = sg.compression_type;
        int32_t codec = -1;
        int64_t value = 0;
        if (c == bitpacking) {
            codec = CUBIT_CODEC_BITPACKING;
        } else if (c == rle) {
            codec = CUBIT_CODEC_RLE;
        } else if (c == uncompressed) {
            codec = CUBIT_CODEC_UNCOMPRESSED;
        } else if (c == constant) {
            // ConstantScanFunction reads NumericStats::Min (compression/numeric_constant.cpp); the
            // public ColumnSegmentInfo carries it as text ("[Min: v, Max: v][Has Null: …]"),
            // parsed back through the column's type (DATE, DECIMAL and BOOL print as literals)
            const string &st = sg.segment_stats;
            const auto a = st.find("[Min: "), b = st.find(", Max: ");
            if (a != 0 || b == string::npos) {
                return false;
            }
            const string lit = st.substr(6, b - 6);
            if (lit != "NULL") {  // an all-NULL segment: any value
                try {
                    value = ConstantAsInt64(Value(lit).DefaultCastAs(ltype));
                } catch (std::exception &) {
                    return false;
                }
            }
            codec = CUBIT_CODEC_CONSTANT;
        }
        if (codec < 0 || (codec != CUBIT_CODEC_CONSTANT && !sg.persistent)) {
            return false;
        }
        codecs.push_back(codec);
        constants.push_back(value);
        next += sg.segment_count;
    }
    if (next != n_rows || segs.empty()) {
        return false;
    }
    const int tsz = ptype == PhysicalType::BOOL || ptype == PhysicalType::INT8 || ptype == PhysicalType::UINT8 ? 1
                    : ptype == PhysicalType::INT16 || ptype == PhysicalType::UINT16                        ? 2
                    : ptype == PhysicalType::INT32 || ptype == PhysicalType::UINT32                        ? 4
                                                                                                           : 8;
    auto &block_manager = TableIOManager::Get(storage).GetBlockManagerForRowData();
    vector<uint8_t> bytes;
    vector<uint64_t> offsets, rows;
    for (size_t i = 0; i < segs.size(); i++) {
        auto &sg = segs[i];
        const uint64_t at = (bytes.size() + 15) / 16 * 16;
        offsets.push_back(at);
        rows.push_back(sg.segment_count);
        if (codecs[i] == CUBIT_CODEC_CONSTANT) {
            continue;  // no bytes
        }
        auto handle = block_manager.RegisterBlock(sg.block_id);
        auto pin = block_manager.buffer_manager.Pin(handle);
        const_data_ptr_t p = pin.Ptr() + sg.block_offset;
        const uint64_t room = block_manager.GetBlockSize() - sg.block_offset;
        uint64_t size = 0;
        if (codecs[i] == CUBIT_CODEC_UNCOMPRESSED) {
            size = sg.segment_count * tsz;  // the values from the segment's start (FixedSizeScan)
            if (size > room) {
                return false;
            }
        } else {
            memcpy(&size, p, sizeof(size));  // BITPACKING: the segment's size; RLE: where its run lengths start
            if (size < 8 || size > room) {
                return false;  // not a segment header
            }
        }
        if (codecs[i] == CUBIT_CODEC_RLE) {  // the run lengths end the segment: read them until they cover its rows
            uint64_t covered = 0, k = 0;
            while (covered < sg.segment_count) {
                if (size + 2 * (k + 1) > room) {
                    return false;
                }
                uint16_t len;
                memcpy(&len, p + size + 2 * k++, 2);
                covered += len;
            }
            size += 2 * k;
        }
        bytes.resize(at + size, 0);
        memcpy(bytes.data() + at, p, size);
    }
    const bool all_bp = std::all_of(codecs.begin(), codecs.end(), [](int32_t c) { return c == CUBIT_CODEC_BITPACKING; });
    const bool all_rle = std::all_of(codecs.begin(), codecs.end(), [](int32_t c) { return c == CUBIT_CODEC_RLE; });
    if (all_bp || all_rle) {
        auto add = all_rle ? cubit_table_add_rle_column : cubit_table_add_bitpacked_column;
        return add(t, (int)col, seg_type, bytes.data(), bytes.size(), offsets.data(), rows.data(), (uint32_t)segs.size(),
                   validity) == CUBIT_OK;
    }
    return cubit_table_add_segment_column(t, (int)col, seg_type, bytes.data(), bytes.size(), offsets.data(), rows.data(),
                                          codecs.data(), constants.data(), (uint32_t)segs.size(), validity) == CUBIT_OK;
}

// The column as registered against the snapshot's values on a sample (the valid rows of a
// stride over the partition, at most 4,096, read back with cubit_table_probe): a column taken
// from the segments stays so only when they agree, so a segment that no longer matches the
// snapshot (the file moved on under it) falls back to the decoded values.
static bool SampleMatches(cubit_ctx *ctx, cubit_table *t, column_t col, const vector<int64_t> &values,
                          const vector<uint64_t> &validity, uint64_t n) {
    vector<int64_t> ids;
    const uint64_t stride = std::max<uint64_t>(1, n / 4096);
    for (uint64_t r = 0; r < n && ids.size() < 4096; r += stride) {
        if ((validity[r >> 6] >> (r & 63)) & 1) {
            ids.push_back((int64_t)r);
        }
    }
    if (ids.empty()) {
        return true;
    }
    const uint64_t k = ids.size();
    void *d_ids = nullptr, *d_cnt = nullptr, *d_out = nullptr;
    vector<int64_t> got(k);
    bool ok = cubit_dev_alloc(ctx, k * 8, &d_ids) == CUBIT_OK && cubit_dev_alloc(ctx, 16, &d_cnt) == CUBIT_OK &&
              cubit_dev_alloc(ctx, k * 8, &d_out) == CUBIT_OK;
    ok = ok && cubit_memcpy_h2d(ctx, d_ids, ids.data(), k * 8) == CUBIT_OK &&
         cubit_memcpy_h2d(ctx, d_cnt, &k, 8) == CUBIT_OK &&
         cubit_table_probe(t, (int)col, nullptr, static_cast<const int64_t *>(d_ids), static_cast<const uint64_t *>(d_cnt),
                           k, static_cast<int64_t *>(d_out)) == CUBIT_OK &&
         cubit_memcpy_d2h(ctx, got.data(), d_out, k * 8) == CUBIT_OK;
    for (void *p : {d_ids, d_cnt, d_out}) {
        if (p) {
            cubit_dev_free(ctx, p);
        }
    }
    if (!ok) {
        return false;
    }
    for (uint64_t i = 0; i < k; i++) {
        if (got[i] != values[(size_t)ids[i]]) {
            return false;
        }
    }
    return true;
}

// Upload a whole snapshot as a new partition set and build its indexes: rows split into one
// contiguous range per context (boundaries on row groups of 122,880 rows = 1,920 bitvector words,
// so every partition's validity words are the snapshot's own), partition i on the contexts' i-th.
// With `entry` and one partition, a column held in persistent BITPACKING segments is registered
// from them (AttachSegmentColumn). Every partition gets the same indexes (the
// every-distinct-value default decided over the whole snapshot). The set is not visible to scans
// until the caller swaps it in.
static std::shared_ptr<CubitPartitionSet> BuildPartition(CubitAttached &attached, const CubitSnapshot &snap,
                                                         DuckTableEntry *entry) {
    auto set = std::make_shared<CubitPartitionSet>();
    set->contexts = attached.contexts;
    const auto &ctxs = set->contexts->ctxs;
    const uint64_t rg = 122880, units = (snap.rows + rg - 1) / rg;
    const uint64_t n_parts = std::max<uint64_t>(1, std::min<uint64_t>(ctxs.size(), units));
    vector<bool> few(attached.column_order.size());
    vector<vector<int32_t>> codes(attached.column_order.size());  // dictionary columns: every row's code
    for (idx_t c = 0; c < attached.column_order.size(); c++) {
        const column_t col = attached.column_order[c];
        if (DictPhysical(attached.columns[col])) {
            cubit_dict *d = EncodeStrings(snap.strings[c], snap.validity[c], codes[c], ctxs[0]);
            set->dicts[col] = d;  // the set owns it from here (its destructor frees it)
            uint64_t size = 0;
            cubit_dict_size(d, &size);
            few[c] = size <= kDefaultDistinctIndexMax;
        } else {
            few[c] = FewDistinct(snap.values[c], snap.validity[c]);
        }
    }
    for (uint64_t p = 0; p < n_parts; p++) {
        const uint64_t b = std::min(snap.rows, units * p / n_parts * rg);
        const uint64_t e = std::min(snap.rows, units * (p + 1) / n_parts * rg);
        cubit_table *t = nullptr;
        Check(cubit_table_create(ctxs[p], e - b, (int64_t)b, &t));
        set->parts.push_back(t);
        set->part_base.push_back(b);
        for (idx_t c = 0; c < attached.column_order.size(); c++) {
            const column_t col = attached.column_order[c];
            const uint64_t *valid = snap.validity[c].data() + b / 64;
            if (DictPhysical(attached.columns[col])) {
                Check(cubit_table_add_dict_column(t, (int)col, set->dicts[col], codes[c].data() + b, valid, 0));
            }
            const bool from_segments =
                !DictPhysical(attached.columns[col]) && entry && n_parts == 1 &&
                AttachSegmentColumn(*entry, col, attached.columns[col], snap.rows, t, valid) &&
                SampleMatches(ctxs[p], t, col, snap.values[c], snap.validity[c], snap.rows);
            if (!from_segments && !DictPhysical(attached.columns[col])) {
                // (re-)registering replaces a column taken from segments
                const bool wide = WidePhysical(attached.columns[col]);
                vector<int32_t> narrow;
                if (!wide) {
                    narrow.assign(snap.values[c].begin() + b, snap.values[c].begin() + e);
                }
                Check(cubit_table_add_column(t, (int)col, UploadType(attached.columns[col]),
                                             wide ? (const void *)(snap.values[c].data() + b) : (const void *)narrow.data(),
                                             valid, 0));
            }
            bool named = false;
            for (auto &ix : attached.indexes) {
                if (ix.column == col) {
                    vector<cubit_string> strs;  // a dictionary column's keys as cubit_strings
                    vector<int64_t> addrs;
                    strs.reserve(ix.str_keys.size());
                    for (auto &k : ix.str_keys) {
                        strs.push_back(cubit_string {k.data(), k.size()});
                        addrs.push_back((int64_t)(intptr_t)&strs.back());
                    }
                    const auto &keys = ix.str_keys.empty() ? ix.keys : addrs;
                    Check(cubit_table_build_index(t, (int)col, ix.encoding, keys.data(), (uint32_t)keys.size()));
                    named = true;
                }
            }
            if (!named && few[c]) {
                Check(cubit_table_build_index(t, (int)col, CUBIT_INDEX_RANGE, nullptr, 0));
            }
        }
    }
    return set;
}

// The committed deletes (row ids the snapshot lacks, visible to every snapshot the swap admits:
// start_time >= the sync's) as each partition's delete list of local rows.
static void SetDeletes(CubitPartitionSet &set, const vector<bool> &present, uint64_t rows) {
    vector<int64_t> gone;
    for (uint64_t r = 0; r < rows; r++) {
        if (r >= present.size() || !present[r]) {
            gone.push_back((int64_t)r);
        }
    }
    for (size_t p = 0; p < set.parts.size(); p++) {
        const int64_t b = (int64_t)set.part_base[p];
        const int64_t e = p + 1 < set.parts.size() ? (int64_t)set.part_base[p + 1] : (int64_t)rows;
        vector<int64_t> local;
        for (auto r : gone) {
            if (r >= b && r < e) {
                local.push_back(r - b);
            }
        }
        vector<uint64_t> ids(local.size(), 0);
        Check(cubit_table_set_deletes(set.parts[p], local.data(), ids.data(), local.size()));
    }
}

// Bring the partition to the table's committed state, reading every attached column in one
// transaction (so no commit lands between two columns). Appends only: the new row ids are
// read and appended (cubit_table_append, every index maintained in place); after an UPDATE of
// an attached column, or when row ids shrank (a checkpoint's vacuum renumbers them), every
// column is read again. Row ids the snapshot lacks are deletes, committed before it began.
static void SyncPartition(ClientContext &context, DuckTableEntry &entry, CubitAttached &attached,
                          const string &table_name, bool rebuild) {
    // the caller holds attached.sync_lock: syncs and attaches of this table run one at a time
    auto &tm = DuckTransactionManager::Get(entry.catalog.GetAttached());
    // writers that finished before the snapshot below begins are in it
    const transaction_t lowest_active = tm.LowestActiveId();
    const uint64_t total_rows = entry.GetStorage().GetTotalRows();  // before the snapshot (ReadRows)
    Connection con(*context.db);
    RegisterContextState(*con.context);
    con.BeginTransaction();
    auto &snap_tx = DuckTransaction::Get(*con.context, entry.catalog);
    const transaction_t start = snap_tx.start_time;
    vector<transaction_t> folded;
    std::shared_ptr<CubitPartitionSet> cur;
    uint64_t gpu_rows = 0;
    {
        lock_guard<mutex> g(attached.lock);
        // writers that were active before this sync and may commit after its snapshot: those
        // recorded before the table was attached too (CubitRegistry::NoteDirty)
        for (auto &d : CubitRegistry::Dirty(entry.catalog.GetAttached(), lowest_active)) {
            auto &w = attached.writers[d.first];
            w = w || d.second;
        }
        for (auto &w : attached.writers) {
            if (w.first < lowest_active) {
                folded.push_back(w.first);
                rebuild |= w.second;
            }
        }
        if (attached.Attached()) {
            cur = attached.set;
            gpu_rows = attached.gpu_rows;  // only syncs change it, and they run one at a time
        }
    }
    // the end of every path: the partition state, the writers it folded and its snapshot, in one
    // hold of the lock (and of the set's rw when it changes in place)
    auto publish = [&](std::shared_ptr<CubitPartitionSet> next, uint64_t rows) {
        lock_guard<mutex> g(attached.lock);
        attached.set = std::move(next);
        attached.gpu_rows = rows;
        for (auto w : folded) {
            attached.writers.erase(w);
        }
        attached.sync_start = start;
    };
    CubitSnapshot snap;
    vector<bool> present;  // presence of every row id of the table in this snapshot
    if (!rebuild && cur) {
        // rows appended since the partition was read, then which older rows remain
        ReadRows(con, table_name, entry, attached.column_order, gpu_rows, total_rows, snap);
        auto res = con.Query("SELECT rowid FROM " + KeywordHelper::WriteOptionallyQuoted(table_name) +
                             " WHERE rowid < " + to_string(gpu_rows));
        if (res->HasError()) {
            res->ThrowError();
        }
        present.assign(gpu_rows, false);
        while (auto chunk = res->Fetch()) {
            chunk->Flatten();
            auto ids = FlatVector::GetData<int64_t>(chunk->data[0]);
            for (idx_t i = 0; i < chunk->size(); i++) {
                present[(uint64_t)ids[i]] = true;
            }
        }
        if (snap.rows == 0 && entry.GetStorage().GetTotalRows() < gpu_rows) {
            rebuild = true;  // fewer rows than the partition: renumbered by a vacuum
        }
        for (idx_t c = 0; c < attached.column_order.size() && !rebuild; c++) {
            auto d = cur->dicts.find(attached.column_order[c]);
            if (d != cur->dicts.end() && !StringsInDict(d->second, snap.strings[c], snap.validity[c])) {
                rebuild = true;  // an appended string the dictionary lacks: a new dictionary
            }
        }
    }
    if (rebuild || !cur) {
        ReadRows(con, table_name, entry, attached.column_order, 0, total_rows, snap);
        if (snap.rows == 0) {
            con.Commit();
            throw InvalidInputException("cubit: %s has no rows to attach", table_name);
        }
        // before the snapshot's transaction ends: while it runs, a commit's updates cannot be
        // checkpointed into the segments (CanCheckpoint, duck_transaction_manager.cpp:126-131)
        // and a concurrent checkpoint does not vacuum deleted rows (:132-135); later appends show
        // as more rows than the snapshot's. Either keeps that column on decoded values, and the
        // sample check in BuildPartition backs this up.
        auto next = BuildPartition(attached, snap, &entry);
        con.Commit();
        SetDeletes(*next, snap.present, snap.rows);
        publish(std::move(next), snap.rows);  // scans still on the old set keep it until they end
        return;
    }
    con.Commit();
    // in place: appended rows continue the last partition's row range; no scan reads the tables
    // meanwhile (the set's rw, exclusive) and none is admitted before the new state is published
    lock_guard<mutex> g(attached.lock);
    std::unique_lock<std::shared_mutex> writing(cur->rw);
    if (snap.rows) {
        vector<int> cols;
        vector<const void *> data;
        vector<const uint64_t *> valid;
        vector<vector<int32_t>> narrow;
        narrow.reserve(attached.column_order.size());
        for (idx_t c = 0; c < attached.column_order.size(); c++) {
            const column_t col = attached.column_order[c];
            cols.push_back((int)col);
            if (DictPhysical(attached.columns[col])) {  // codes in the kept dictionary
                vector<char> bytes;
                vector<uint64_t> offsets;
                PackStrings(snap.strings[c], bytes, offsets);
                narrow.emplace_back(snap.rows, 0);
                Check(cubit_dict_encode(cur->dicts.at(col), bytes.data(), offsets.data(), snap.rows,
                                        snap.validity[c].data(), narrow.back().data()));
                data.push_back(narrow.back().data());
            } else if (WidePhysical(attached.columns[col])) {
                data.push_back(snap.values[c].data());
            } else {
                narrow.emplace_back(snap.values[c].begin(), snap.values[c].end());
                data.push_back(narrow.back().data());
            }
            valid.push_back(snap.validity[c].data());
        }
        Check(cubit_table_append(cur->parts.back(), snap.rows, cols.data(), data.data(), valid.data(),
                                 (uint32_t)cols.size(), 0));
        gpu_rows += snap.rows;
        present.insert(present.end(), snap.present.begin(), snap.present.end());
    }
    SetDeletes(*cur, present, gpu_rows);
    attached.gpu_rows = gpu_rows;
    for (auto w : folded) {
        attached.writers.erase(w);
    }
    attached.sync_start = start;
}

// PRAGMA cubit_sync(table)
static void CubitSync(ClientContext &context, const FunctionParameters &parameters) {
    const auto table_name = parameters.values[0].ToString();
    auto &entry = Catalog::GetEntry<TableCatalogEntry>(context, INVALID_CATALOG, DEFAULT_SCHEMA, table_name);
    auto attached = CubitRegistry::Find(entry);
    if (!attached || !attached->Current()) {
        throw InvalidInputException("cubit_sync: %s is not attached", table_name);
    }
    lock_guard<mutex> one(attached->sync_lock);
    SyncPartition(context, entry.Cast<DuckTableEntry>(), *attached, table_name, false);
}

// Index specification of cubit_attach's third argument: `column=encoding[:v1,v2,…]` items
// separated by ';' — encoding range | equality | bins, values as SQL literals of the column's
// type (dates, decimals), e.g.
//   'l_shipdate=range:1994-01-01,1995-01-01;l_shipdate=bins:1992-01-01,1993-01-01,…;l_discount=range'
static vector<CubitIndexSpec> ParseIndexSpec(DuckTableEntry &entry, const string &spec) {
    vector<CubitIndexSpec> out;
    for (auto item : StringUtil::Split(spec, ';')) {
        StringUtil::Trim(item);
        if (item.empty()) {
            continue;
        }
        const auto eq = item.find('=');
        if (eq == string::npos) {
            throw InvalidInputException("cubit_attach: index item '%s' is not column=encoding[:values]", item);
        }
        auto name = item.substr(0, eq);
        auto rest = item.substr(eq + 1);
        StringUtil::Trim(name);
        const auto colon = rest.find(':');
        auto enc = StringUtil::Lower(rest.substr(0, colon));
        StringUtil::Trim(enc);
        const auto &def = entry.GetColumn(name);
        CubitIndexSpec ix;
        ix.column = def.StorageOid();
        if (enc == "range") {
            ix.encoding = CUBIT_INDEX_RANGE;
        } else if (enc == "equality") {
            ix.encoding = CUBIT_INDEX_EQUALITY;
        } else if (enc == "bins") {
            ix.encoding = CUBIT_INDEX_BINS;
        } else {
            throw InvalidInputException("cubit_attach: unknown index encoding '%s'", enc);
        }
        const auto phys = def.GetType().InternalType();
        if (colon != string::npos && DictPhysical(phys)) {
            for (auto lit : StringUtil::Split(rest.substr(colon + 1), ',')) {
                StringUtil::Trim(lit);
                // byte order = DuckDB's string order (string_type.hpp:176-206); HUGEINT / UHUGEINT
                // literals as their order keys (byte order = the values' order)
                ix.str_keys.push_back(phys == PhysicalType::VARCHAR ? lit
                                                                    : Key128(Value(lit).DefaultCastAs(def.GetType())));
            }
            std::sort(ix.str_keys.begin(), ix.str_keys.end());
            ix.str_keys.erase(std::unique(ix.str_keys.begin(), ix.str_keys.end()), ix.str_keys.end());
        } else if (colon != string::npos) {
            for (auto lit : StringUtil::Split(rest.substr(colon + 1), ',')) {
                StringUtil::Trim(lit);
                ix.keys.push_back(ConstantAsInt64(Value(lit).DefaultCastAs(def.GetType())));
            }
            // ascending in the column's order (FLOAT / DOUBLE patterns by their comparison keys)
            const int type = UploadType(def.GetType().InternalType());
            auto key = [type](int64_t v) { return cubit_fp_key(type, v); };
            std::sort(ix.keys.begin(), ix.keys.end(), [&](int64_t a, int64_t b) { return key(a) < key(b); });
            ix.keys.erase(std::unique(ix.keys.begin(), ix.keys.end(), [&](int64_t a, int64_t b) { return key(a) == key(b); }),
                          ix.keys.end());
        }
        if (ix.encoding == CUBIT_INDEX_BINS && ix.keys.size() + ix.str_keys.size() < 2) {
            throw InvalidInputException("cubit_attach: bins on %s need at least two edges", name);
        }
        out.push_back(std::move(ix));
    }
    return out;
}

// PRAGMA cubit_attach(table, 'col,col,…' [, index_spec]): read the columns in row-id order in
// one transaction, upload them and build the named indexes (by default an every-distinct-value
// range index on the columns with few distinct values). Attaching again replaces the partition.
static void CubitAttachImpl(ClientContext &context, const string &table_name, const string &column_list,
                            const string &spec, int devices = 1) {
    auto &entry = Catalog::GetEntry<TableCatalogEntry>(context, INVALID_CATALOG, DEFAULT_SCHEMA, table_name);
    if (!entry.IsDuckTable()) {
        throw InvalidInputException("cubit_attach: %s is not a DuckDB table", table_name);
    }
    auto &duck = entry.Cast<DuckTableEntry>();
    auto &attached = CubitRegistry::Insert(entry);
    // one context per device: `devices` of them (0 = every visible device), kept across attaches
    // with the same count; a new count gets new contexts, and the old ones go with the last
    // partition set (and scan) built on them
    int visible = 1;
    Check(cubit_device_count(&visible));
    const int want = devices <= 0 ? visible : std::min(devices, visible);
    lock_guard<mutex> one(attached.sync_lock);  // through the rebuild below
    if (!attached.contexts || (int)attached.contexts->ctxs.size() != want) {
        auto fresh = std::make_shared<CubitContexts>();
        for (int d = 0; d < want; d++) {
            cubit_ctx *c = nullptr;
            Check(cubit_ctx_create(d, &c));
            fresh->ctxs.push_back(c);
        }
        attached.contexts = std::move(fresh);
    }
    {
        lock_guard<mutex> g(attached.lock);
        attached.set.reset();  // not current until the rebuild below publishes the new set
        attached.devices = devices;
        attached.columns.clear();
        attached.column_order.clear();
        for (auto name : StringUtil::Split(column_list, ',')) {
            StringUtil::Trim(name);
            const auto &def = duck.GetColumn(name);
            const auto phys = def.GetType().InternalType();
            if (!GpuPhysical(phys)) {
                throw InvalidInputException("cubit_attach: column %s is not integer-, FLOAT- or DOUBLE-backed", name);
            }
            attached.columns[def.StorageOid()] = phys;
            attached.column_order.push_back(def.StorageOid());
        }
        attached.indexes = ParseIndexSpec(duck, spec);
        for (auto &ix : attached.indexes) {
            if (!attached.columns.count(ix.column)) {
                throw InvalidInputException("cubit_attach: an index names a column that is not attached");
            }
        }
    }
    SyncPartition(context, duck, attached, table_name, true);
}

static void CubitAttach(ClientContext &context, const FunctionParameters &parameters) {
    CubitAttachImpl(context, parameters.values[0].ToString(), parameters.values[1].ToString(), "");
}

static void CubitAttachIndexed(ClientContext &context, const FunctionParameters &parameters) {
    CubitAttachImpl(context, parameters.values[0].ToString(), parameters.values[1].ToString(),
                    parameters.values[2].ToString());
}

// PRAGMA cubit_attach(table, columns, index_spec, devices): the table as one row-range partition
// per device (devices = 0: every visible device), scanned by one process through one cursor
static void CubitAttachDevices(ClientContext &context, const FunctionParameters &parameters) {
    CubitAttachImpl(context, parameters.values[0].ToString(), parameters.values[1].ToString(),
                    parameters.values[2].ToString(), parameters.values[3].GetValue<int32_t>());
}

} // namespace duckdb

extern "C" {

DUCKDB_EXTENSION_API void cubit_init(duckdb::DatabaseInstance &db) {
    using namespace duckdb;
    auto &config = DBConfig::GetConfig(db);
    OptimizerExtension ext;
    ext.optimize_function = CubitOptimize;
    config.optimizer_extensions.push_back(std::move(ext));
    PragmaFunctionSet attach("cubit_attach");
    attach.AddFunction(PragmaFunction::PragmaCall("cubit_attach", CubitAttach, {LogicalType::VARCHAR, LogicalType::VARCHAR}));
    attach.AddFunction(PragmaFunction::PragmaCall("cubit_attach", CubitAttachIndexed,
                                                  {LogicalType::VARCHAR, LogicalType::VARCHAR, LogicalType::VARCHAR}));
    attach.AddFunction(PragmaFunction::PragmaCall(
        "cubit_attach", CubitAttachDevices,
        {LogicalType::VARCHAR, LogicalType::VARCHAR, LogicalType::VARCHAR, LogicalType::INTEGER}));
    ExtensionUtil::RegisterFunction(db, attach);
    ExtensionUtil::RegisterFunction(db, PragmaFunction::PragmaCall("cubit_sync", CubitSync, {LogicalType::VARCHAR}));
    // connections opened from now on carry the writer hook from the start; those already open
    // (the one running LOAD among them) get it on their next optimized plan (CubitOptimize) —
    // registered_state belongs to its connection's thread, so it is not touched from here
    config.extension_callbacks.push_back(make_uniq<CubitExtensionCallback>());
}

DUCKDB_EXTENSION_API const char *cubit_version() {
    return duckdb::DuckDB::LibraryVersion();
}
}
