// DuckDB v1.1.2 loadable extension that routes table scans with pushed filters to the MI355X
// bitmap-indexed scan (include/cubit_gpu.h, include/cubit_scan.h).
//
// This file is the DuckDB-side binding a maintainer adds. It compiles
// against the DuckDB headers only: `make -C duckdb-cubit_amd shim-check DUCKDB_INCLUDE=…`
// runs a full semantic check (g++ -fsyntax-only) against a DuckDB v1.1.2 source tree.
// Linking it needs libduckdb, which this repository does not build.
//
//   PRAGMA cubit_attach('lineitem', 'l_shipdate,l_discount,l_quantity,l_extendedprice');
//     copies those columns to the GPU (one partition per call), builds an exact range index on
//     each, and adds a CUBIT index (CubitIndex, a BoundIndex) to the table so DuckDB hands it
//     every committed append and every index removal from then on;
//   PRAGMA cubit_sync('lineitem');
//     brings the partition to the table's committed state (uploads the appends the index
//     buffered, records committed deletes) and stamps it with the last commit.
//   The optimizer swaps seq_scan for cubit_scan when every pushed filter of the scan is
//   supported, every scanned column is attached, and the partition is exactly the state the
//   scanning transaction sees: no transaction-local rows or deletes on the table (those stay
//   on seq_scan, which scans them after the persistent rows: DataTable::Scan,
//   data_table.cpp:277-287), no commit since the stamp, and a snapshot that includes it.
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
#include "duckdb.hpp"
#include "duckdb/catalog/catalog_entry/duck_table_entry.hpp"
#include "duckdb/catalog/catalog_entry/table_catalog_entry.hpp"
#include "duckdb/function/pragma_function.hpp"
#include "duckdb/function/table_function.hpp"
#include "duckdb/main/extension_util.hpp"
#include "duckdb/optimizer/optimizer_extension.hpp"
#include "duckdb/planner/filter/conjunction_filter.hpp"
#include "duckdb/planner/filter/constant_filter.hpp"
#include "duckdb/planner/filter/null_filter.hpp"
#include "duckdb/planner/operator/logical_get.hpp"
#include "duckdb/planner/table_filter.hpp"
#include "duckdb/transaction/duck_transaction.hpp"
#include "duckdb/transaction/duck_transaction_manager.hpp"
#include "duckdb/transaction/local_storage.hpp"
#include "duckdb/execution/index/bound_index.hpp"
#include "duckdb/execution/index/index_type.hpp"
#include "duckdb/execution/index/index_type_set.hpp"
#include "duckdb/planner/expression/bound_reference_expression.hpp"
#include "duckdb/storage/data_table.hpp"
#include "duckdb/storage/table_io_manager.hpp"
#include "duckdb/storage/table/append_state.hpp"
#include "duckdb/storage/table_storage_info.hpp"

#include "cubit_gpu.h"
#include "cubit_scan.h"

#include <mutex>

namespace duckdb {

// ------------------------------------------------------------------ registry

// One GPU partition per attached table: the device context, the cubit_table and which
// storage columns it holds (with their physical width).
struct CubitAttached {
    cubit_ctx *ctx = nullptr;
    cubit_table *table = nullptr;
    unordered_map<column_t, PhysicalType> columns;
    vector<column_t> column_order;  // attached storage columns, in the CubitIndex's key order
    uint64_t gpu_rows = 0;          // rows of the GPU partition (row ids 0 … gpu_rows-1)
    // the last commit the partition reflects (DuckTransactionManager::GetLastCommit at the
    // attach / sync that produced it); the swap needs GetLastCommit() == stamp
    transaction_t stamp = 0;
    // committed appends handed to the CubitIndex since the last sync: first row id + one
    // buffer per attached column (int64 values, DuckDB validity), uploaded by cubit_sync
    struct Pending {
        row_t first = 0;
        idx_t count = 0;
        vector<vector<int64_t>> values;
        vector<vector<uint64_t>> validity;
    };
    vector<Pending> pending;
    vector<int64_t> deleted;  // row ids removed through the index (cleanup of committed deletes)
    bool index_added = false; // the table's index list holds this partition's CubitIndex
    mutex lock;               // the hooks run on DuckDB's commit / cleanup threads
};

class CubitRegistry {
public:
    static CubitAttached *Find(const TableCatalogEntry &t) {
        lock_guard<mutex> g(lock);
        auto it = map().find(&t);
        return it == map().end() ? nullptr : &it->second;
    }
    static CubitAttached &Insert(const TableCatalogEntry &t) {
        lock_guard<mutex> g(lock);
        return map()[&t];
    }

private:
    static unordered_map<const TableCatalogEntry *, CubitAttached> &map() {
        static unordered_map<const TableCatalogEntry *, CubitAttached> m;
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

// Physical types whose values the GPU compares exactly as int64: the signed integers up to
// 64 bits (DATE, TIME, TIMESTAMP*, DECIMAL(≤18) included), BOOLEAN and the unsigned integers
// up to 32 bits. UBIGINT, HUGEINT, UHUGEINT, FLOAT, DOUBLE and VARCHAR stay on seq_scan.
static bool IntegerPhysical(PhysicalType t) {
    switch (t) {
    case PhysicalType::BOOL:
    case PhysicalType::INT8:
    case PhysicalType::INT16:
    case PhysicalType::INT32:
    case PhysicalType::INT64:
    case PhysicalType::UINT8:
    case PhysicalType::UINT16:
    case PhysicalType::UINT32:
        return true;
    default:
        return false;
    }
}

// uploaded as CUBIT_TYPE_INT64 (else CUBIT_TYPE_INT32)
static bool WidePhysical(PhysicalType t) {
    return t == PhysicalType::INT64 || t == PhysicalType::UINT32;
}

static bool Supported(const TableFilter &f) {
    switch (f.filter_type) {
    case TableFilterType::CONSTANT_COMPARISON: {
        auto &c = f.Cast<ConstantFilter>();
        if (!IntegerPhysical(c.constant.type().InternalType())) {
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
    default:
        return v.GetValueUnsafe<int64_t>();  // BIGINT, DECIMAL(10..18) scaled
    }
}

// prefix-order cubit_filter_node tree of one column's TableFilter (kinds are numbered like
// TableFilterType, comparisons like the CUBIT_CMP_* of ExpressionType::COMPARE_*)
static void Emit(const TableFilter &f, int32_t column, vector<cubit_filter_node> &out) {
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
        n.constant = ConstantAsInt64(c.constant);
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
            Emit(*ch, column, out);
        }
        return;
    }
    default:
        throw InternalException("cubit: unsupported table filter reached Emit");
    }
}

// ------------------------------------------------------------------ table function

struct CubitBindData : public TableFunctionData {
    CubitBindData(DuckTableEntry &table_p, CubitAttached &attached_p) : table(table_p), attached(attached_p) {
    }
    DuckTableEntry &table;
    CubitAttached &attached;
};

struct CubitGlobalState : public GlobalTableFunctionState {
    ~CubitGlobalState() override {
        if (scan) {
            cubit_scan_destroy(scan);
        }
    }
    idx_t MaxThreads() const override {
        return max_threads;
    }
    cubit_scan *scan = nullptr;
    idx_t max_threads = 1;
    vector<LogicalType> out_types;  // output chunk column types, in output order
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
};

static unique_ptr<GlobalTableFunctionState> CubitInitGlobal(ClientContext &context, TableFunctionInitInput &input) {
    auto &bind = input.bind_data->Cast<CubitBindData>();
    vector<cubit_filter_node> nodes;
    if (input.filters && !input.filters->filters.empty()) {
        // the TableFilterSet is an AND over columns; its keys index column_ids
        nodes.push_back(cubit_filter_node {CUBIT_FILTER_AND, 0, 0, (int32_t)input.filters->filters.size(), 0});
        for (auto &kv : input.filters->filters) {
            Emit(*kv.second, (int32_t)input.column_ids[kv.first], nodes);
        }
    }
    auto &tx = DuckTransaction::Get(context, bind.table.catalog);
    cubit_txn txn {tx.start_time, tx.transaction_id};
    vector<uint64_t> cols;
    for (auto c : input.column_ids) {
        cols.push_back(c == COLUMN_IDENTIFIER_ROW_ID ? CUBIT_COLUMN_ROW_ID : (uint64_t)c);
    }
    vector<uint64_t> proj(input.projection_ids.begin(), input.projection_ids.end());
    auto g = make_uniq<CubitGlobalState>();
    if (cubit_scan_init_global(bind.attached.table, cols.data(), (uint32_t)cols.size(), proj.data(),
                               (uint32_t)proj.size(), nodes.data(), (uint32_t)nodes.size(), &txn,
                               &g->scan) != CUBIT_OK) {
        throw InvalidInputException("cubit_scan: %s", cubit_scan_last_error());
    }
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
    }
    return std::move(g);
}

static unique_ptr<LocalTableFunctionState> CubitInitLocal(ExecutionContext &context, TableFunctionInitInput &input,
                                                          GlobalTableFunctionState *global_state) {
    auto &g = global_state->Cast<CubitGlobalState>();
    auto l = make_uniq<CubitLocalState>();
    if (cubit_scan_init_local(g.scan, &l->local) != CUBIT_OK) {
        throw InternalException("cubit_scan: %s", cubit_scan_last_error());
    }
    l->staging.resize(g.out_types.size(), vector<int64_t>(STANDARD_VECTOR_SIZE));
    for (auto &s : l->staging) {
        l->ptrs.push_back(s.data());
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

// int64 staging → the column's physical type (DATE/INTEGER narrow, BIGINT/DECIMAL copy)
static void CopyOut(const int64_t *src, Vector &dst, idx_t n) {
    switch (dst.GetType().InternalType()) {
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
    default:
        memcpy(FlatVector::GetData<int64_t>(dst), src, n * sizeof(int64_t));
        break;
    }
}

static void CubitScanFunc(ClientContext &context, TableFunctionInput &data, DataChunk &output) {
    auto &g = data.global_state->Cast<CubitGlobalState>();
    auto &l = data.local_state->Cast<CubitLocalState>();
    uint64_t n = 0;
    if (cubit_scan_function(g.scan, l.local, l.ptrs.data(), &n) != CUBIT_OK) {
        throw InternalException("cubit_scan: %s", cubit_scan_last_error());
    }
    for (idx_t c = 0; c < output.ColumnCount(); c++) {
        CopyOut(l.ptrs[c], output.data[c], n);
    }
    output.SetCardinality(n);  // 0 rows = finished (PhysicalTableScan::GetData)
}

static idx_t CubitBatchIndex(ClientContext &context, const FunctionData *bind_data,
                             LocalTableFunctionState *local_state, GlobalTableFunctionState *global_state) {
    auto &g = global_state->Cast<CubitGlobalState>();
    auto &l = local_state->Cast<CubitLocalState>();
    uint64_t b = 0;
    cubit_scan_batch_index(g.scan, l.local, &b);
    return b;
}

static double CubitProgress(ClientContext &context, const FunctionData *bind_data,
                            const GlobalTableFunctionState *global_state) {
    auto &g = global_state->Cast<CubitGlobalState>();
    double p = 0;
    cubit_scan_progress(g.scan, &p);
    return p;
}

// TableScanCardinality (table_scan.cpp:201-208) over the attached partition
static unique_ptr<NodeStatistics> CubitCardinality(ClientContext &context, const FunctionData *bind_data) {
    auto &bind = bind_data->Cast<CubitBindData>();
    uint64_t estimated = 0, max = 0;
    if (cubit_scan_cardinality(bind.attached.table, &estimated, &max) != CUBIT_OK) {
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
    if (cubit_scan_statistics(bind.attached.table, column_id, &lo, &hi, &has_null, &has_no_null) != CUBIT_OK) {
        return nullptr;
    }
    const auto &type = bind.table.GetColumn(LogicalIndex(column_id)).GetType();
    auto stats = BaseStatistics::CreateEmpty(type);
    if (has_no_null) {
        NumericStats::SetMin(stats, Value::Numeric(type, lo));  // DECIMAL: lo is the storage value
        NumericStats::SetMax(stats, Value::Numeric(type, hi));
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
//  * no transaction-local storage on the table: DataTable::Scan reads the persistent row groups
//    and then the transaction's LocalStorage (data_table.cpp:277-287, local_storage.cpp:326-341),
//    and local deletes hide persistent rows; none of that is on the GPU;
//  * no commit since the partition's stamp (a DELETE reaches no index hook until cleanup, so
//    any later commit may have changed rows the partition shows) and every appended row synced;
//  * the transaction's snapshot includes the stamp (start_time > stamp: an older snapshot
//    must not see commits the partition already shows).
static bool CubitPartitionIsCurrent(ClientContext &context, DuckTableEntry &table, CubitAttached &attached) {
    auto &tx = DuckTransaction::Get(context, table.catalog);
    auto &storage = table.GetStorage();
    if (LocalStorage::Get(tx).Find(storage)) {
        return false;
    }
    auto &tm = DuckTransactionManager::Get(table.catalog.GetAttached());
    lock_guard<mutex> g(attached.lock);
    return attached.pending.empty() && tm.GetLastCommit() == attached.stamp && tx.start_time > attached.stamp &&
           storage.GetTotalRows() == attached.gpu_rows;
}

static void CubitOptimize(OptimizerExtensionInput &input, unique_ptr<LogicalOperator> &plan) {
    for (auto &child : plan->children) {
        CubitOptimize(input, child);
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
    if (!CubitPartitionIsCurrent(input.context, table->Cast<DuckTableEntry>(), *attached)) {
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
    get.function = GetCubitScanFunction();
    get.bind_data = make_uniq<CubitBindData>(table->Cast<DuckTableEntry>(), *attached);
}

// ------------------------------------------------------------------ index maintenance

// CUBIT's bitmap index as a DuckDB index type ("CUBIT"; DBConfig::GetIndexTypes, registered as
// IndexTypeSet registers ART, index_type_set.cpp:7-13). cubit_attach adds one instance to the
// table (DataTable::AddIndex), and from then on DuckDB calls it like any BoundIndex
// (bound_index.hpp:67-126):
//   Append  ← DataTable::AppendToIndexes (data_table.cpp:1000-1040), once per committed chunk
//             (LocalStorage::Flush at commit), and for the insert half of an UPDATE of an
//             attached column (an UPDATE of an indexed column runs as delete + insert,
//             table_catalog_entry.cpp:288-308). The chunk's attached columns are buffered; the
//             next cubit_sync uploads them with cubit_table_append (every bitmap index on the
//             GPU maintained in place) — until then the swap is refused.
//   Delete  ← DataTable::RemoveFromIndexes: the revert of a failed append (data_table.cpp:
//             1032-1037) and the cleanup of committed deletes (cleanup_state.cpp:93); the rows
//             become deletes of the partition (cubit_table_set_deletes at the next sync).
//   Insert  ← an index build over existing rows (not used: cubit_attach uploads them itself).
// Constraint checks pass (CUBIT is not a constraint index), and the index holds no DuckDB-side
// storage (GetStorageInfo: nothing to persist; the GPU index is rebuilt by cubit_attach).
class CubitIndex : public BoundIndex {
public:
    static constexpr const char *TYPE_NAME = "CUBIT";

    CubitIndex(const string &name, const vector<column_t> &column_ids, TableIOManager &io,
               const vector<unique_ptr<Expression>> &exprs, AttachedDatabase &db, CubitAttached *attached_p)
        : BoundIndex(name, TYPE_NAME, IndexConstraintType::NONE, column_ids, io, exprs, db), attached(attached_p) {
    }

    // IndexType::create_instance: a CUBIT index bound to the table's attached partition
    static unique_ptr<BoundIndex> Create(CreateIndexInput &input) {
        return make_uniq<CubitIndex>(input.name, input.column_ids, input.table_io_manager, input.unbound_expressions,
                                     input.db, nullptr);
    }

    ErrorData Append(IndexLock &, DataChunk &entries, Vector &row_identifiers) override {
        if (!attached || entries.size() == 0) {
            return ErrorData();
        }
        DataChunk keys;
        keys.Initialize(Allocator::DefaultAllocator(), logical_types);
        ExecuteExpressions(entries, keys);  // the attached columns, in key order
        keys.Flatten();
        row_identifiers.Flatten(entries.size());
        auto rows = FlatVector::GetData<row_t>(row_identifiers);
        CubitAttached::Pending p;
        p.first = rows[0];
        p.count = entries.size();
        for (idx_t c = 0; c < keys.ColumnCount(); c++) {
            vector<int64_t> v(p.count, 0);
            vector<uint64_t> valid((p.count + 63) / 64, 0);
            auto &vec = keys.data[c];
            auto &mask = FlatVector::Validity(vec);
            for (idx_t i = 0; i < p.count; i++) {
                if (!mask.RowIsValid(i)) {
                    continue;
                }
                valid[i >> 6] |= 1ull << (i & 63);
                v[i] = PhysicalAsInt64(vec, i);
            }
            p.values.push_back(std::move(v));
            p.validity.push_back(std::move(valid));
        }
        lock_guard<mutex> g(attached->lock);
        attached->pending.push_back(std::move(p));
        return ErrorData();
    }

    void Delete(IndexLock &, DataChunk &entries, Vector &row_identifiers) override {
        if (!attached) {
            return;
        }
        row_identifiers.Flatten(entries.size());
        auto rows = FlatVector::GetData<row_t>(row_identifiers);
        lock_guard<mutex> g(attached->lock);
        for (idx_t i = 0; i < entries.size(); i++) {
            attached->deleted.push_back(rows[i]);
        }
    }

    ErrorData Insert(IndexLock &state, DataChunk &input, Vector &row_identifiers) override {
        return Append(state, input, row_identifiers);
    }
    void VerifyAppend(DataChunk &) override {
    }
    void VerifyAppend(DataChunk &, ConflictManager &) override {
    }
    void CheckConstraintsForChunk(DataChunk &, ConflictManager &) override {
    }
    void CommitDrop(IndexLock &) override {
        attached = nullptr;
    }
    bool MergeIndexes(IndexLock &, BoundIndex &) override {
        return true;  // local (transaction) indexes are never CUBIT: nothing to merge
    }
    void Vacuum(IndexLock &) override {
    }
    idx_t GetInMemorySize(IndexLock &) override {
        return 0;  // the bitvectors live in GPU memory (cubit_table_index_info)
    }
    string VerifyAndToString(IndexLock &, const bool) override {
        return "CUBIT index (GPU partition)";
    }
    string GetConstraintViolationMessage(VerifyExistenceType, idx_t, DataChunk &) override {
        return "CUBIT indexes enforce no constraint";
    }
    IndexStorageInfo GetStorageInfo(const bool) override {
        IndexStorageInfo info(name);
        return info;
    }

    CubitAttached *attached;
};

// Upload what the CubitIndex buffered and record the committed deletes, under a snapshot that
// no commit overtakes (stamp taken before the row-id scan, checked unchanged after it).
static void SyncPartition(ClientContext &context, TableCatalogEntry &entry, CubitAttached &attached,
                          const string &table_name) {
    auto &tm = DuckTransactionManager::Get(entry.catalog.GetAttached());
    for (int attempt = 0; attempt < 3; attempt++) {
        const transaction_t t0 = tm.GetLastCommit();
        Connection con(*context.db);
        auto res = con.Query("SELECT rowid FROM " + KeywordHelper::WriteOptionallyQuoted(table_name));
        if (res->HasError()) {
            res->ThrowError();
        }
        vector<bool> present;
        while (auto chunk = res->Fetch()) {
            chunk->Flatten();
            auto rows = FlatVector::GetData<int64_t>(chunk->data[0]);
            for (idx_t i = 0; i < chunk->size(); i++) {
                const uint64_t r = (uint64_t)rows[i];
                if (r >= present.size()) {
                    present.resize(r + 1, false);
                }
                present[r] = true;
            }
        }
        if (tm.GetLastCommit() != t0) {
            continue;  // a commit landed during the scan: take a new snapshot
        }
        lock_guard<mutex> g(attached.lock);
        // appends in row order, each continuing the partition
        std::sort(attached.pending.begin(), attached.pending.end(),
                  [](const CubitAttached::Pending &a, const CubitAttached::Pending &b) { return a.first < b.first; });
        for (auto &p : attached.pending) {
            if ((uint64_t)p.first != attached.gpu_rows) {
                throw InvalidInputException("cubit_sync: appended rows start at %lld, the partition holds %llu rows; "
                                            "run cubit_attach again",
                                            (long long)p.first, (unsigned long long)attached.gpu_rows);
            }
            vector<int> cols;
            vector<const void *> data;
            vector<const uint64_t *> valid;
            vector<vector<int32_t>> narrow;
            narrow.reserve(attached.column_order.size());
            for (idx_t c = 0; c < attached.column_order.size(); c++) {
                const column_t col = attached.column_order[c];
                cols.push_back((int)col);
                if (WidePhysical(attached.columns[col])) {
                    data.push_back(p.values[c].data());
                } else {
                    narrow.emplace_back(p.values[c].begin(), p.values[c].end());
                    data.push_back(narrow.back().data());
                }
                valid.push_back(p.validity[c].data());
            }
            Check(cubit_table_append(attached.table, p.count, cols.data(), data.data(), valid.data(),
                                     (uint32_t)cols.size(), 0));
            attached.gpu_rows += p.count;
        }
        attached.pending.clear();
        // committed deletes: rows of the partition the snapshot does not see (and the rows the
        // index was told to remove), committed before every later snapshot
        vector<int64_t> gone;
        for (uint64_t r = 0; r < attached.gpu_rows; r++) {
            if (r >= present.size() || !present[r]) {
                gone.push_back((int64_t)r);
            }
        }
        attached.deleted.clear();
        vector<uint64_t> ids(gone.size(), 0);
        Check(cubit_table_set_deletes(attached.table, gone.data(), ids.data(), gone.size()));
        attached.stamp = t0;
        return;
    }
    throw InvalidInputException("cubit_sync: commits kept landing during the sync of %s; retry", table_name);
}

// PRAGMA cubit_sync(table)
static void CubitSync(ClientContext &context, const FunctionParameters &parameters) {
    const auto table_name = parameters.values[0].ToString();
    auto &entry = Catalog::GetEntry<TableCatalogEntry>(context, INVALID_CATALOG, DEFAULT_SCHEMA, table_name);
    auto attached = CubitRegistry::Find(entry);
    if (!attached || !attached->table) {
        throw InvalidInputException("cubit_sync: %s is not attached", table_name);
    }
    SyncPartition(context, entry, *attached, table_name);
}

// ------------------------------------------------------------------ attach

// PRAGMA cubit_attach(table, 'col,col,…'): read the columns in row-id order through a second
// connection (its own transaction), upload them and build an exact range index per column.
// Row ids missing from the scan (deleted rows) become committed deletes of the partition.
static void CubitAttach(ClientContext &context, const FunctionParameters &parameters) {
    const auto table_name = parameters.values[0].ToString();
    const auto column_list = StringUtil::Split(parameters.values[1].ToString(), ',');
    auto &entry = Catalog::GetEntry<TableCatalogEntry>(context, INVALID_CATALOG, DEFAULT_SCHEMA, table_name);
    Connection con(*context.db);
    auto max_row = con.Query("SELECT max(rowid) FROM " + KeywordHelper::WriteOptionallyQuoted(table_name));
    if (max_row->HasError()) {
        max_row->ThrowError();
    }
    const auto top = max_row->GetValue(0, 0);
    const uint64_t n_rows = top.IsNull() ? 0 : (uint64_t)top.GetValue<int64_t>() + 1;
    if (n_rows == 0) {
        throw InvalidInputException("cubit_attach: %s is empty", table_name);
    }
    auto &attached = CubitRegistry::Insert(entry);
    if (!attached.ctx) {
        Check(cubit_ctx_create(0, &attached.ctx));
    }
    if (attached.table) {
        cubit_table_destroy(attached.table);
        attached.columns.clear();
        attached.column_order.clear();
    }
    Check(cubit_table_create(attached.ctx, n_rows, 0, &attached.table));
    vector<bool> present(n_rows, false);
    for (auto name : column_list) {
        StringUtil::Trim(name);
        const auto &def = entry.GetColumn(name);
        const auto phys = def.GetType().InternalType();
        if (!IntegerPhysical(phys)) {
            throw InvalidInputException("cubit_attach: column %s is not integer-backed", name);
        }
        const bool wide = WidePhysical(phys);
        vector<int32_t> v32(wide ? 0 : n_rows, 0);
        vector<int64_t> v64(wide ? n_rows : 0, 0);
        vector<uint64_t> valid((n_rows + 63) / 64, 0);
        auto res = con.Query("SELECT rowid, " + KeywordHelper::WriteOptionallyQuoted(name) + " FROM " +
                             KeywordHelper::WriteOptionallyQuoted(table_name) + " ORDER BY rowid");
        if (res->HasError()) {
            res->ThrowError();
        }
        while (auto chunk = res->Fetch()) {
            chunk->Flatten();
            auto rows = FlatVector::GetData<int64_t>(chunk->data[0]);
            auto &vals = chunk->data[1];
            auto &mask = FlatVector::Validity(vals);
            for (idx_t i = 0; i < chunk->size(); i++) {
                const uint64_t r = (uint64_t)rows[i];
                present[r] = true;
                if (!mask.RowIsValid(i)) {
                    continue;
                }
                valid[r >> 6] |= 1ull << (r & 63);
                if (wide) {
                    v64[r] = PhysicalAsInt64(vals, i);
                } else {
                    v32[r] = (int32_t)PhysicalAsInt64(vals, i);
                }
            }
        }
        const column_t storage = def.StorageOid();
        Check(cubit_table_add_column(attached.table, (int)storage, wide ? CUBIT_TYPE_INT64 : CUBIT_TYPE_INT32,
                                     wide ? (const void *)v64.data() : (const void *)v32.data(), valid.data(), 0));
        Check(cubit_table_build_index(attached.table, (int)storage, CUBIT_INDEX_RANGE, nullptr, 0));
        attached.columns[storage] = phys;
        attached.column_order.push_back(storage);
    }
    attached.gpu_rows = n_rows;
    attached.pending.clear();
    attached.deleted.clear();
    // from here DuckDB reports every committed append and index removal to the CubitIndex; the
    // deletes and the stamp come from a snapshot no commit overtook (SyncPartition)
    auto &duck = entry.Cast<DuckTableEntry>();
    auto &storage = duck.GetStorage();
    if (!attached.index_added) {
        vector<unique_ptr<Expression>> exprs;
        vector<column_t> ids;
        for (auto c : attached.column_order) {
            exprs.push_back(make_uniq<BoundReferenceExpression>(duck.GetColumn(LogicalIndex(c)).GetType(), c));
            ids.push_back(c);
        }
        storage.AddIndex(make_uniq<CubitIndex>("cubit_" + table_name, ids, TableIOManager::Get(storage), exprs,
                                               entry.catalog.GetAttached(), &attached));
        attached.index_added = true;
    }
    SyncPartition(context, entry, attached, table_name);
}

} // namespace duckdb

extern "C" {

DUCKDB_EXTENSION_API void cubit_init(duckdb::DatabaseInstance &db) {
    auto &config = duckdb::DBConfig::GetConfig(db);
    duckdb::OptimizerExtension ext;
    ext.optimize_function = duckdb::CubitOptimize;
    config.optimizer_extensions.push_back(std::move(ext));
    duckdb::ExtensionUtil::RegisterFunction(
        db, duckdb::PragmaFunction::PragmaCall("cubit_attach", duckdb::CubitAttach,
                                               {duckdb::LogicalType::VARCHAR, duckdb::LogicalType::VARCHAR}));
    duckdb::ExtensionUtil::RegisterFunction(
        db, duckdb::PragmaFunction::PragmaCall("cubit_sync", duckdb::CubitSync, {duckdb::LogicalType::VARCHAR}));
    // the index type (index_type_set.cpp:7-13 registers ART the same way)
    duckdb::IndexType cubit_index;
    cubit_index.name = duckdb::CubitIndex::TYPE_NAME;
    cubit_index.create_instance = duckdb::CubitIndex::Create;
    config.GetIndexTypes().RegisterIndexType(cubit_index);
}

DUCKDB_EXTENSION_API const char *cubit_version() {
    return duckdb::DuckDB::LibraryVersion();
}
}
