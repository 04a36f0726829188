// cubit_scan: DuckDB TableFunction callbacks over libcubitgpu (see cubit_scan_function.hpp)
// plus the extern "C" surface of include/cubit_scan.h.
#include "cubit_scan_function.hpp"

#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

#include "../../include/cubit_scan.h"

namespace cubit {
namespace duck {

namespace {

struct ScanError : public std::runtime_error {
    int code;
    ScanError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void check(int rc, const char* what) {
    if (rc != CUBIT_OK) throw ScanError(rc, std::string(what) + ": " + cubit_last_error());
}

// Page-locked buffers outlive one scan: pinning ~100 MB costs milliseconds, more than its
// copy, and DuckDB runs init_global once per query. Freed buffers wait here (≤ 4 GiB) and a
// request takes the smallest one that fits without wasting more than half of it. Never
// destroyed (the process exit releases the pages; a static destructor could run after the
// HIP runtime's).
class PinnedPool {
  public:
    static PinnedPool& get() {
        static PinnedPool* pool = new PinnedPool();
        return *pool;
    }
    void* take(cubit_ctx* ctx, size_t bytes, size_t* got) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            auto it = free_.lower_bound(bytes);
            if (it != free_.end() && it->first <= 2 * bytes) {
                void* p = it->second;
                *got = it->first;
                cached_ -= it->first;
                free_.erase(it);
                return p;
            }
        }
        void* h = nullptr;
        check(cubit_host_alloc(ctx, bytes, &h), "cubit_host_alloc");
        *got = bytes;
        return h;
    }
    void give(void* p, size_t bytes) {
        std::lock_guard<std::mutex> lk(mu_);
        free_.emplace(bytes, p);
        cached_ += bytes;
        while (cached_ > kMaxCached && !free_.empty()) {  // drop the largest first
            auto it = std::prev(free_.end());
            cached_ -= it->first;
            cubit_host_free(nullptr, it->second);
            free_.erase(it);
        }
    }

  private:
    static constexpr size_t kMaxCached = 4ull << 30;
    std::mutex mu_;
    std::multimap<size_t, void*> free_;
    size_t cached_ = 0;
};

// Page-locked host staging (cubit_host_alloc via PinnedPool): device → host copies run at the
// link's rate instead of through a pageable bounce buffer.
struct PinnedBuffer {
    int64_t* p = nullptr;
    size_t bytes = 0;
    PinnedBuffer() = default;
    PinnedBuffer(const PinnedBuffer&) = delete;
    PinnedBuffer& operator=(const PinnedBuffer&) = delete;
    PinnedBuffer(PinnedBuffer&& o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; }
    void allocate(cubit_ctx* c, idx_t count);
    int64_t* data() { return p; }
    const int64_t* data() const { return p; }
    ~PinnedBuffer() {
        if (p) PinnedPool::get().give(p, bytes);
    }
};

// Device result of one scan, copied to host once (the GPU work is one fused launch plus one
// gather per emitted column; DataChunks are then served from host memory).
struct CubitScanGlobalState : public GlobalTableFunctionState {
    std::vector<column_t> column_ids;
    std::vector<idx_t> emit;  // positions of column_ids that reach the output
    idx_t count = 0;
    idx_t rows_per_tile = 0;
    PinnedBuffer rowids;                // tile-run order
    std::vector<PinnedBuffer> columns;  // per emitted position (row ids or probed values)
    std::vector<uint32_t> tiles;                // non-empty tiles, ascending
    std::vector<uint64_t> dir;                  // {start, length} per tile
    std::atomic<uint32_t> next{0};
    std::atomic<idx_t> emitted{0};
    idx_t MaxThreads() const override {
        const idx_t hw = std::max<unsigned>(1, std::thread::hardware_concurrency());
        return std::max<idx_t>(1, std::min<idx_t>(tiles.size(), hw));
    }
};

struct CubitScanLocalState : public LocalTableFunctionState {
    int64_t tile_slot = -1;  // index into tiles, -1 = none yet
    idx_t pos = 0;           // next row of the tile's run to emit
};

struct DeviceBuffer {
    cubit_ctx* ctx;
    void* p = nullptr;
    DeviceBuffer(cubit_ctx* c, uint64_t bytes) : ctx(c) { check(cubit_dev_alloc(c, bytes, &p), "cubit_dev_alloc"); }
    ~DeviceBuffer() {
        if (p) cubit_dev_free(ctx, p);
    }
};

void PinnedBuffer::allocate(cubit_ctx* c, idx_t count) {
    p = static_cast<int64_t*>(PinnedPool::get().take(c, std::max<idx_t>(count, 1) * sizeof(int64_t), &bytes));
}

std::unique_ptr<GlobalTableFunctionState> CubitScanInitGlobal(TableFunctionInitInput& input) {
    auto& bind = static_cast<const CubitScanBindData&>(*input.bind_data);
    auto g = std::make_unique<CubitScanGlobalState>();
    g->column_ids = input.column_ids;
    if (input.CanRemoveFilterColumns()) {
        g->emit = input.projection_ids;
    } else {
        for (idx_t i = 0; i < input.column_ids.size(); ++i) g->emit.push_back(i);
    }
    cubit_ctx* ctx = bind.ctx;
    DeviceBuffer d_cnt(ctx, 16);
    const cubit_txn* txn = bind.has_txn ? &bind.txn : nullptr;
    const auto& nodes = input.filters ? input.filters->nodes : std::vector<cubit_filter_node>{};
    // count first (one evaluate pass, no row ids), so the row-id and probe buffers are sized to
    // the result rather than to the table (4.8 GB per query at SF100 otherwise)
    check(cubit_table_scan(bind.table, nodes.empty() ? nullptr : nodes.data(), (uint32_t)nodes.size(), txn, nullptr,
                           0, static_cast<uint64_t*>(d_cnt.p), CUBIT_SCAN_COUNT_ONLY),
          "cubit_table_scan (count)");
    uint64_t want = 0;
    check(cubit_memcpy_d2h(ctx, &want, d_cnt.p, 8), "count");
    const uint64_t cap = std::max<uint64_t>(want, 1);
    DeviceBuffer d_ids(ctx, cap * 8);
    check(cubit_table_scan(bind.table, nodes.empty() ? nullptr : nodes.data(), (uint32_t)nodes.size(), txn,
                           static_cast<int64_t*>(d_ids.p), cap, static_cast<uint64_t*>(d_cnt.p), 0),
          "cubit_table_scan");
    check(cubit_ctx_check(ctx), "scan kernel");
    check(cubit_memcpy_d2h(ctx, &g->count, d_cnt.p, 8), "count");
    const uint64_t* d_dir = nullptr;
    uint32_t n_tiles = 0;
    check(cubit_ctx_last_tiles(ctx, &d_dir, &n_tiles, &g->rows_per_tile), "tiles");
    if (g->count > cap) throw ScanError(CUBIT_ERR_CAPACITY, "cubit_table_scan: count changed between the passes");
    if (g->count == 0) n_tiles = 0;  // nothing qualified: no run to hand out, whatever the directory holds
    g->dir.resize(2 * (size_t)n_tiles);
    if (n_tiles) check(cubit_memcpy_d2h(ctx, g->dir.data(), d_dir, g->dir.size() * 8), "directory");
    g->rowids.allocate(ctx, g->count);
    if (g->count) check(cubit_memcpy_d2h(ctx, g->rowids.data(), d_ids.p, g->count * 8), "row ids");
    uint64_t covered = 0;
    for (uint32_t t = 0; t < n_tiles; ++t) {
        const uint64_t start = g->dir[2 * t], len = g->dir[2 * t + 1];
        if (!len) continue;
        // every run lies inside this scan's output (a directory of another launch would not)
        if (start > g->count || len > g->count - start)
            throw ScanError(CUBIT_ERR_INVALID, "cubit_scan: tile directory does not describe this scan's output");
        covered += len;
        g->tiles.push_back(t);
    }
    if (covered != g->count)
        throw ScanError(CUBIT_ERR_INVALID, "cubit_scan: tile runs cover " + std::to_string(covered) + " of " +
                                               std::to_string(g->count) + " row ids");
    // probe every emitted storage column at the row ids (ColumnData::FilterScan semantics)
    g->columns.resize(g->emit.size());
    std::unique_ptr<DeviceBuffer> d_vals;
    for (size_t e = 0; e < g->emit.size(); ++e) {
        const column_t col = g->column_ids[g->emit[e]];
        if (col == COLUMN_IDENTIFIER_ROW_ID || g->count == 0) continue;
        if (!d_vals) d_vals = std::make_unique<DeviceBuffer>(ctx, g->count * 8);
        check(cubit_table_probe(bind.table, (int)col, txn, static_cast<int64_t*>(d_ids.p),
                                static_cast<uint64_t*>(d_cnt.p), g->count, static_cast<int64_t*>(d_vals->p)),
              "cubit_table_probe");
        g->columns[e].allocate(ctx, g->count);
        check(cubit_memcpy_d2h(ctx, g->columns[e].data(), d_vals->p, g->count * 8), "probe values");
    }
    return g;
}

std::unique_ptr<LocalTableFunctionState> CubitScanInitLocal(TableFunctionInitInput&, GlobalTableFunctionState*) {
    return std::make_unique<CubitScanLocalState>();
}

// TableScanParallelStateNext analogue: take the next non-empty tile (row_group_collection.cpp
// hands out row groups under a mutex; one atomic suffices here).
bool NextTile(CubitScanGlobalState& g, CubitScanLocalState& l) {
    const uint32_t s = g.next.fetch_add(1);
    if (s >= g.tiles.size()) {
        l.tile_slot = (int64_t)g.tiles.size();
        return false;
    }
    l.tile_slot = s;
    l.pos = 0;
    return true;
}

void CubitScanFunc(TableFunctionInput& data, DataChunk& output) {
    auto& g = static_cast<CubitScanGlobalState&>(*data.global_state);
    auto& l = static_cast<CubitScanLocalState&>(*data.local_state);
    output.Reset();
    for (;;) {
        if (l.tile_slot < 0 && !NextTile(g, l)) return;
        if ((size_t)l.tile_slot >= g.tiles.size()) return;
        const uint32_t tile = g.tiles[l.tile_slot];
        const uint64_t start = g.dir[2 * tile], len = g.dir[2 * tile + 1];
        if (l.pos < len) {
            const idx_t n = std::min<idx_t>(STANDARD_VECTOR_SIZE, len - l.pos);
            for (size_t e = 0; e < g.emit.size(); ++e) {
                const column_t col = g.column_ids[g.emit[e]];
                const int64_t* src = col == COLUMN_IDENTIFIER_ROW_ID ? g.rowids.data() : g.columns[e].data();
                std::memcpy(output.data[e].data(), src + start + l.pos, n * sizeof(int64_t));
            }
            l.pos += n;
            output.SetCardinality(n);
            g.emitted.fetch_add(n);
            return;
        }
        if (!NextTile(g, l)) return;
    }
}

idx_t CubitScanGetBatchIndex(const FunctionData*, LocalTableFunctionState* lstate, GlobalTableFunctionState* gstate) {
    auto& g = static_cast<CubitScanGlobalState&>(*gstate);
    auto& l = static_cast<CubitScanLocalState&>(*lstate);
    if (l.tile_slot < 0 || (size_t)l.tile_slot >= g.tiles.size()) return 0;
    return g.tiles[l.tile_slot];
}

double CubitScanProgress(const FunctionData*, const GlobalTableFunctionState* gstate) {
    auto& g = static_cast<const CubitScanGlobalState&>(*gstate);
    if (g.count == 0) return 100.0;
    return 100.0 * (double)g.emitted.load() / (double)g.count;
}

// TableScanCardinality (table_scan.cpp:201-208): NodeStatistics(table rows, table rows +
// transaction-local rows); transaction-local rows stay on the CPU, so both are
// the partition's rows
NodeStatistics CubitScanCardinality(const FunctionData* bind_data) {
    auto& bind = static_cast<const CubitScanBindData&>(*bind_data);
    NodeStatistics st;
    st.has_estimated_cardinality = st.has_max_cardinality = true;
    st.estimated_cardinality = st.max_cardinality = bind.n_rows;
    return st;
}

// TableScanStatistics (table_scan.cpp:108-117) → DataTable::GetStatistics: none for the row id
bool CubitScanStatistics(const FunctionData* bind_data, column_t column_id, ColumnStatistics& out) {
    auto& bind = static_cast<const CubitScanBindData&>(*bind_data);
    if (column_id == COLUMN_IDENTIFIER_ROW_ID) return false;
    int hn = 0, hv = 0;
    check(cubit_table_column_statistics(bind.table, (int)column_id, &out.min, &out.max, &hn, &hv),
          "cubit_table_column_statistics");
    out.has_null = hn != 0;
    out.has_no_null = hv != 0;
    return true;
}

}  // namespace

TableFunction GetCubitScanFunction() {
    TableFunction f;
    f.name = "cubit_scan";
    f.function = CubitScanFunc;
    f.init_global = CubitScanInitGlobal;
    f.init_local = CubitScanInitLocal;
    f.get_batch_index = CubitScanGetBatchIndex;
    f.table_scan_progress = CubitScanProgress;
    f.cardinality = CubitScanCardinality;
    f.statistics = CubitScanStatistics;
    f.projection_pushdown = true;  // as seq_scan (table_scan.cpp:436-438)
    f.filter_pushdown = true;
    f.filter_prune = true;
    return f;
}

}  // namespace duck
}  // namespace cubit

// ------------------------------------------------------------------ C surface (include/cubit_scan.h)

using namespace cubit::duck;

struct cubit_scan {
    CubitScanBindData bind;
    TableFilterSet filters;
    TableFunctionInitInput input;
    TableFunction fn;
    std::unique_ptr<GlobalTableFunctionState> gstate;
    std::string error;
};

struct cubit_scan_local {
    std::unique_ptr<LocalTableFunctionState> lstate;
    DataChunk chunk;
};

namespace {
thread_local std::string g_scan_error;
int scan_fail(int code, const std::string& m) {
    g_scan_error = m;
    return code;
}
}  // namespace

extern "C" {

const char* cubit_scan_last_error(void) { return g_scan_error.c_str(); }

int cubit_scan_init_global(cubit_table* table, const uint64_t* column_ids, uint32_t n_column_ids,
                           const uint64_t* projection_ids, uint32_t n_projection_ids, const cubit_filter_node* nodes,
                           uint32_t n_nodes, const cubit_txn* txn, cubit_scan** out) {
    if (!table || !out || (n_column_ids && !column_ids)) return scan_fail(CUBIT_ERR_INVALID, "null argument");
    try {
        auto s = std::make_unique<cubit_scan>();
        s->fn = GetCubitScanFunction();
        uint64_t n = 0;
        int64_t base = 0;
        check(cubit_table_info(table, &n, &base, &s->bind.ctx), "cubit_table_info");
        s->bind.table = table;
        s->bind.n_rows = n;
        s->bind.row_base = base;
        if (txn) {
            s->bind.has_txn = true;
            s->bind.txn = *txn;
        }
        s->filters.nodes.assign(nodes, nodes + n_nodes);
        s->input.bind_data = &s->bind;
        s->input.column_ids.assign(column_ids, column_ids + n_column_ids);
        if (projection_ids) s->input.projection_ids.assign(projection_ids, projection_ids + n_projection_ids);
        for (idx_t p : s->input.projection_ids)
            if (p >= n_column_ids) return scan_fail(CUBIT_ERR_INVALID, "projection id out of range");
        s->input.filters = &s->filters;
        s->gstate = s->fn.init_global(s->input);
        *out = s.release();
        return CUBIT_OK;
    } catch (const ScanError& e) {
        return scan_fail(e.code, e.what());
    } catch (const std::exception& e) {
        return scan_fail(CUBIT_ERR_INVALID, e.what());
    }
}

int cubit_scan_max_threads(cubit_scan* s, uint64_t* out) {
    if (!s || !out) return scan_fail(CUBIT_ERR_INVALID, "null argument");
    *out = s->gstate->MaxThreads();
    return CUBIT_OK;
}

int cubit_scan_init_local(cubit_scan* s, cubit_scan_local** out) {
    if (!s || !out) return scan_fail(CUBIT_ERR_INVALID, "null argument");
    auto l = std::make_unique<cubit_scan_local>();
    l->lstate = s->fn.init_local(s->input, s->gstate.get());
    const size_t n_out = s->input.CanRemoveFilterColumns() ? s->input.projection_ids.size() : s->input.column_ids.size();
    l->chunk.Initialize(n_out);
    *out = l.release();
    return CUBIT_OK;
}

int cubit_scan_function(cubit_scan* s, cubit_scan_local* l, int64_t* const* out_columns, uint64_t* out_count) {
    if (!s || !l || !out_count) return scan_fail(CUBIT_ERR_INVALID, "null argument");
    TableFunctionInput in{&s->bind, l->lstate.get(), s->gstate.get()};
    s->fn.function(in, l->chunk);
    const idx_t n = l->chunk.size();
    if (out_columns)
        for (size_t c = 0; c < l->chunk.data.size(); ++c)
            if (out_columns[c]) std::memcpy(out_columns[c], l->chunk.data[c].data(), n * sizeof(int64_t));
    *out_count = n;
    return CUBIT_OK;
}

int cubit_scan_batch_index(cubit_scan* s, cubit_scan_local* l, uint64_t* out) {
    if (!s || !l || !out) return scan_fail(CUBIT_ERR_INVALID, "null argument");
    *out = s->fn.get_batch_index(&s->bind, l->lstate.get(), s->gstate.get());
    return CUBIT_OK;
}

int cubit_scan_progress(cubit_scan* s, double* out) {
    if (!s || !out) return scan_fail(CUBIT_ERR_INVALID, "null argument");
    *out = s->fn.table_scan_progress(&s->bind, s->gstate.get());
    return CUBIT_OK;
}

// bind-time callbacks: the bind data is the partition (no scan state needed)
int cubit_scan_cardinality(cubit_table* table, uint64_t* estimated, uint64_t* max) {
    if (!table) return scan_fail(CUBIT_ERR_INVALID, "null table");
    try {
        CubitScanBindData bind;
        int64_t base = 0;
        check(cubit_table_info(table, &bind.n_rows, &base, &bind.ctx), "cubit_table_info");
        bind.table = table;
        const NodeStatistics st = GetCubitScanFunction().cardinality(&bind);
        if (estimated) *estimated = st.estimated_cardinality;
        if (max) *max = st.max_cardinality;
        return CUBIT_OK;
    } catch (const ScanError& e) {
        return scan_fail(e.code, e.what());
    }
}

int cubit_scan_statistics(cubit_table* table, uint64_t column_id, int64_t* min, int64_t* max, int* has_null,
                          int* has_no_null) {
    if (!table) return scan_fail(CUBIT_ERR_INVALID, "null table");
    try {
        CubitScanBindData bind;
        bind.table = table;
        ColumnStatistics st;
        if (!GetCubitScanFunction().statistics(&bind, column_id, st))
            return scan_fail(CUBIT_ERR_UNSUPPORTED, "no statistics for the row-id column");
        if (min) *min = st.min;
        if (max) *max = st.max;
        if (has_null) *has_null = st.has_null ? 1 : 0;
        if (has_no_null) *has_no_null = st.has_no_null ? 1 : 0;
        return CUBIT_OK;
    } catch (const ScanError& e) {
        return scan_fail(e.code, e.what());
    }
}

int cubit_scan_local_destroy(cubit_scan_local* l) {
    delete l;
    return CUBIT_OK;
}

int cubit_scan_destroy(cubit_scan* s) {
    delete s;
    return CUBIT_OK;
}

}  // extern "C"
