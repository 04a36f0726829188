// cubit_scan: DuckDB TableFunction callbacks over libcubitgpu (see cubit_scan_function.hpp)
// plus the extern "C" surface of include/cubit_scan.h.
#include "cubit_scan_function.hpp"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

#include <immintrin.h>

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

// Buffers outlive one scan: pinning or allocating ~100 MB costs milliseconds, more than the
// work, and DuckDB runs init_global once per query. Freed buffers wait here and a request takes
// the smallest one that fits without wasting more than half of it. The cap bounds what an idle
// process keeps (CUBIT_SCAN_CACHE_MB, default 1 GiB of page-locked and 16 GiB of device
// memory: the probes are sized by the decode's capacity guess, an eighth of the partition's rows,
// and a 4 GiB cap evicted — hipFree — a query's buffers between its runs: SF100 Q6 over 4
// partitions 5.3 ms against 3.1 with room, profiles/r05n_*); cubit_scan_release_cached() frees
// everything cached. Never destroyed (the process
// exit releases the pages; a static destructor could run after the HIP runtime's).
class BufferPool {
  public:
    BufferPool(bool pinned, size_t cap) : pinned_(pinned), cap_(cap) {}
    void* take(cubit_ctx* ctx, size_t bytes, size_t* got) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            // page-locked buffers are filed under no context (give), device buffers under theirs
            cubit_ctx* owner = pinned_ ? nullptr : ctx;
            auto it = free_.lower_bound(Key{owner, bytes});
            if (it != free_.end() && it->first.ctx == owner && it->first.bytes <= 2 * bytes) {
                void* p = it->second;
                *got = it->first.bytes;
                cached_ -= it->first.bytes;
                free_.erase(it);
                return p;
            }
        }
        void* h = nullptr;
        if (pinned_) check(cubit_host_alloc(ctx, bytes, &h), "cubit_host_alloc");
        else check(cubit_dev_alloc(ctx, bytes, &h), "cubit_dev_alloc");
        *got = bytes;
        return h;
    }
    void give(cubit_ctx* ctx, void* p, size_t bytes) {
        std::lock_guard<std::mutex> lk(mu_);
        free_.emplace(Key{pinned_ ? nullptr : ctx, bytes}, p);
        cached_ += bytes;
        while (cached_ > cap_ && !free_.empty()) {  // drop the largest first
            auto it = std::prev(free_.end());
            drop(it);
        }
    }
    void release_all() {
        std::lock_guard<std::mutex> lk(mu_);
        while (!free_.empty()) drop(free_.begin());
    }
    // device buffers of a context that is going away
    void release_ctx(cubit_ctx* ctx) {
        std::lock_guard<std::mutex> lk(mu_);
        for (auto it = free_.begin(); it != free_.end();) {
            auto nx = std::next(it);
            if (it->first.ctx == ctx) drop(it);
            it = nx;
        }
    }
    size_t cached() {
        std::lock_guard<std::mutex> lk(mu_);
        return cached_;
    }

  private:
    struct Key {
        cubit_ctx* ctx;  // owning context of device memory (pinned memory: nullptr, any context)
        size_t bytes;
        bool operator<(const Key& o) const { return ctx != o.ctx ? ctx < o.ctx : bytes < o.bytes; }
    };
    void drop(std::multimap<Key, void*>::iterator it) {
        cached_ -= it->first.bytes;
        if (pinned_) cubit_host_free(nullptr, it->second);
        else cubit_dev_free(it->first.ctx, it->second);
        free_.erase(it);
    }
    const bool pinned_;
    const size_t cap_;
    std::mutex mu_;
    std::multimap<Key, void*> free_;
    size_t cached_ = 0;
};

size_t cache_cap_mb(size_t dflt) {
    const char* e = std::getenv("CUBIT_SCAN_CACHE_MB");
    return (e && *e ? std::strtoull(e, nullptr, 10) : dflt) << 20;
}
BufferPool& pinned_pool() {
    static BufferPool* p = new BufferPool(true, cache_cap_mb(1024));
    return *p;
}
BufferPool& device_pool() {
    static BufferPool* p = new BufferPool(false, cache_cap_mb(1024) * 16);
    return *p;
}

// A buffer from one of the pools, returned on destruction.
struct PooledBuffer {
    BufferPool* pool = nullptr;
    cubit_ctx* ctx = nullptr;
    void* p = nullptr;
    size_t bytes = 0;
    PooledBuffer() = default;
    PooledBuffer(const PooledBuffer&) = delete;
    PooledBuffer& operator=(const PooledBuffer&) = delete;
    PooledBuffer(PooledBuffer&& o) noexcept : pool(o.pool), ctx(o.ctx), p(o.p), bytes(o.bytes) { o.p = nullptr; }
    void allocate(BufferPool& pl, cubit_ctx* c, size_t want) {
        reset();
        pool = &pl;
        ctx = c;
        p = pl.take(c, std::max<size_t>(want, 16), &bytes);
    }
    void reset() {
        if (p) pool->give(ctx, p, bytes);
        p = nullptr;
    }
    int64_t* i64() { return static_cast<int64_t*>(p); }
    ~PooledBuffer() { reset(); }
};

// Streaming result of one scan. init_global runs the GPU work — one decode (ordered: the runs
// laid out in tile order, so consecutive tiles are one contiguous range of ids) and the probe
// of every emitted column, all on the device — and copies only the count and the tile
// directory to the host. The ids and values then reach the host per *window* (consecutive
// non-empty tiles of about window_rows() rows): the local state that claims a window copies its
// range of every emitted column into its own page-locked buffer (or reads it where init_global
// staged it) and hands the window's rows out as full DataChunks of 2,048, one batch index per
// window. The reference hands out one row group per NextParallelScan and produces
// its chunks on demand (table_scan.cpp:119-156); a window is the unit a GPU→host copy is worth.
// Window size: at most window_rows() rows and window_rows() / 4,096 tiles (2^18 rows and 64
// tiles by default; CUBIT_SCAN_WINDOW_ROWS sets the row bound, a power of two ≥ 2^14).
idx_t window_rows() {
    static const idx_t rows = [] {
        const char* e = std::getenv("CUBIT_SCAN_WINDOW_ROWS");
        idx_t r = e && *e ? (idx_t)std::strtoull(e, nullptr, 10) : (idx_t)1 << 18;
        return std::max<idx_t>(r, (idx_t)1 << 14);
    }();
    return rows;
}

struct Window {
    uint32_t part;         // the partition the window's tiles belong to
    uint32_t first, last;  // index range [first, last) into that partition's non-empty tiles
    idx_t off, len;        // the window's rows in the partition's ordered output
    uint32_t group = 0;    // staged partitions: the group of copies that brings the window's rows
};

// Staging: init_global copies every emitted column's transfer form (and validity words) to
// page-locked host memory on ONE copy stream per device, in row order, in about stage_groups()
// groups of consecutive windows per partition: each group's probes and narrowing fill its block
// on the context stream, the copy stream waits for them, copies the block and records an event. A
// pipeline task that claims a window waits for its group's event and reads the rows in place. One stream of multi-megabyte
// copies runs the link at its own rate (56.6 GB/s for one 64 MiB copy on the MI355X box); the
// tasks' concurrent per-window copies (0.5–1 MB each on up to 16 streams) reached ~20 GB/s
// (profiles/r05k_*). CUBIT_SCAN_STAGE_MB (default 1024) bounds the bytes one scan stages over all
// of its partitions: a partition past the budget, or whose blocks cannot be allocated, is copied
// per window by the task that claims it.
uint64_t stage_groups() {  // 8; CUBIT_SCAN_STAGE_GROUPS overrides (diagnostic)
    static const uint64_t n = [] {
        const char* e = std::getenv("CUBIT_SCAN_STAGE_GROUPS");
        const uint64_t v = e && *e ? std::strtoull(e, nullptr, 10) : 8;
        return std::max<uint64_t>(v, 1);
    }();
    return n;
}

uint64_t stage_cap_bytes() {  // read per init_global; MiB, fractions allowed (tests)
    const char* e = std::getenv("CUBIT_SCAN_STAGE_MB");
    const double mb = e && *e ? std::strtod(e, nullptr) : 1024.0;
    return mb > 0 ? (uint64_t)(mb * 1048576.0) : 0;
}

// The device side of one partition's scan: its ordered row ids, the probed columns and the
// non-empty tiles' runs.
struct PartScan {
    CubitPartition part;
    idx_t count = 0;
    idx_t rows_per_tile = 0;
    uint64_t tile_base = 0;   // tiles of the earlier partitions: batch index = tile_base + tile
    uint32_t decodes = 0;     // decode launches (a second one only when the capacity fell short)
    PooledBuffer d_cnt;  // the decode's count (2 words), then its tile directory: one read brings both
    PooledBuffer d_ids;                  // device: ordered row ids
    std::vector<PooledBuffer> d_cols;    // device: per emitted position, probed values
    // transfer compaction per emitted position: the window copies move `width` bytes per value
    // (1, 2, 3 or 4: value - offset as an unsigned integer, the smallest width the column's
    // statistics allow; 0 = the 8-byte values) from d_narrow, and the chunk fill widens them back
    std::vector<int> width;
    std::vector<int64_t> offset;
    std::vector<PooledBuffer> d_narrow;
    // the compaction bound is checked on the device (cubit_narrow_checked): one flag word per
    // group and emitted position — staged, at the head of the group's block and read by the tasks
    // that claim its windows; per-window copies, read once before the partition's first window —
    // and a column whose flag is set goes back to its 8-byte values
    PooledBuffer d_overflow;
    std::once_flag overflow_checked;
    // NULL-ness per emitted position: a column whose statistics admit NULLs (update records
    // included) is probed with its validity (cubit_table_probe_validity): d_valid holds one bit
    // per ordered output row, and the windows copy their words beside the values
    std::vector<bool> nullable;
    std::vector<PooledBuffer> d_valid;
    std::vector<uint32_t> tiles;         // non-empty tiles, ascending
    std::vector<idx_t> tile_off, tile_len;  // per non-empty tile: its run in the ordered output
    // staging (see stage_groups()): per group one block (BlockLayout) on the device and its copy
    // in page-locked memory, both laid out back to back; the group's events
    bool staged = false;
    PooledBuffer d_block, h_block;
    std::vector<uint64_t> blk_off;          // per group: its block's first byte (+ the end)
    std::vector<uint64_t> col_rel, val_rel;  // per group × emitted position: its regions in the block
    std::vector<void*> probe_ev, group_ev;  // per group: probes done (context stream), copies done
    std::vector<idx_t> group_off, group_len;  // per group: its first row (bit 0 of its validity words), rows
    uint32_t groups_launched = 0;          // group_ev[k] exists for k below it (CubitScanGlobalState::stage_mu)
    ~PartScan() {
        for (void* ev : group_ev)
            if (ev) cubit_copy_event_destroy(part.ctx, ev);
        for (void* ev : probe_ev) cubit_copy_event_destroy(part.ctx, ev);
    }
};

struct CubitScanGlobalState : public GlobalTableFunctionState {
    std::vector<std::unique_ptr<PartScan>> parts;  // row order
    std::vector<column_t> column_ids;
    std::vector<idx_t> emit;  // positions of column_ids that reach the output
    idx_t count = 0;          // all partitions
    std::vector<Window> windows;  // partition by partition, each in tile order
    idx_t max_window = 0;
    uint64_t stage_left = 0;  // staging bytes the partitions not yet staged may still take
    std::atomic<uint32_t> next{0};
    std::atomic<idx_t> emitted{0};
    // one staging copy stream per context, shared by the partitions on that device (their copies
    // run in row order on it; a stream per partition put several copy streams on one device's
    // four hardware queues and measured slower)
    std::vector<std::pair<cubit_ctx*, void*>> stage_streams;
    // the staged groups' device work (probes, narrowing, block copies, events) is launched by this
    // thread after init_global has returned, so the pipeline's tasks start while it launches; a task
    // that claims a window of a group not launched yet waits on stage_cv
    std::thread stager;
    std::mutex stage_mu;
    std::condition_variable stage_cv;
    std::string stage_error;  // a launch failed: every waiting task throws it
    void* StageStream(cubit_ctx* ctx) {
        for (auto& s : stage_streams)
            if (s.first == ctx) return s.second;
        void* st = nullptr;
        check(cubit_copy_stream_create(ctx, &st), "staging stream");  // after the probes and narrowing
        stage_streams.emplace_back(ctx, st);
        return st;
    }
    idx_t MaxThreads() const override {
        const idx_t hw = std::max<unsigned>(1, std::thread::hardware_concurrency());
        return std::max<idx_t>(1, std::min<idx_t>(windows.size(), hw));
    }
    ~CubitScanGlobalState() override {
        if (stager.joinable()) stager.join();
        // probes launched by init_global may still read the buffers returned to the pool
        for (auto& p : parts)
            if (p->part.ctx) cubit_sync(p->part.ctx);
        parts.clear();  // their staging events first
        for (auto& s : stage_streams) cubit_copy_stream_destroy(s.first, s.second);
    }
};

bool phases_enabled() {
    static const bool on = std::getenv("CUBIT_SCAN_PHASES") != nullptr;
    return on;
}

struct CubitScanLocalState : public LocalTableFunctionState {
    int64_t window = -1;           // claimed window, -1 = none yet
    idx_t pos = 0;                 // next row of the window to emit
    std::vector<PooledBuffer> host;  // per emitted position: the window's rows (page-locked)
    std::vector<PooledBuffer> host_valid;  // per nullable position: the window's validity words
    // per emitted position: the window's first row on the host (its own copy, or the partition's
    // staged rows), the transfer width of the window's values, and validity words whose bit 0 is
    // the partition's output row valid_bit0
    std::vector<const char*> src;
    std::vector<int> width;
    std::vector<const uint64_t*> src_valid;
    idx_t valid_bit0 = 0;
    // this task's copy stream per context (ordered after init_global's device work on it):
    // the tasks' window copies run side by side, each from its own device; partitions that share
    // a context (several on one device) share the stream — a stream per partition and task put
    // 64 streams on one device at 8 × 8 and ran 4x slower (profiles/r05d_partitioned_pipeline.txt)
    std::vector<std::pair<cubit_ctx*, void*>> streams;
    void* stream_for(cubit_ctx* ctx) {
        for (auto& s : streams)
            if (s.first == ctx) return s.second;
        void* st = nullptr;
        check(cubit_copy_stream_create(ctx, &st), "copy stream");
        streams.emplace_back(ctx, st);
        return st;
    }
    // CUBIT_SCAN_PHASES=1 (diagnostic): windows claimed and the time spent waiting for their
    // staged groups / copies, on stderr when the state goes away
    uint32_t n_windows = 0;
    double wait_us = 0;
    ~CubitScanLocalState() override {
        if (phases_enabled() && n_windows)
            std::fprintf(stderr, "cubit_scan task windows %u wait_us %.1f\n", n_windows, wait_us);
        for (auto& s : streams)
            if (s.second) cubit_copy_stream_destroy(s.first, s.second);
    }
};

int64_t* device_ptr(PooledBuffer& b) { return b.i64(); }

// The decode of one partition into a buffer of `cap` row ids, launched and not waited for; the
// count and directory are read after every partition has been launched, so the partitions'
// devices decode side by side.
void LaunchDecode(PartScan& P, const std::vector<cubit_filter_node>& nodes, const cubit_txn* txn, uint64_t cap) {
    cubit_ctx* ctx = P.part.ctx;
    ++P.decodes;
    // this scan's tile directory, copied out within the scan call: other pipeline tasks or
    // queries may scan on the same context right after it (cubit_table_scan_tiles)
    const uint32_t dir_cap = (uint32_t)((P.part.n_rows + 131071) / 131072 + 1);
    if (!P.d_cnt.p) P.d_cnt.allocate(device_pool(), ctx, 16 + 2ull * dir_cap * 8);
    P.d_ids.allocate(device_pool(), ctx, std::max<uint64_t>(cap, 1) * 8);
    uint32_t n_tiles = 0;
    check(cubit_table_scan_tiles(P.part.table, nodes.empty() ? nullptr : nodes.data(), (uint32_t)nodes.size(), txn,
                                 device_ptr(P.d_ids), P.d_ids.bytes / 8, static_cast<uint64_t*>(P.d_cnt.p),
                                 CUBIT_SCAN_ORDERED, static_cast<uint64_t*>(P.d_cnt.p) + 2, dir_cap, &n_tiles,
                                 &P.rows_per_tile),
          "cubit_table_scan_tiles");
    P.tiles.assign(n_tiles, 0);  // the directory's size until FinishDecode reads it
}

// The first decode's capacity: twice the planner's estimate of the qualifying rows
// (cubit_table_estimate_rows: zone statistics, no scan), at least an eighth of the partition, at
// most all of it — so a filter keeping half the rows decodes once into a buffer of every row
// (device memory is pooled across queries, and an unfilled buffer costs no bandwidth). Only an
// estimate off by more than 2x (correlated columns) takes the second pass.
uint64_t DecodeCapacity(const PartScan& P, const std::vector<cubit_filter_node>& nodes) {
    const uint64_t n = P.part.n_rows;
    uint64_t est = n;
    if (!nodes.empty())
        check(cubit_table_estimate_rows(P.part.table, nodes.data(), (uint32_t)nodes.size(), &est),
              "cubit_table_estimate_rows");
    return std::min<uint64_t>(n + 1, std::max<uint64_t>(n / 8, 2 * est) + 4096);
}

// Count and tile runs of a launched decode; a filter that kept more rows than the capacity runs
// a second time with the exact count.
void FinishDecode(PartScan& P, const std::vector<cubit_filter_node>& nodes, const cubit_txn* txn) {
    cubit_ctx* ctx = P.part.ctx;
    // the count and the directory in one read (the tile count is known from the launch)
    std::vector<uint64_t> head(2 + 2 * P.tiles.size());
    check(cubit_memcpy_d2h(ctx, head.data(), P.d_cnt.p, head.size() * 8), "count and directory");
    P.count = head[0];
    if (P.count > P.d_ids.bytes / 8) {
        LaunchDecode(P, nodes, txn, P.count);
        head.assign(2 + 2 * P.tiles.size(), 0);
        check(cubit_memcpy_d2h(ctx, head.data(), P.d_cnt.p, head.size() * 8), "count and directory");
        if (head[0] != P.count) throw ScanError(CUBIT_ERR_CAPACITY, "cubit_table_scan: count changed between the passes");
    }
    const uint32_t n_tiles = P.count ? (uint32_t)P.tiles.size() : 0;  // nothing qualified: no run
    P.tiles.clear();
    const uint64_t* dir = head.data() + 2;
    // the ordered layout: tile t's run starts at the sum of the earlier tiles' lengths
    idx_t off = 0;
    for (uint32_t t = 0; t < n_tiles; ++t) {
        const uint64_t len = dir[2 * t + 1];
        if (!len) continue;
        if (len > P.count - off)
            throw ScanError(CUBIT_ERR_INVALID, "cubit_scan: tile directory does not describe this scan's output");
        P.tiles.push_back(t);
        P.tile_off.push_back(off);
        P.tile_len.push_back(len);
        off += len;
    }
    if (off != P.count)
        throw ScanError(CUBIT_ERR_INVALID, "cubit_scan: tile runs cover " + std::to_string(off) + " of " +
                                               std::to_string(P.count) + " row ids");
}

// The transfer plan of a partition's emitted columns. The statistics (DataTable::GetStatistics,
// update records of any version included) say which columns can hold a NULL: those probe with
// their validity, which also leaves 0 in a NULL row's value. The transfer compaction: a column
// whose values all lie within 2^32 of an offset crosses PCIe as value - offset in the fewest of
// 1, 2, 3 and 4 bytes that hold the range (row ids: the partition's rows, offset row_base;
// probed columns: their statistics' range, widened by any update records — a NULL row holds 0
// after the validity probe, so 0 joins the range of a nullable column). Q6's l_discount (0 … 10)
// crosses as one byte, l_extendedprice as three. The device checks the bound as it narrows (one
// flag per group and column).
void PlanWidths(PartScan& P, const std::vector<column_t>& column_ids, const std::vector<idx_t>& emit) {
    const size_t n_emit = emit.size();
    P.nullable.assign(n_emit, false);
    P.width.assign(n_emit, 0);
    P.offset.assign(n_emit, 0);
    // CUBIT_SCAN_TEST_SHIFT_OFFSET=1 (tests only): every compacted column's offset one above its
    // minimum, so the device flags the groups that hold the minimum and their windows take the
    // 8-byte fallback
    const char* shift_env = std::getenv("CUBIT_SCAN_TEST_SHIFT_OFFSET");
    const int64_t shift = shift_env && *shift_env == '1' ? 1 : 0;
    for (size_t e = 0; e < n_emit; ++e) {
        const column_t col = column_ids[emit[e]];
        int64_t lo, hi;
        if (col == COLUMN_IDENTIFIER_ROW_ID) {
            lo = P.part.row_base;
            hi = P.part.row_base + (int64_t)P.part.n_rows - 1;
        } else {
            int hn = 0, hv = 0, type = 0;
            const void* data = nullptr;
            check(cubit_table_column_statistics(P.part.table, (int)col, &lo, &hi, &hn, &hv),
                  "cubit_table_column_statistics");
            check(cubit_table_column_data(P.part.table, (int)col, &data, &type), "cubit_table_column_data");
            P.nullable[e] = hn != 0;
            // FLOAT: the 32-bit patterns (zero-extended) cross as 4 bytes; DOUBLE: the 8-byte patterns
            if (type == CUBIT_TYPE_DOUBLE) continue;
            if (type == CUBIT_TYPE_FLOAT) {
                lo = 0;
                hi = 0xffffffffll;
            }
            if (P.nullable[e] && type == CUBIT_TYPE_UINT64) {
                lo = 0;  // bits of unsigned bounds: 0 is below every value, and the span stays unsigned
            } else if (P.nullable[e]) {
                lo = std::min<int64_t>(lo, 0);
                hi = std::max<int64_t>(hi, 0);
            }
        }
        const uint64_t span = (uint64_t)hi - (uint64_t)lo;  // hi >= lo
        const int width = span < (1ull << 8) ? 1 : span < (1ull << 16) ? 2 : span < (1ull << 24) ? 3 : span < (1ull << 32) ? 4 : 0;
        if (!width) continue;
        P.width[e] = width;
        P.offset[e] = lo + shift;
    }
}

// Bytes per row of an emitted column's transfer form: its compacted width, or the 8-byte value.
uint64_t transfer_bytes(const PartScan& P, size_t e) { return P.width[e] ? (uint64_t)P.width[e] : 8; }

constexpr uint64_t round16(uint64_t b) { return (b + 15) & ~15ull; }

// One group's staging block (offsets from the block's first byte, every region 16-byte aligned):
// the overflow flags (one word per emitted position), each emitted column's transfer form (+ 16
// bytes: the 3-byte widen reads past the last value), then the validity words of each nullable
// column (+ 2 words: the chunk fill reads one word ahead). Returns the block's size.
uint64_t BlockLayout(const PartScan& P, idx_t len, uint64_t* col_rel, uint64_t* val_rel) {
    const size_t n_emit = P.width.size();
    uint64_t rel = round16(n_emit * 4);
    for (size_t e = 0; e < n_emit; ++e) {
        col_rel[e] = rel;
        rel += round16(len * transfer_bytes(P, e) + 16);
    }
    for (size_t e = 0; e < n_emit; ++e) {
        val_rel[e] = rel;
        if (P.nullable[e]) rel += round16(((len + 63) / 64 + 2) * 8);
    }
    return rel;
}

// Probe every emitted storage column at rows [off, off + len) of the partition's ordered row ids
// (ColumnData::FilterScan semantics, column_data.cpp:305-309: values with their validity), then
// narrow them; all on the context stream. Per emitted position: values to `cols[e]` (a narrowed
// column: to d_cols, read by the narrowing and by the 8-byte fallback), validity words to
// `valid[e]`, the transfer form to `out[e]` and the overflow flag to `flags + e`. The row id
// column's transfer form is its narrowing, or (width 0) a copy of the ids when `out` is a staging
// block (`copy_ids`).
void ProbeRange(PartScan& P, const std::vector<column_t>& column_ids, const std::vector<idx_t>& emit,
                const cubit_txn* txn, idx_t off, idx_t len, int64_t* const* cols, uint64_t* const* valid,
                char* const* out, uint32_t* flags, bool copy_ids) {
    cubit_ctx* ctx = P.part.ctx;
    cubit_table* table = P.part.table;
    const size_t n_emit = emit.size();
    uint64_t* d_cnt = static_cast<uint64_t*>(P.d_cnt.p);  // ≥ off + len: the kernels take min(count, len)
    for (size_t e = 0; e < n_emit; ++e) {
        const column_t col = column_ids[emit[e]];
        if (col == COLUMN_IDENTIFIER_ROW_ID) continue;
        if (P.nullable[e]) {
            check(cubit_table_probe_validity(table, (int)col, txn, device_ptr(P.d_ids) + off, d_cnt, len, cols[e], valid[e]),
                  "cubit_table_probe_validity");
        } else {
            check(cubit_table_probe(table, (int)col, txn, device_ptr(P.d_ids) + off, d_cnt, len, cols[e]),
                  "cubit_table_probe");
        }
    }
    for (size_t e = 0; e < n_emit; ++e) {
        const bool rowid = column_ids[emit[e]] == COLUMN_IDENTIFIER_ROW_ID;
        if (P.width[e]) {
            const int64_t* src = rowid ? device_ptr(P.d_ids) + off : cols[e];
            check(cubit_narrow_checked(ctx, src, d_cnt, len, P.offset[e], P.width[e], out[e], flags + e),
                  "cubit_narrow_checked");
        } else if (rowid && copy_ids) {
            check(cubit_memcpy_d2d(ctx, out[e], device_ptr(P.d_ids) + off, len * 8), "row id copy");
        }
    }
}

// The probes, compaction and (staged) copies of partition p. Staged (see stage_groups()): the
// partition's windows are cut into groups, each with one staging block on the device and its
// image in page-locked memory; here the groups are laid out and the blocks allocated, and the
// stager thread launches each group's work (LaunchStagedGroups: the probes and narrowing fill the
// block on the context stream and close with an event, and the staging stream waits for it and
// copies the block in ONE copy — the link starts on the first group while the device probes the
// next; one copy per column and a separate flags copy left ≈ 35 µs of gaps per group on the link,
// profiles/r05ae_*). Not staged: one probe over every row into partition-wide buffers, launched
// here, and each task copies the window it claims.
void ProbeAndStage(CubitScanGlobalState& g, uint32_t p, const cubit_txn* txn) {
    PartScan& P = *g.parts[p];
    cubit_ctx* ctx = P.part.ctx;
    const size_t n_emit = g.emit.size();
    PlanWidths(P, g.column_ids, g.emit);
    // groups of consecutive windows: about an eighth of the partition each (each group costs a
    // probe and a narrowing launch per column, a few microseconds apiece), at least 2^18 rows
    std::vector<idx_t> g_off, g_len;
    const uint64_t rows_per_group = std::max<uint64_t>((P.count + stage_groups() - 1) / stage_groups(), 1ull << 18);
    for (Window& w : g.windows) {
        if (w.part != p) continue;
        if (g_off.empty() || g_len.back() + w.len > rows_per_group) {
            g_off.push_back(w.off);
            g_len.push_back(0);
        }
        w.group = (uint32_t)g_off.size() - 1;
        g_len.back() += w.len;
    }
    const size_t n_groups = g_off.size();
    P.col_rel.assign(n_groups * n_emit, 0);
    P.val_rel.assign(n_groups * n_emit, 0);
    P.blk_off.assign(n_groups + 1, 0);
    for (size_t k = 0; k < n_groups; ++k)
        P.blk_off[k + 1] = P.blk_off[k] + BlockLayout(P, g_len[k], &P.col_rel[k * n_emit], &P.val_rel[k * n_emit]);
    P.d_cols.resize(n_emit);
    P.d_valid.resize(n_emit);
    P.d_narrow.resize(n_emit);
    if (P.count == 0 || n_emit == 0) return;
    // staged when the partition's blocks fit what is left of the scan's staging budget (one
    // budget over all partitions: N partitions must not pin N budgets) and both the device and the
    // page-locked block can be had; else each task copies the windows it claims
    bool staged = P.blk_off[n_groups] <= g.stage_left;
    if (staged) {
        try {
            P.d_block.allocate(device_pool(), ctx, P.blk_off[n_groups]);
            P.h_block.allocate(pinned_pool(), ctx, P.blk_off[n_groups]);
            g.stage_left -= P.blk_off[n_groups];
        } catch (const ScanError&) {
            P.d_block.reset();
            P.h_block.reset();
            staged = false;
        }
    }
    // partition-wide values of every probed column that the staging does not take whole: the
    // narrowed ones (their 8-byte fallback) and, not staged, all
    for (size_t e = 0; e < n_emit; ++e)
        if (g.column_ids[g.emit[e]] != COLUMN_IDENTIFIER_ROW_ID && (P.width[e] || !staged))
            P.d_cols[e].allocate(device_pool(), ctx, P.count * 8);
    std::vector<int64_t*> cols(n_emit, nullptr);
    std::vector<uint64_t*> valid(n_emit, nullptr);
    std::vector<char*> out(n_emit, nullptr);
    if (!staged) {  // one probe over every row, validity words in row order
        for (size_t e = 0; e < n_emit; ++e) {
            cols[e] = device_ptr(P.d_cols[e]);
            if (P.nullable[e]) {
                P.d_valid[e].allocate(device_pool(), ctx, ((P.count + 63) / 64 + 2) * 8);
                valid[e] = static_cast<uint64_t*>(P.d_valid[e].p);
            }
            if (P.width[e]) {
                P.d_narrow[e].allocate(device_pool(), ctx, P.count * (uint64_t)P.width[e] + 16);
                out[e] = static_cast<char*>(P.d_narrow[e].p);
            }
        }
        P.d_overflow.allocate(device_pool(), ctx, n_emit * 4);
        check(cubit_memset_d(ctx, P.d_overflow.p, 0, n_emit * 4), "overflow flags");
        ProbeRange(P, g.column_ids, g.emit, txn, 0, P.count, cols.data(), valid.data(), out.data(),
                   static_cast<uint32_t*>(P.d_overflow.p), false);
        return;
    }
    g.StageStream(ctx);  // created here: the stager only looks it up
    P.group_off = g_off;
    P.group_len = g_len;
    P.group_ev.assign(n_groups, nullptr);
    P.staged = true;
}

// The staged groups of partition p, launched in row order (the stager thread): per group the
// overflow flags are cleared, the probes and narrowing fill its device block on the context
// stream, an event closes them, and the staging stream waits for it, copies the block into its
// page-locked image and records the group's event.
void LaunchStagedGroups(CubitScanGlobalState& g, uint32_t p, const cubit_txn* txn) {
    PartScan& P = *g.parts[p];
    cubit_ctx* ctx = P.part.ctx;
    const size_t n_emit = g.emit.size();
    void* st = g.StageStream(ctx);
    std::vector<int64_t*> cols(n_emit, nullptr);
    std::vector<uint64_t*> valid(n_emit, nullptr);
    std::vector<char*> out(n_emit, nullptr);
    for (size_t k = 0; k < P.group_off.size(); ++k) {
        const idx_t off = P.group_off[k], len = P.group_len[k];
        char* blk = static_cast<char*>(P.d_block.p) + P.blk_off[k];
        for (size_t e = 0; e < n_emit; ++e) {
            char* region = blk + P.col_rel[k * n_emit + e];
            const bool rowid = g.column_ids[g.emit[e]] == COLUMN_IDENTIFIER_ROW_ID;
            cols[e] = rowid ? nullptr : P.width[e] ? device_ptr(P.d_cols[e]) + off : reinterpret_cast<int64_t*>(region);
            valid[e] = P.nullable[e] ? reinterpret_cast<uint64_t*>(blk + P.val_rel[k * n_emit + e]) : nullptr;
            out[e] = region;
        }
        check(cubit_memset_d(ctx, blk, 0, n_emit * 4), "overflow flags");
        ProbeRange(P, g.column_ids, g.emit, txn, off, len, cols.data(), valid.data(), out.data(),
                   reinterpret_cast<uint32_t*>(blk), true);
        void* probed = nullptr;
        check(cubit_copy_event_record(ctx, nullptr, &probed), "probe event");  // on the context stream
        P.probe_ev.push_back(probed);
        check(cubit_copy_stream_wait_event(ctx, st, probed), "staging wait");
        check(cubit_memcpy_d2h_async(ctx, st, static_cast<char*>(P.h_block.p) + P.blk_off[k], blk,
                                     P.blk_off[k + 1] - P.blk_off[k]),
              "staged block");
        void* ev = nullptr;
        check(cubit_copy_event_record(ctx, st, &ev), "staged group event");
        {
            std::lock_guard<std::mutex> lk(g.stage_mu);
            P.group_ev[k] = ev;
            P.groups_launched = (uint32_t)k + 1;
        }
        g.stage_cv.notify_all();
    }
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
    const cubit_txn* txn = bind.has_txn ? &bind.txn : nullptr;
    const auto& nodes = input.filters ? input.filters->nodes : std::vector<cubit_filter_node>{};
    uint64_t tile_base = 0;
    for (const CubitPartition& part : bind.parts) {
        auto P = std::make_unique<PartScan>();
        P->part = part;
        P->tile_base = tile_base;
        tile_base += (part.n_rows + 131071) / 131072;
        g->parts.push_back(std::move(P));
    }
    // CUBIT_SCAN_PHASES=1: the host time of init_global's phases on stderr (diagnostic)
    const bool phases = phases_enabled();
    auto t0 = std::chrono::steady_clock::now(), t1 = t0, t2 = t0;
    // every partition's decode in flight before any count is read: one per device at a time
    for (auto& P : g->parts) LaunchDecode(*P, nodes, txn, DecodeCapacity(*P, nodes));
    if (phases) t1 = std::chrono::steady_clock::now();
    for (auto& P : g->parts) FinishDecode(*P, nodes, txn);
    if (phases) t2 = std::chrono::steady_clock::now();
    // windows: consecutive non-empty tiles of one partition, at most window_rows() rows and
    // window_rows() / 4,096 tiles
    const idx_t max_rows = window_rows(), max_tiles = max_rows / 4096;
    for (uint32_t p = 0; p < g->parts.size(); ++p) {
        const PartScan& P = *g->parts[p];
        g->count += P.count;
        for (uint32_t i = 0; i < P.tiles.size();) {
            Window w{p, i, i, P.tile_off[i], 0};
            while (w.last < P.tiles.size() &&
                   (w.last == w.first || (w.len + P.tile_len[w.last] <= max_rows && w.last - w.first < max_tiles))) {
                w.len += P.tile_len[w.last];
                ++w.last;
            }
            g->max_window = std::max(g->max_window, w.len);
            g->windows.push_back(w);
            i = w.last;
        }
    }
    g->stage_left = stage_cap_bytes();
    bool any_staged = false;
    for (uint32_t p = 0; p < g->parts.size(); ++p) {
        ProbeAndStage(*g, p, txn);
        any_staged |= g->parts[p]->staged;
    }
    if (any_staged) {
        CubitScanGlobalState* gs = g.get();
        gs->stager = std::thread([gs, txn] {
            try {
                for (uint32_t p = 0; p < gs->parts.size(); ++p)
                    if (gs->parts[p]->staged) LaunchStagedGroups(*gs, p, txn);
            } catch (const std::exception& e) {
                std::lock_guard<std::mutex> lk(gs->stage_mu);
                gs->stage_error = e.what();
            }
            gs->stage_cv.notify_all();
        });
    }
    if (phases) {
        const auto t3 = std::chrono::steady_clock::now();
        auto us = [](auto a, auto b) { return std::chrono::duration<double, std::micro>(b - a).count(); };
        std::fprintf(stderr, "cubit_scan phases launch_decode_us %.1f finish_decode_us %.1f probe_stage_us %.1f\n",
                     us(t0, t1), us(t1, t2), us(t2, t3));
    }
    return g;
}

std::unique_ptr<LocalTableFunctionState> CubitScanInitLocal(TableFunctionInitInput&, GlobalTableFunctionState*) {
    return std::make_unique<CubitScanLocalState>();
}

// TableScanParallelStateNext analogue: take the next window (row_group_collection.cpp hands
// out row groups under a mutex; one atomic suffices here). Staged partitions: wait for the
// window's group and point at its rows in the staged buffers. Otherwise: copy the window's rows
// of every emitted column to this state's page-locked buffers, from the window's partition on
// that partition's device, one window at a time (claiming the next window and copying it while
// the current one is handed out measured slower at 8 and 16 tasks: 12.4 vs 5.09 ms,
// profiles/r04c_pipeline_prefetch_not_kept.txt; round 3: profiles/r03mn_*).
bool NextWindow(CubitScanGlobalState& g, CubitScanLocalState& l) {
    const uint32_t w = g.next.fetch_add(1);
    if (w >= g.windows.size()) {
        l.window = (int64_t)g.windows.size();
        return false;
    }
    const Window& win = g.windows[w];
    PartScan& P = *g.parts[win.part];
    const size_t n_emit = g.emit.size();
    if (l.host.size() != n_emit) {
        l.host.resize(n_emit);
        l.host_valid.resize(n_emit);
        l.src.resize(n_emit);
        l.width.resize(n_emit);
        l.src_valid.resize(n_emit);
    }
    l.window = w;
    l.pos = 0;
    // progress counts rows when their window is claimed, as TableScanProgress counts the row
    // groups the parallel cursor has handed out (table_scan.cpp:158-177); one atomic per window
    g.emitted.fetch_add(win.len, std::memory_order_relaxed);
    ++l.n_windows;
    const bool timed = phases_enabled();
    const auto t_claim = timed ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point{};
    auto waited = [&] {
        if (timed) l.wait_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_claim).count();
    };
    if (P.staged) {
        const uint32_t k = win.group;
        void* ev = nullptr;
        {
            std::unique_lock<std::mutex> lk(g.stage_mu);
            g.stage_cv.wait(lk, [&] { return P.groups_launched > k || !g.stage_error.empty(); });
            if (P.groups_launched <= k) throw ScanError(CUBIT_ERR_DEVICE, "cubit_scan staging: " + g.stage_error);
            ev = P.group_ev[k];
        }
        check(cubit_copy_event_sync(P.part.ctx, ev), "staged group");
        waited();
        // the group's overflow flags came at the head of its block: a column whose compaction
        // overflowed in this group is copied per window as its 8-byte values instead
        const char* blk = static_cast<const char*>(P.h_block.p) + P.blk_off[k];
        const uint32_t* ov = reinterpret_cast<const uint32_t*>(blk);
        l.valid_bit0 = P.group_off[k];
        bool copied = false;
        for (size_t e = 0; e < n_emit; ++e) {
            if (P.nullable[e]) l.src_valid[e] = reinterpret_cast<const uint64_t*>(blk + P.val_rel[k * n_emit + e]);
            l.width[e] = P.width[e];
            if (!(P.width[e] && ov[e])) {
                l.src[e] = blk + P.col_rel[k * n_emit + e] + (win.off - P.group_off[k]) * transfer_bytes(P, e);
                continue;
            }
            l.width[e] = 0;
            if (!l.host[e].p) l.host[e].allocate(pinned_pool(), P.part.ctx, g.max_window * 8);
            PooledBuffer& src = g.column_ids[g.emit[e]] == COLUMN_IDENTIFIER_ROW_ID ? P.d_ids : P.d_cols[e];
            check(cubit_memcpy_d2h_async(P.part.ctx, l.stream_for(P.part.ctx), l.host[e].p, device_ptr(src) + win.off,
                                         win.len * 8),
                  "window copy");
            l.src[e] = static_cast<const char*>(l.host[e].p);
            copied = true;
        }
        if (copied) check(cubit_copy_stream_sync(P.part.ctx, l.stream_for(P.part.ctx)), "window copies");
        return true;
    }
    void* stream = l.stream_for(P.part.ctx);
    // the device's verdict on the compaction bounds, once per partition before any of its window
    // copies (the copy stream starts after init_global's work, the narrowing included)
    std::call_once(P.overflow_checked, [&] {
        if (!P.d_overflow.p) return;
        std::vector<uint32_t> ov(n_emit);
        check(cubit_memcpy_d2h_stream(P.part.ctx, stream, ov.data(), P.d_overflow.p, ov.size() * 4), "overflow flags");
        for (size_t e = 0; e < ov.size(); ++e)
            if (ov[e]) P.width[e] = 0;
    });
    // validity words covering the window's rows [off, off + len) of the partition's output
    const uint64_t w0 = win.off / 64, w1 = (win.off + win.len + 63) / 64;
    l.valid_bit0 = w0 * 64;
    for (size_t e = 0; e < n_emit; ++e) {
        // page-locked memory is filed under no context: any partition's copies may use it
        if (!l.host[e].p) l.host[e].allocate(pinned_pool(), P.part.ctx, g.max_window * 8);
        if (P.nullable[e]) {
            // + 2 words: a window may start and end inside a word, and the chunk fill reads one ahead
            if (!l.host_valid[e].p) l.host_valid[e].allocate(pinned_pool(), P.part.ctx, (g.max_window / 64 + 3) * 8);
            check(cubit_memcpy_d2h_async(P.part.ctx, stream, l.host_valid[e].p,
                                         static_cast<const uint64_t*>(P.d_valid[e].p) + w0, (w1 - w0) * 8),
                  "window validity copy");
            l.src_valid[e] = static_cast<const uint64_t*>(l.host_valid[e].p);
        }
        l.src[e] = static_cast<const char*>(l.host[e].p);
        l.width[e] = P.width[e];
        if (P.width[e]) {
            const int wd = P.width[e];
            const char* src = static_cast<const char*>(P.d_narrow[e].p) + win.off * (uint64_t)wd;
            check(cubit_memcpy_d2h_async(P.part.ctx, stream, l.host[e].p, src, win.len * (uint64_t)wd), "window copy");
            continue;
        }
        PooledBuffer& src = g.column_ids[g.emit[e]] == COLUMN_IDENTIFIER_ROW_ID ? P.d_ids : P.d_cols[e];
        check(cubit_memcpy_d2h_async(P.part.ctx, stream, l.host[e].p, device_ptr(src) + win.off, win.len * 8),
              "window copy");
    }
    check(cubit_copy_stream_sync(P.part.ctx, stream), "window copies");  // one wait for the window's columns
    waited();
    return true;
}

// The chunk's mask from the window's validity words: rows [first, first + n) of the window
// copy (bit positions counted from its first word). Left all-valid when every row is valid, as
// a vector of a segment without NULLs (validity_mask.hpp: no buffer = all valid).
void FillValidity(const uint64_t* words, uint64_t first, idx_t n, ValidityMask& mask) {
    const uint64_t q = first / 64;
    const unsigned sh = (unsigned)(first % 64);
    uint64_t all = ~0ull;
    const idx_t nw = (n + 63) / 64;
    for (idx_t j = 0; j < nw; ++j) {
        uint64_t w = words[q + j] >> sh;
        if (sh) w |= words[q + j + 1] << (64 - sh);
        if (j == nw - 1 && (n & 63)) w |= ~0ull << (n & 63);  // rows past the chunk read as valid
        mask.words[j] = w;
        all &= w;
    }
    mask.all_valid = all == ~0ull;
}

template <typename U>
void widen(const U* __restrict__ src, int64_t off, idx_t n, int64_t* __restrict__ dst) {
    for (idx_t k = 0; k < n; ++k) dst[k] = off + (int64_t)src[k];
}

// three little-endian bytes per value; the buffers hold at least 8 bytes past the last value, so
// the wide loads of the last values stay inside them
void widen24_scalar(const uint8_t* __restrict__ src, int64_t off, idx_t n, int64_t* __restrict__ dst) {
    idx_t k = 0;
    for (; k + 4 <= n; k += 4) {  // four values from 12 bytes: two 8-byte loads
        uint64_t a, b;
        std::memcpy(&a, src + 3 * k, 8);
        std::memcpy(&b, src + 3 * k + 4, 8);
        dst[k] = off + (int64_t)(a & 0xffffff);
        dst[k + 1] = off + (int64_t)((a >> 24) & 0xffffff);
        dst[k + 2] = off + (int64_t)((b >> 16) & 0xffffff);
        dst[k + 3] = off + (int64_t)((b >> 40) & 0xffffff);
    }
    for (; k < n; ++k) {
        uint32_t v;
        std::memcpy(&v, src + 3 * k, 4);
        dst[k] = off + (int64_t)(v & 0xffffffu);
    }
}

// AVX2 (chosen at run time): 4 values per 16-byte load, byte-shuffled into 32-bit lanes and
// zero-extended to 64 — 1.75x the scalar form in a host microbenchmark
__attribute__((target("avx2"))) void widen24_avx2(const uint8_t* __restrict__ src, int64_t off, idx_t n,
                                                  int64_t* __restrict__ dst) {
    const __m128i shuf = _mm_setr_epi8(0, 1, 2, -1, 3, 4, 5, -1, 6, 7, 8, -1, 9, 10, 11, -1);
    const __m256i vo = _mm256_set1_epi64x(off);
    idx_t k = 0;
    for (; k + 8 <= n; k += 8) {  // reads bytes [3k, 3k + 28): at most 3n + 4
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + 3 * k));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + 3 * k + 12));
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + k),
                            _mm256_add_epi64(vo, _mm256_cvtepu32_epi64(_mm_shuffle_epi8(a, shuf))));
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + k + 4),
                            _mm256_add_epi64(vo, _mm256_cvtepu32_epi64(_mm_shuffle_epi8(b, shuf))));
    }
    widen24_scalar(src + 3 * k, off, n - k, dst + k);
}

void widen24(const uint8_t* __restrict__ src, int64_t off, idx_t n, int64_t* __restrict__ dst) {
    static const bool avx2 = __builtin_cpu_supports("avx2");
    if (avx2) widen24_avx2(src, off, n, dst);
    else widen24_scalar(src, off, n, dst);
}

void CubitScanFunc(TableFunctionInput& data, DataChunk& output) {
    auto& g = static_cast<CubitScanGlobalState&>(*data.global_state);
    auto& l = static_cast<CubitScanLocalState&>(*data.local_state);
    output.Reset();
    for (;;) {
        if (l.window < 0 && !NextWindow(g, l)) return;
        if ((size_t)l.window >= g.windows.size()) return;
        const Window& win = g.windows[l.window];
        const PartScan& P = *g.parts[win.part];
        if (l.pos >= win.len) {
            if (!NextWindow(g, l)) return;
            continue;
        }
        // a chunk of up to 2,048 of the window's rows: they are contiguous in the partition's
        // ordered output whatever tiles they come from, and one batch index covers the window
        const idx_t n = std::min<idx_t>(STANDARD_VECTOR_SIZE, win.len - l.pos);
        const idx_t at = l.pos;
        for (size_t e = 0; e < g.emit.size(); ++e) {
            if (P.nullable[e]) FillValidity(l.src_valid[e], win.off + at - l.valid_bit0, n, output.validity[e]);
            int64_t* dst = output.Column(e);
            const int64_t off = P.offset[e];
            switch (l.width[e]) {  // widen the compacted transfer
            case 1:
                widen(reinterpret_cast<const uint8_t*>(l.src[e]) + at, off, n, dst);
                break;
            case 2:
                widen(reinterpret_cast<const uint16_t*>(l.src[e]) + at, off, n, dst);
                break;
            case 3:
                widen24(reinterpret_cast<const uint8_t*>(l.src[e]) + 3 * at, off, n, dst);
                break;
            case 4:
                widen(reinterpret_cast<const uint32_t*>(l.src[e]) + at, off, n, dst);
                break;
            default:
                std::memcpy(dst, reinterpret_cast<const int64_t*>(l.src[e]) + at, n * sizeof(int64_t));
            }
        }
        l.pos += n;
        output.SetCardinality(n);
        return;
    }
}

// batch index = the partition's tile base + the window's first tile: one batch per window (a
// morsel, as seq_scan's batch is one row group, table_scan.cpp:179-189), so a chunk may hold rows
// of several tiles; a local state's batch indexes ascend (windows are claimed in order —
// partition by partition — and hold consecutive tiles), as PipelineExecutor::NextBatch requires
// (pipeline_executor.cpp:132)
idx_t CubitScanGetBatchIndex(const FunctionData*, LocalTableFunctionState* lstate, GlobalTableFunctionState* gstate) {
    auto& g = static_cast<CubitScanGlobalState&>(*gstate);
    auto& l = static_cast<CubitScanLocalState&>(*lstate);
    if (l.window < 0 || (size_t)l.window >= g.windows.size()) return 0;
    const PartScan& P = *g.parts[g.windows[l.window].part];
    return P.tile_base + P.tiles[g.windows[l.window].first];
}
double CubitScanProgress(const FunctionData*, const GlobalTableFunctionState* gstate) {
    auto& g = static_cast<const CubitScanGlobalState&>(*gstate);
    if (g.count == 0) return 100.0;
    return 100.0 * (double)g.emitted.load() / (double)g.count;
}

// TableScanCardinality (table_scan.cpp:201-208): NodeStatistics(table rows, table rows +
// transaction-local rows); transaction-local rows stay on the CPU, so both are
// the partitions' rows
NodeStatistics CubitScanCardinality(const FunctionData* bind_data) {
    auto& bind = static_cast<const CubitScanBindData&>(*bind_data);
    NodeStatistics st;
    st.has_estimated_cardinality = st.has_max_cardinality = true;
    st.estimated_cardinality = st.max_cardinality = bind.n_rows;
    return st;
}

// TableScanStatistics (table_scan.cpp:108-117) → DataTable::GetStatistics: none for the row id;
// over several partitions, the merge of theirs (BaseStatistics::Merge: min of mins, max of
// maxes over the partitions holding a valid value, either NULL flag)
bool CubitScanStatistics(const FunctionData* bind_data, column_t column_id, ColumnStatistics& out) {
    auto& bind = static_cast<const CubitScanBindData&>(*bind_data);
    if (column_id == COLUMN_IDENTIFIER_ROW_ID) return false;
    out = ColumnStatistics{};
    for (const CubitPartition& part : bind.parts) {
        int64_t mn = 0, mx = 0;
        int hn = 0, hv = 0, type = 0;
        const void* data = nullptr;
        check(cubit_table_column_statistics(part.table, (int)column_id, &mn, &mx, &hn, &hv),
              "cubit_table_column_statistics");
        check(cubit_table_column_data(part.table, (int)column_id, &data, &type), "cubit_table_column_data");
        if (hv) {
            // FLOAT / DOUBLE bounds are bit patterns: ordered by their comparison keys
            auto less = [type](int64_t a, int64_t b) { return cubit_fp_key(type, a) < cubit_fp_key(type, b); };
            out.min = out.has_no_null ? std::min(out.min, mn, less) : mn;
            out.max = out.has_no_null ? std::max(out.max, mx, less) : mx;
            out.has_no_null = true;
        }
        out.has_null = out.has_null || hn != 0;
    }
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

}  // extern "C"

namespace {

// The partitions of a scan, in row order: disjoint, ascending row ranges.
void bind_partitions(cubit_table* const* tables, uint32_t n_tables, CubitScanBindData& bind) {
    bind.parts.clear();
    bind.n_rows = 0;
    for (uint32_t i = 0; i < n_tables; ++i) {
        if (!tables[i]) throw ScanError(CUBIT_ERR_INVALID, "null partition");
        CubitPartition p;
        p.table = tables[i];
        check(cubit_table_info(tables[i], &p.n_rows, &p.row_base, &p.ctx), "cubit_table_info");
        if (!bind.parts.empty()) {
            const CubitPartition& q = bind.parts.back();
            if (p.row_base < q.row_base + (int64_t)q.n_rows)
                throw ScanError(CUBIT_ERR_INVALID, "partitions must hold disjoint row ranges in row order");
        }
        bind.n_rows += p.n_rows;
        bind.parts.push_back(p);
    }
}

}  // namespace

extern "C" {

int cubit_scan_init_global(cubit_table* table, const uint64_t* column_ids, uint32_t n_column_ids,
                           const uint64_t* projection_ids, uint32_t n_projection_ids, const cubit_filter_node* nodes,
                           uint32_t n_nodes, const cubit_txn* txn, cubit_scan** out) {
    if (!table) return scan_fail(CUBIT_ERR_INVALID, "null argument");
    return cubit_scan_init_global_multi(&table, 1, column_ids, n_column_ids, projection_ids, n_projection_ids, nodes,
                                        n_nodes, txn, out);
}

int cubit_scan_init_global_multi(cubit_table* const* tables, uint32_t n_tables, const uint64_t* column_ids,
                                 uint32_t n_column_ids, const uint64_t* projection_ids, uint32_t n_projection_ids,
                                 const cubit_filter_node* nodes, uint32_t n_nodes, const cubit_txn* txn,
                                 cubit_scan** out) {
    if (!tables || !n_tables || !out || (n_column_ids && !column_ids))
        return scan_fail(CUBIT_ERR_INVALID, "null argument");
    try {
        auto s = std::make_unique<cubit_scan>();
        s->fn = GetCubitScanFunction();
        bind_partitions(tables, n_tables, s->bind);
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

int cubit_scan_function_validity(cubit_scan* s, cubit_scan_local* l, int64_t* const* out_columns,
                                 uint64_t* const* out_validity, uint64_t* out_count) {
    if (!s || !l || !out_count) return scan_fail(CUBIT_ERR_INVALID, "null argument");
    try {
        TableFunctionInput in{&s->bind, l->lstate.get(), s->gstate.get()};
        l->chunk.external = out_columns;  // values go straight into the caller's vectors
        s->fn.function(in, l->chunk);
        l->chunk.external = nullptr;
    } catch (const ScanError& e) {
        l->chunk.external = nullptr;
        return scan_fail(e.code, e.what());
    }
    const idx_t n = l->chunk.size();
    for (size_t c = 0; c < l->chunk.data.size(); ++c) {
        if (out_validity && out_validity[c]) {
            const ValidityMask& m = l->chunk.validity[c];
            // the chunk's words; rows past n read as valid (the words past ⌈n / 64⌉ hold an earlier
            // chunk's bits)
            for (idx_t j = 0; j < STANDARD_VECTOR_SIZE / 64; ++j) {
                uint64_t w = m.all_valid || j * 64 >= n ? ~0ull : m.words[j];
                if (j * 64 < n && n - j * 64 < 64) w |= ~0ull << (n - j * 64);
                out_validity[c][j] = w;
            }
        }
    }
    *out_count = n;
    return CUBIT_OK;
}

int cubit_scan_function(cubit_scan* s, cubit_scan_local* l, int64_t* const* out_columns, uint64_t* out_count) {
    return cubit_scan_function_validity(s, l, out_columns, nullptr, out_count);
}

int cubit_scan_batch_index(cubit_scan* s, cubit_scan_local* l, uint64_t* out) {
    if (!s || !l || !out) return scan_fail(CUBIT_ERR_INVALID, "null argument");
    *out = s->fn.get_batch_index(&s->bind, l->lstate.get(), s->gstate.get());
    return CUBIT_OK;
}

int cubit_scan_decodes(cubit_scan* s, uint32_t* out) {
    if (!s || !out) return scan_fail(CUBIT_ERR_INVALID, "null argument");
    uint32_t n = 0;
    for (const auto& P : static_cast<CubitScanGlobalState*>(s->gstate.get())->parts) n += P->decodes;
    *out = n;
    return CUBIT_OK;
}

int cubit_scan_progress(cubit_scan* s, double* out) {
    if (!s || !out) return scan_fail(CUBIT_ERR_INVALID, "null argument");
    *out = s->fn.table_scan_progress(&s->bind, s->gstate.get());
    return CUBIT_OK;
}

// bind-time callbacks: the bind data is the partitions (no scan state needed)
int cubit_scan_cardinality(cubit_table* table, uint64_t* estimated, uint64_t* max) {
    if (!table) return scan_fail(CUBIT_ERR_INVALID, "null table");
    return cubit_scan_cardinality_multi(&table, 1, estimated, max);
}

int cubit_scan_cardinality_multi(cubit_table* const* tables, uint32_t n_tables, uint64_t* estimated, uint64_t* max) {
    if (!tables || !n_tables) return scan_fail(CUBIT_ERR_INVALID, "null table");
    try {
        CubitScanBindData bind;
        bind_partitions(tables, n_tables, bind);
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
    return cubit_scan_statistics_multi(&table, 1, column_id, min, max, has_null, has_no_null);
}

int cubit_scan_statistics_multi(cubit_table* const* tables, uint32_t n_tables, uint64_t column_id, int64_t* min,
                                int64_t* max, int* has_null, int* has_no_null) {
    if (!tables || !n_tables) return scan_fail(CUBIT_ERR_INVALID, "null table");
    try {
        CubitScanBindData bind;
        bind_partitions(tables, n_tables, bind);
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

int cubit_scan_release_cached(uint64_t* pinned_bytes, uint64_t* device_bytes) {
    if (pinned_bytes) *pinned_bytes = pinned_pool().cached();
    if (device_bytes) *device_bytes = device_pool().cached();
    pinned_pool().release_all();
    device_pool().release_all();
    return CUBIT_OK;
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
