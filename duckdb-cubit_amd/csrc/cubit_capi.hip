// C ABI of libcubitgpu.so (include/cubit_gpu.h) and the host-side planner that turns a
// DuckDB-style predicate tree (TableFilter mirror) into bitvector programs for the
// fused eval/decode kernel.
//
// Planner semantics (all exact; a leaf the index cannot answer exactly is built from the raw
// column — by the candidate check of its bin, or by K0 — never approximated):
//   range index, L(k) = {valid & v < k}:  v<c = L(c'), v<=c = L(c+1), v>c = NN∖L(c+1),
//     v>=c = NN∖L(c), v==c = L(c+1)∖L(c), v!=c = (NN∖L(c+1)) ∪ L(c); where L(c') is the
//     bitvector of the smallest key ≥ c when the index holds every distinct value. A
//     constant between keys k_lo < c < k_hi: v<c = L(k_lo) ∪ {r ∈ L(k_hi)∖L(k_lo) : v[r] < c}
//     (candidate check), v==c = {r ∈ L(k_hi)∖L(k_lo) : v[r] == c}.
//   equality index, E(k) = {v == k}: v==c = E(c), v!=c = NN∖E(c), ranges = ∪ E(k).
//   NULLs never satisfy a comparison (TemplatedFilterSelection HAS_NULL path,
//   column_segment.cpp:261-276) — NN is the column's validity bitvector.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <chrono>
#include <cmath>
#include <cstring>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <tuple>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../../include/cubit_gpu.h"
#include "cubit_internal.hpp"

using namespace cubit;

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_CHECK(expr)                                                                                  \
    do {                                                                                                 \
        hipError_t _e = (expr);                                                                          \
        if (_e != hipSuccess) return fail(CUBIT_ERR_HIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                                          __FILE__, __LINE__);                                           \
    } while (0)

}  // namespace

// ------------------------------------------------------------------ context

struct cubit_ctx {
    int device = 0;
    int n_cus = 256;
    hipStream_t stream = nullptr;
    bool timing = false;
    // one (start, stop) event pair per timed filter-kernel launch since the last reset
    std::vector<std::pair<hipEvent_t, hipEvent_t>> evs;
    size_t n_timed = 0;
    // tile directory of the last decode ({start, length} per tile) + ordered-pass scratch
    uint64_t* dir = nullptr;
    uint64_t* dst_off = nullptr;
    uint64_t dir_tiles = 0;
    uint32_t last_tiles = 0;
    uint64_t last_tile_rows = 0;
    int64_t* tmp_ids = nullptr;
    uint64_t tmp_cap = 0;
    int64_t* partials = nullptr;
    uint64_t* ticket = nullptr;  // claim ticket of the evaluate kernels (EvalArgs::ticket)
    uint64_t* flags = nullptr;   // look-back flag words of eval_decode_lookback (EvalArgs::flags)
    uint64_t epoch = 0;          // the last look-back launch's epoch (EvalArgs::epoch)
    uint32_t lookback_spins = 0; // EvalArgs::spin_limit (cubit_ctx_set_lookback_spins; 0 = default)
    int decode_kernel = CUBIT_DECODE_AUTO;  // cubit_ctx_set_decode_kernel
    int last_decode = 0;                    // kernel of the last decode (CUBIT_DECODE_PAIRS / _RUNS)
    // zonemap skip: the live-tile list of a launch, staged in page-locked memory and copied to
    // the device on the stream; live_ev marks the copy done before the staging is rewritten
    uint32_t* live_host = nullptr;
    uint32_t* live_dev = nullptr;
    uint64_t live_cap = 0;
    hipEvent_t live_ev = nullptr;
    bool live_pending = false;
    // cubit_ctx_set_repeat: the next decode launch is issued `repeat` times back to back
    // between two stream events (rep_ev); rep_launches of them went into the last measurement
    uint32_t repeat = 0;
    uint32_t rep_launches = 0;
    hipEvent_t rep_ev[2] = {nullptr, nullptr};
    // copy streams handed back by cubit_copy_stream_destroy, each with its ordering event
    // (creating a HIP stream costs milliseconds; the table function's tasks take one per scan)
    std::vector<std::pair<hipStream_t, hipEvent_t>> copy_pool;
    std::unordered_map<hipStream_t, hipEvent_t> copy_live;
    // copy events (cubit_copy_event_record): handed out and returned through a pool
    std::vector<hipEvent_t> copy_ev_pool;
    std::unordered_set<hipEvent_t> copy_ev_live;
    std::recursive_mutex mu;     // CUBIT_LOCK
};

namespace {

// Every entry point that reads or changes a context's state (its stream, claim ticket, tile
// directory, timing events, tables) holds the context's mutex, so DuckDB pipeline threads
// may share one context; results named "last" belong to its most recent call.
#define CUBIT_LOCK(c) std::lock_guard<std::recursive_mutex> cubit_lock_((c)->mu)

int ensure_dir(cubit_ctx* ctx, uint64_t tiles) {
    if (tiles <= ctx->dir_tiles && ctx->dir) return CUBIT_OK;
    if (ctx->dir) HIP_CHECK(hipFree(ctx->dir));
    if (ctx->dst_off) HIP_CHECK(hipFree(ctx->dst_off));
    ctx->dir = ctx->dst_off = nullptr;
    const uint64_t want = std::max<uint64_t>(tiles, 1024);
    if (hipMalloc(&ctx->dir, 2 * want * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc(&ctx->dst_off, want * sizeof(uint64_t)) != hipSuccess)
        return fail(CUBIT_ERR_OOM, "tile directory allocation of %llu tiles failed", (unsigned long long)want);
    ctx->dir_tiles = want;
    return CUBIT_OK;
}

int ensure_tmp(cubit_ctx* ctx, uint64_t cap) {
    if (cap <= ctx->tmp_cap && ctx->tmp_ids) return CUBIT_OK;
    if (ctx->tmp_ids) HIP_CHECK(hipFree(ctx->tmp_ids));
    ctx->tmp_ids = nullptr;
    if (hipMalloc(&ctx->tmp_ids, std::max<uint64_t>(cap, 1) * sizeof(int64_t)) != hipSuccess)
        return fail(CUBIT_ERR_OOM, "ordered-pass scratch of %llu ids failed", (unsigned long long)cap);
    ctx->tmp_cap = cap;
    return CUBIT_OK;
}

int set_device(cubit_ctx* ctx) {
    HIP_CHECK(hipSetDevice(ctx->device));
    return CUBIT_OK;
}

// Start/stop events for the next timed kernel (stamped by its dispatch through
// hipExtLaunchKernelGGL); both stay null when timing is off.
int timing_events(cubit_ctx* ctx, hipEvent_t& start, hipEvent_t& stop) {
    start = stop = nullptr;
    if (!ctx->timing) return CUBIT_OK;
    if (ctx->n_timed == ctx->evs.size()) {
        // timing-only events: no system-scope release when they are recorded, so a stamp does
        // not wait for an L2 writeback of the kernel's dirty lines (HIP documents this for
        // timing accuracy on AMD devices). Measured: the stamped mean stays 2-4 % above
        // rocprofv3's kernel trace (73.7 vs 71.1 µs at SF100 Q6), as with default events.
        // Results stay ordered by the stream; readers synchronise on it.
        hipEvent_t e0, e1;
        HIP_CHECK(hipEventCreateWithFlags(&e0, hipEventDisableSystemFence));
        HIP_CHECK(hipEventCreateWithFlags(&e1, hipEventDisableSystemFence));
        ctx->evs.emplace_back(e0, e1);
    }
    start = ctx->evs[ctx->n_timed].first;
    stop = ctx->evs[ctx->n_timed].second;
    ctx->n_timed++;
    return CUBIT_OK;
}

// Stage the live-tile list of a zonemap-skipping launch on the device (asynchronous on the
// context stream): zone z becomes tiles z·per_zone … z·per_zone + per_zone - 1 of the kernel.
int upload_live(cubit_ctx* ctx, const std::vector<uint32_t>& zones, uint32_t per_zone, const uint32_t** d_live,
                uint32_t* n_live) {
    const uint64_t n = (uint64_t)zones.size() * per_zone;
    if (ctx->live_pending) {  // the previous list's copy must be done before its staging is reused
        HIP_CHECK(hipEventSynchronize(ctx->live_ev));
        ctx->live_pending = false;
    }
    if (n > ctx->live_cap) {
        if (ctx->live_dev) HIP_CHECK(hipFree(ctx->live_dev));
        if (ctx->live_host) HIP_CHECK(hipHostFree(ctx->live_host));
        ctx->live_dev = nullptr;
        ctx->live_host = nullptr;
        ctx->live_cap = 0;
        const uint64_t cap = std::max<uint64_t>(n, 4096);
        if (hipMalloc(&ctx->live_dev, cap * 4) != hipSuccess || hipHostMalloc(&ctx->live_host, cap * 4) != hipSuccess)
            return fail(CUBIT_ERR_OOM, "live-tile list of %llu tiles failed", (unsigned long long)cap);
        ctx->live_cap = cap;
    }
    if (!ctx->live_ev) HIP_CHECK(hipEventCreateWithFlags(&ctx->live_ev, hipEventDisableTiming));
    uint64_t k = 0;
    for (uint32_t z : zones)
        for (uint32_t j = 0; j < per_zone; ++j) ctx->live_host[k++] = z * per_zone + j;
    HIP_CHECK(hipMemcpyAsync(ctx->live_dev, ctx->live_host, n * 4, hipMemcpyHostToDevice, ctx->stream));
    HIP_CHECK(hipEventRecord(ctx->live_ev, ctx->stream));
    ctx->live_pending = true;
    *d_live = ctx->live_dev;
    *n_live = (uint32_t)n;
    return CUBIT_OK;
}

enum class RunMode { kDecode, kCount };

// Launch the evaluator over a compiled program (asynchronous on the context stream).
//   kDecode: row ids as per-tile ascending runs + tile directory (ordered = lay them out in
//            row order: the look-back decode writes them so, up to kLookbackMaxTiles tiles;
//            past that, one extra pass); kCount: count(*) and/or result words.
// live_zones (optional, non-empty, ascending): evaluate only these zones (zonemap skip); the
// other tiles hold no qualifying row. Not with result_words (the skipped words stay unwritten).
int run_eval(cubit_ctx* ctx, const EvalProgram& prog, uint64_t n_rows, int64_t row_base, int64_t* rowids,
             uint64_t capacity, uint64_t* d_count, uint64_t* result_words, RunMode mode, bool timed = false,
             bool ordered = false, bool check_capacity = false, const std::vector<uint32_t>* live_zones = nullptr,
             const uint64_t* tile_prefix = nullptr) {
    // the directory describes only the decode launched here: a count, a failed launch or a
    // folded-away filter leaves no tiles behind for cubit_ctx_last_tiles to hand out
    ctx->last_tiles = 0;
    // the claim ticket carries row sums in 48 bits (finish_ticket)
    if (n_rows >= (1ull << 47)) return fail(CUBIT_ERR_INVALID, "%llu rows exceed 2^47", (unsigned long long)n_rows);
    EvalArgs a{};
    a.prog = prog;
    a.n_rows = n_rows;
    a.n_words = (n_rows + 63) / 64;
    a.row_base = row_base;
    a.count = d_count;
    a.result_words = result_words;
    a.ticket = ctx->ticket;
    const uint64_t pw = padded_words(n_rows);
    if (live_zones && (live_zones->empty() || result_words)) live_zones = nullptr;
    hipEvent_t start = nullptr, stop = nullptr;
    if (timed)
        if (int rc = timing_events(ctx, start, stop)) return rc;
    if (mode == RunMode::kCount) {
        a.num_tiles = (uint32_t)(pw / count_tile_words(prog.n_leaves));
        if (live_zones) {
            uint32_t n_live = 0;
            if (int rc = upload_live(ctx, *live_zones, (uint32_t)(kZoneWords / count_tile_words(prog.n_leaves)),
                                     &a.live, &n_live))
                return rc;
            a.num_tiles = n_live;
        }
        HIP_CHECK(launch_eval_count(a, ctx->stream, start, stop));
        return CUBIT_OK;
    }
    // the tiles that hold rows (the padding past the last word needs no workgroup); the
    // directory is sized for every padded tile, as a live-tile list may name any of them
    const uint64_t tiles = (a.n_words + decode_tile_words() - 1) / decode_tile_words();
    if (int rc = ensure_dir(ctx, pw / decode_tile_words())) return rc;
    // per-tile offsets known up front (tile_prefix): the look-back kernel without its walk, at any
    // size, unless another kernel is forced; an ordered scan takes the look-back decode (runs in
    // tile order) unless a kernel is forced
    const bool prefixed = tile_prefix && rowids && (ctx->decode_kernel == 0 || ctx->decode_kernel == 3);
    const int kernel = prefixed || (ordered && rowids && ctx->decode_kernel == 0 && tiles <= kLookbackMaxTiles)
                           ? 3
                           : ctx->decode_kernel;
    const bool order_pass = ordered && rowids && !(kernel == 3 && (prefixed || tiles <= kLookbackMaxTiles));
    if (order_pass)
        if (int rc = ensure_tmp(ctx, capacity)) return rc;
    a.num_tiles = (uint32_t)tiles;
    a.flags = ctx->flags;
    a.epoch = ++ctx->epoch;
    a.spin_limit = ctx->lookback_spins;
    a.tile_prefix = prefixed ? tile_prefix : nullptr;
    a.rowids = order_pass ? ctx->tmp_ids : rowids;
    a.capacity = rowids ? capacity : 0;
    if (live_zones) {
        static_assert(kZoneWords == 2048, "a zone is one decode tile");
        uint32_t n_live = 0;
        if (int rc = upload_live(ctx, *live_zones, 1, &a.live, &n_live)) return rc;
        a.num_tiles = n_live;
        // skipped tiles hold no rows: their directory entries are {0, 0}
        HIP_CHECK(hipMemsetAsync(ctx->dir, 0, 2 * tiles * sizeof(uint64_t), ctx->stream));
    }
    // persistent grid: two 512-thread workgroups per CU (VGPR-limited to 4 waves per SIMD).
    // Between one and two tiles per workgroup, every workgroup takes a whole pair instead
    // (grid = tiles / 2): the same critical path (one pair), a third fewer claims queued on
    // the ticket word at once (768 tiles: 384 instead of 512, ≈11 ns each).
    const uint64_t work = a.num_tiles;
    const uint64_t max_grid = (uint64_t)ctx->n_cus * 2;
    // (a grid of ceil(work / ceil(work / max_grid)) workgroups, every one the same number of tiles,
    // measured slower: SF100 / 4 18.5 -> 21.0 µs, fewer workgroups than the last round's leave HBM
    // unsaturated; profiles/r06k_balanced_grid_not_kept.txt)
    const unsigned grid = (unsigned)(work <= max_grid ? work : work <= 2 * max_grid ? (work + 1) / 2 : max_grid);
    if (tiles == 0) {  // no row: the count is 0 and no kernel runs
        if (start) ctx->n_timed--;
        HIP_CHECK(hipMemsetAsync(d_count, 0, sizeof(uint64_t), ctx->stream));
        ctx->last_decode = 0;
        return CUBIT_OK;
    }
    if (ctx->repeat) {
        // steady-state kernel time: the same launch `repeat` times back to back, bracketed by two
        // stream events (a dispatch-stamped pair adds a marker and its gap to each sample). Every
        // repeat rewrites the same outputs from the same inputs; the look-back takes a new epoch.
        if (start) {
            ctx->n_timed--;
            start = stop = nullptr;
        }
        if (!ctx->rep_ev[0]) {
            HIP_CHECK(hipEventCreate(&ctx->rep_ev[0]));
            HIP_CHECK(hipEventCreate(&ctx->rep_ev[1]));
        }
        HIP_CHECK(hipEventRecord(ctx->rep_ev[0], ctx->stream));
        for (uint32_t i = 1; i < ctx->repeat; ++i) {
            HIP_CHECK(launch_eval_decode(a, ctx->dir, grid, ctx->stream, nullptr, nullptr, kernel, ctx->n_cus));
            a.epoch = ++ctx->epoch;
        }
    }
    HIP_CHECK(launch_eval_decode(a, ctx->dir, grid, ctx->stream, start, stop, kernel, ctx->n_cus));
    if (ctx->repeat) {
        HIP_CHECK(hipEventRecord(ctx->rep_ev[1], ctx->stream));
        ctx->rep_launches = ctx->repeat;
        ctx->repeat = 0;
    }
    ctx->last_decode = prefixed && prog.n_leaves == 1
                           ? CUBIT_DECODE_PREFIXED
                           : decode_kernel_for(prog.n_leaves, a.num_tiles, grid, kernel, a.live != nullptr, ctx->n_cus,
                                               prefixed);
    ctx->last_tiles = (uint32_t)tiles;
    ctx->last_tile_rows = decode_tile_words() * 64;
    if (order_pass)
        HIP_CHECK(launch_order_runs(ctx->dir, (uint32_t)tiles, ctx->dst_off, ctx->tmp_ids, capacity, rowids,
                                    ctx->stream));
    if (check_capacity && rowids) {
        uint64_t n = 0;
        HIP_CHECK(hipMemcpyAsync(&n, d_count, sizeof(n), hipMemcpyDeviceToHost, ctx->stream));
        HIP_CHECK(hipStreamSynchronize(ctx->stream));
        if (n > capacity)
            return fail(CUBIT_ERR_CAPACITY, "%llu qualifying rows exceed the capacity of %llu row ids",
                        (unsigned long long)n, (unsigned long long)capacity);
    }
    return CUBIT_OK;
}

}  // namespace

extern "C" {

int cubit_abi_version(void) { return 1; }
int cubit_vector_size(void) { return (int)kVectorSize; }
int cubit_row_group_size(void) { return (int)kRowGroupSize; }
uint64_t cubit_padded_words(uint64_t n_rows) { return padded_words(n_rows); }
const char* cubit_last_error(void) { return g_last_error.c_str(); }

int cubit_device_count(int* n) {
    if (!n) return fail(CUBIT_ERR_INVALID, "null argument");
    HIP_CHECK(hipGetDeviceCount(n));
    return CUBIT_OK;
}

int cubit_ctx_create(int device, cubit_ctx** out) {
    if (!out) return fail(CUBIT_ERR_INVALID, "out is null");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(CUBIT_ERR_HIP, "no HIP device visible");
    if (device < 0 || device >= n) return fail(CUBIT_ERR_INVALID, "device %d out of range (%d devices)", device, n);
    HIP_CHECK(hipSetDevice(device));
    auto* ctx = new cubit_ctx();
    ctx->device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        ctx->n_cus = prop.multiProcessorCount;
    if (hipMalloc(&ctx->partials, 2 * kSumBlocks * sizeof(int64_t)) != hipSuccess ||
        hipMalloc(&ctx->ticket, kTicketWords * sizeof(uint64_t)) != hipSuccess ||
        hipMemset(ctx->ticket, 0, kTicketWords * sizeof(uint64_t)) != hipSuccess ||
        hipMalloc(&ctx->flags, kLookbackMaxTiles * sizeof(uint64_t)) != hipSuccess ||
        hipMemset(ctx->flags, 0, kLookbackMaxTiles * sizeof(uint64_t)) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
        if (ctx->partials) (void)hipFree(ctx->partials);
        if (ctx->ticket) (void)hipFree(ctx->ticket);
        if (ctx->flags) (void)hipFree(ctx->flags);
        delete ctx;
        return fail(CUBIT_ERR_OOM, "context workspace allocation failed");
    }
    *out = ctx;
    return CUBIT_OK;
}

int cubit_ctx_destroy(cubit_ctx* ctx) {
    if (!ctx) return CUBIT_OK;
    (void)hipSetDevice(ctx->device);
    if (ctx->dir) (void)hipFree(ctx->dir);
    if (ctx->dst_off) (void)hipFree(ctx->dst_off);
    if (ctx->tmp_ids) (void)hipFree(ctx->tmp_ids);
    if (ctx->partials) (void)hipFree(ctx->partials);
    if (ctx->ticket) (void)hipFree(ctx->ticket);
    if (ctx->flags) (void)hipFree(ctx->flags);
    if (ctx->live_pending) (void)hipEventSynchronize(ctx->live_ev);
    if (ctx->live_dev) (void)hipFree(ctx->live_dev);
    if (ctx->live_host) (void)hipHostFree(ctx->live_host);
    if (ctx->live_ev) (void)hipEventDestroy(ctx->live_ev);
    for (hipEvent_t e : ctx->rep_ev)
        if (e) (void)hipEventDestroy(e);
    for (auto& se : ctx->copy_live) ctx->copy_pool.push_back(se);
    for (auto& se : ctx->copy_pool) {
        (void)hipStreamDestroy(se.first);
        (void)hipEventDestroy(se.second);
    }
    for (hipEvent_t e : ctx->copy_ev_live) (void)hipEventDestroy(e);
    for (hipEvent_t e : ctx->copy_ev_pool) (void)hipEventDestroy(e);
    for (auto& e : ctx->evs) {
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    delete ctx;
    return CUBIT_OK;
}

int cubit_ctx_set_stream(cubit_ctx* ctx, void* stream) {
    if (!ctx) return fail(CUBIT_ERR_INVALID, "ctx is null");
    CUBIT_LOCK(ctx);
    hipStream_t next = static_cast<hipStream_t>(stream);
    if (next != ctx->stream) {
        // the claim ticket, tile directory, scratch ids and partials are re-armed / reused in
        // stream order: a launch still in flight on the old stream must finish before the
        // first launch on the new one
        if (int rc = set_device(ctx)) return rc;
        HIP_CHECK(hipStreamSynchronize(ctx->stream));
    }
    ctx->stream = next;
    return CUBIT_OK;
}

int cubit_ctx_set_decode_kernel(cubit_ctx* ctx, int kernel) {
    if (!ctx) return fail(CUBIT_ERR_INVALID, "null context");
    if (kernel < CUBIT_DECODE_AUTO || kernel > CUBIT_DECODE_LOOKBACK) return fail(CUBIT_ERR_INVALID, "decode kernel %d", kernel);
    CUBIT_LOCK(ctx);
    ctx->decode_kernel = kernel;
    return CUBIT_OK;
}

int cubit_ctx_set_lookback_spins(cubit_ctx* ctx, uint32_t spins) {
    if (!ctx) return fail(CUBIT_ERR_INVALID, "null context");
    CUBIT_LOCK(ctx);
    ctx->lookback_spins = spins;
    return CUBIT_OK;
}

int cubit_ctx_last_decode_kernel(cubit_ctx* ctx, int* kernel) {
    if (!ctx || !kernel) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(ctx);
    *kernel = ctx->last_decode;
    return CUBIT_OK;
}

int cubit_ctx_enable_timing(cubit_ctx* ctx, int on) {
    if (!ctx) return fail(CUBIT_ERR_INVALID, "ctx is null");
    CUBIT_LOCK(ctx);
    ctx->timing = on != 0;
    return CUBIT_OK;
}

int cubit_last_kernel_ms(cubit_ctx* ctx, float* ms) {
    if (!ctx || !ms) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(ctx);
    if (ctx->n_timed == 0) return fail(CUBIT_ERR_INVALID, "no timed kernel recorded (enable timing first)");
    const auto& e = ctx->evs[ctx->n_timed - 1];
    HIP_CHECK(hipEventSynchronize(e.second));
    HIP_CHECK(hipEventElapsedTime(ms, e.first, e.second));
    return CUBIT_OK;
}

int cubit_ctx_timing_reset(cubit_ctx* ctx) {
    if (!ctx) return fail(CUBIT_ERR_INVALID, "ctx is null");
    CUBIT_LOCK(ctx);
    ctx->n_timed = 0;
    return CUBIT_OK;
}

int cubit_ctx_kernel_times(cubit_ctx* ctx, float* ms, uint32_t cap, uint32_t* n) {
    if (!ctx || !n) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(ctx);
    const uint32_t m = (uint32_t)std::min<size_t>(cap, ctx->n_timed);
    for (uint32_t i = 0; i < m; ++i) {
        HIP_CHECK(hipEventSynchronize(ctx->evs[i].second));
        HIP_CHECK(hipEventElapsedTime(&ms[i], ctx->evs[i].first, ctx->evs[i].second));
    }
    *n = (uint32_t)ctx->n_timed;
    return CUBIT_OK;
}

int cubit_ctx_set_repeat(cubit_ctx* ctx, uint32_t reps) {
    if (!ctx) return fail(CUBIT_ERR_INVALID, "ctx is null");
    if (reps > 100000) return fail(CUBIT_ERR_INVALID, "%u repeats", reps);
    CUBIT_LOCK(ctx);
    ctx->repeat = reps;
    return CUBIT_OK;
}

int cubit_ctx_repeat_time(cubit_ctx* ctx, double* ms_per_launch, uint32_t* launches) {
    if (!ctx || !ms_per_launch) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(ctx);
    if (!ctx->rep_launches) return fail(CUBIT_ERR_INVALID, "no repeated decode launch recorded (cubit_ctx_set_repeat)");
    if (int rc = set_device(ctx)) return rc;
    HIP_CHECK(hipEventSynchronize(ctx->rep_ev[1]));
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, ctx->rep_ev[0], ctx->rep_ev[1]));
    *ms_per_launch = (double)ms / ctx->rep_launches;
    if (launches) *launches = ctx->rep_launches;
    return CUBIT_OK;
}

int cubit_dev_alloc(cubit_ctx* ctx, uint64_t bytes, void** dptr) {
    if (!ctx || !dptr) return fail(CUBIT_ERR_INVALID, "null argument");
    if (int rc = set_device(ctx)) return rc;
    if (hipMalloc(dptr, std::max<uint64_t>(bytes, 16)) != hipSuccess)
        return fail(CUBIT_ERR_OOM, "hipMalloc(%llu) failed", (unsigned long long)bytes);
    return CUBIT_OK;
}

int cubit_dev_free(cubit_ctx* ctx, void* dptr) {
    if (!ctx) return fail(CUBIT_ERR_INVALID, "ctx is null");
    if (dptr) HIP_CHECK(hipFree(dptr));
    return CUBIT_OK;
}

int cubit_host_alloc(cubit_ctx* ctx, uint64_t bytes, void** hptr) {
    if (!ctx || !hptr) return fail(CUBIT_ERR_INVALID, "null argument");
    if (int rc = set_device(ctx)) return rc;
    // portable: the table function's pinned pool serves copies from every device's partitions
    if (hipHostMalloc(hptr, std::max<uint64_t>(bytes, 16), hipHostMallocPortable) != hipSuccess)
        return fail(CUBIT_ERR_OOM, "hipHostMalloc(%llu) failed", (unsigned long long)bytes);
    return CUBIT_OK;
}

int cubit_host_free(cubit_ctx* ctx, void* hptr) {
    (void)ctx;  // page-locked memory is not tied to a context: NULL is accepted
    if (hptr) HIP_CHECK(hipHostFree(hptr));
    return CUBIT_OK;
}

int cubit_memcpy_h2d(cubit_ctx* ctx, void* dst, const void* src, uint64_t bytes) {
    if (!ctx) return fail(CUBIT_ERR_INVALID, "ctx is null");
    HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return CUBIT_OK;
}

int cubit_memcpy_d2h(cubit_ctx* ctx, void* dst, const void* src, uint64_t bytes) {
    if (!ctx) return fail(CUBIT_ERR_INVALID, "ctx is null");
    HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return CUBIT_OK;
}

int cubit_copy_stream_create(cubit_ctx* ctx, void** stream) {
    if (!ctx || !stream) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(ctx);
    if (int rc = set_device(ctx)) return rc;
    std::pair<hipStream_t, hipEvent_t> se{nullptr, nullptr};
    if (!ctx->copy_pool.empty()) {
        se = ctx->copy_pool.back();
        ctx->copy_pool.pop_back();
    } else {
        HIP_CHECK(hipStreamCreateWithFlags(&se.first, hipStreamNonBlocking));
        if (hipEventCreateWithFlags(&se.second, hipEventDisableTiming) != hipSuccess) {
            (void)hipStreamDestroy(se.first);
            return fail(CUBIT_ERR_DEVICE, "copy stream: event creation failed");
        }
    }
    ctx->copy_live[se.first] = se.second;
    // the stream starts behind the context stream's enqueued work (the scan and its probes)
    HIP_CHECK(hipEventRecord(se.second, ctx->stream));
    HIP_CHECK(hipStreamWaitEvent(se.first, se.second, 0));
    *stream = se.first;
    return CUBIT_OK;
}

int cubit_copy_stream_destroy(cubit_ctx* ctx, void* stream) {
    if (!ctx) return fail(CUBIT_ERR_INVALID, "ctx is null");
    if (!stream) return CUBIT_OK;
    CUBIT_LOCK(ctx);
    auto it = ctx->copy_live.find(static_cast<hipStream_t>(stream));
    if (it == ctx->copy_live.end()) return fail(CUBIT_ERR_INVALID, "not a copy stream of this context");
    if (int rc = set_device(ctx)) return rc;
    HIP_CHECK(hipStreamSynchronize(it->first));  // its copies are done before another task reuses it
    ctx->copy_pool.push_back(*it);
    ctx->copy_live.erase(it);
    return CUBIT_OK;
}

int cubit_memcpy_d2h_stream(cubit_ctx* ctx, void* stream, void* dst, const void* src, uint64_t bytes) {
    if (!ctx || !stream) return fail(CUBIT_ERR_INVALID, "null argument");
    if (int rc = set_device(ctx)) return rc;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    return CUBIT_OK;
}

int cubit_memcpy_d2h_async(cubit_ctx* ctx, void* stream, void* dst, const void* src, uint64_t bytes) {
    if (!ctx || !stream) return fail(CUBIT_ERR_INVALID, "null argument");
    if (int rc = set_device(ctx)) return rc;
    HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, static_cast<hipStream_t>(stream)));
    return CUBIT_OK;
}

int cubit_copy_stream_sync(cubit_ctx* ctx, void* stream) {
    if (!ctx || !stream) return fail(CUBIT_ERR_INVALID, "null argument");
    if (int rc = set_device(ctx)) return rc;
    HIP_CHECK(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    return CUBIT_OK;
}

int cubit_copy_event_record(cubit_ctx* ctx, void* stream, void** event) {
    if (!ctx || !event) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(ctx);
    if (int rc = set_device(ctx)) return rc;
    hipEvent_t e = nullptr;
    if (!ctx->copy_ev_pool.empty()) {
        e = ctx->copy_ev_pool.back();
        ctx->copy_ev_pool.pop_back();
    } else {
        HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    ctx->copy_ev_live.insert(e);
    HIP_CHECK(hipEventRecord(e, stream ? static_cast<hipStream_t>(stream) : ctx->stream));
    *event = e;
    return CUBIT_OK;
}

int cubit_copy_stream_wait_event(cubit_ctx* ctx, void* stream, void* event) {
    if (!ctx || !stream || !event) return fail(CUBIT_ERR_INVALID, "null argument");
    if (int rc = set_device(ctx)) return rc;
    HIP_CHECK(hipStreamWaitEvent(static_cast<hipStream_t>(stream), static_cast<hipEvent_t>(event), 0));
    return CUBIT_OK;
}

int cubit_copy_event_sync(cubit_ctx* ctx, void* event) {
    if (!ctx || !event) return fail(CUBIT_ERR_INVALID, "null argument");
    if (int rc = set_device(ctx)) return rc;
    HIP_CHECK(hipEventSynchronize(static_cast<hipEvent_t>(event)));
    return CUBIT_OK;
}

int cubit_copy_event_destroy(cubit_ctx* ctx, void* event) {
    if (!ctx) return fail(CUBIT_ERR_INVALID, "ctx is null");
    if (!event) return CUBIT_OK;
    CUBIT_LOCK(ctx);
    auto it = ctx->copy_ev_live.find(static_cast<hipEvent_t>(event));
    if (it == ctx->copy_ev_live.end()) return fail(CUBIT_ERR_INVALID, "not a copy event of this context");
    if (int rc = set_device(ctx)) return rc;
    HIP_CHECK(hipEventSynchronize(*it));  // its copies are done before the event is reused
    ctx->copy_ev_pool.push_back(*it);
    ctx->copy_ev_live.erase(it);
    return CUBIT_OK;
}

int cubit_memset_d(cubit_ctx* ctx, void* dst, int value, uint64_t bytes) {
    if (!ctx) return fail(CUBIT_ERR_INVALID, "ctx is null");
    HIP_CHECK(hipMemsetAsync(dst, value, bytes, ctx->stream));
    return CUBIT_OK;
}

int cubit_memcpy_d2d(cubit_ctx* ctx, void* dst, const void* src, uint64_t bytes) {
    if (!ctx || ((!dst || !src) && bytes)) return fail(CUBIT_ERR_INVALID, "null argument");
    if (!bytes) return CUBIT_OK;
    HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    return CUBIT_OK;
}

int cubit_ctx_check(cubit_ctx* ctx) {
    if (!ctx) return fail(CUBIT_ERR_INVALID, "ctx is null");
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    HIP_CHECK(hipGetLastError());
    return CUBIT_OK;
}

int cubit_ctx_last_tiles(cubit_ctx* ctx, const uint64_t** d_dir, uint32_t* n_tiles, uint64_t* rows_per_tile) {
    if (!ctx) return fail(CUBIT_ERR_INVALID, "ctx is null");
    CUBIT_LOCK(ctx);
    if (d_dir) *d_dir = ctx->dir;
    if (n_tiles) *n_tiles = ctx->last_tiles;
    if (rows_per_tile) *rows_per_tile = ctx->last_tile_rows;
    return CUBIT_OK;
}

int cubit_sync(cubit_ctx* ctx) {
    if (!ctx) return fail(CUBIT_ERR_INVALID, "ctx is null");
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return CUBIT_OK;
}

int cubit_build_bitvector(cubit_ctx* ctx, const void* d_col, int type, const uint64_t* d_validity, uint64_t n_rows,
                          int cmp, int64_t constant, uint64_t* d_words) {
    if (!ctx || !d_col || !d_words) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(ctx);
    if (type != CUBIT_TYPE_INT32 && type != CUBIT_TYPE_INT64 && !type_is_keyed(type))
        return fail(CUBIT_ERR_UNSUPPORTED, "type %d", type);
    if (cmp < 0 || cmp > 5) return fail(CUBIT_ERR_INVALID, "cmp %d", cmp);
    HIP_CHECK(launch_compare_bitvector(d_col, type, d_validity, n_rows, cmp, value_key(type, constant), d_words,
                                       ctx->stream));
    return CUBIT_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ program compilation

namespace {

// Expression over bitvectors. Leaves carry the row predicate they encode so that MVCC
// update patches can recompute a row's bit from its visible value.
struct Leaf {
    const uint64_t* bv = nullptr;
    int column = -1;  // -1: not derived from a column value (visibility, temp)
    int pred = 0;     // 0 = cmp (v CMP c), 1 = valid (NN), 2 = bin (c <= v < constant2)
    int cmp = 0;
    int64_t constant = 0;
    int64_t constant2 = 0;
    // where its zone classes (zonemaps) come from: kZoneBits = bv is a table-owned index leaf or
    // validity bitvector, classified from its own bits; kZoneStats = bv holds exactly the valid
    // rows whose base value passes (cmp, constant) — a K0 or candidate-check leaf — classified
    // from the column's per-zone min / max like a ConstantFilter's CheckStatistics; kZoneNone
    // = visibility and materialised leaves (mixed everywhere)
    int zsrc = 0;
    // a leaf patched with MVCC updates keeps the classes of the base leaf it was copied from
    // (zbv: that bitvector, for kZoneBits) except in the zones that hold an update record of
    // column zdirty (there: mixed)
    const uint64_t* zbv = nullptr;
    int zdirty = -1;
};
enum { kZoneNone = 0, kZoneBits = 1, kZoneStats = 2 };

struct Expr;
using ExprP = std::shared_ptr<Expr>;
struct Expr {
    enum Kind { LEAF, AND, OR, ANDNOT, CONST_TRUE, CONST_FALSE } kind = CONST_FALSE;
    Leaf leaf;
    bool neg = false;  // LEAF only
    ExprP a, b;
};

ExprP mk_true() {
    auto e = std::make_shared<Expr>();
    e->kind = Expr::CONST_TRUE;
    return e;
}
ExprP mk_false() {
    auto e = std::make_shared<Expr>();
    e->kind = Expr::CONST_FALSE;
    return e;
}
ExprP mk_leaf(const Leaf& l, bool neg = false) {
    auto e = std::make_shared<Expr>();
    e->kind = Expr::LEAF;
    e->leaf = l;
    e->neg = neg;
    return e;
}
ExprP mk_not(const ExprP& x);
ExprP mk_bin(Expr::Kind k, ExprP a, ExprP b) {
    using K = Expr::Kind;
    const bool at = a->kind == K::CONST_TRUE, af = a->kind == K::CONST_FALSE;
    const bool bt = b->kind == K::CONST_TRUE, bf = b->kind == K::CONST_FALSE;
    switch (k) {
    case K::AND:
        if (af || bf) return mk_false();
        if (at) return b;
        if (bt) return a;
        break;
    case K::OR:
        if (at || bt) return mk_true();
        if (af) return b;
        if (bf) return a;
        break;
    case K::ANDNOT:
        if (af || bt) return mk_false();
        if (bf) return a;
        if (at) return mk_not(b);
        break;
    default:
        break;
    }
    auto e = std::make_shared<Expr>();
    e->kind = k;
    e->a = std::move(a);
    e->b = std::move(b);
    return e;
}
// NOT pushed to the leaves (De Morgan); ANDNOT(a,b) = a & ~b → ~a | b
ExprP mk_not(const ExprP& x) {
    using K = Expr::Kind;
    switch (x->kind) {
    case K::CONST_TRUE: return mk_false();
    case K::CONST_FALSE: return mk_true();
    case K::LEAF: return mk_leaf(x->leaf, !x->neg);
    case K::AND: return mk_bin(K::OR, mk_not(x->a), mk_not(x->b));
    case K::OR: return mk_bin(K::AND, mk_not(x->a), mk_not(x->b));
    case K::ANDNOT: return mk_bin(K::OR, mk_not(x->a), x->b);
    }
    return mk_false();
}

int count_leaves(const ExprP& e) {
    if (e->kind == Expr::LEAF) return 1;
    if (e->kind == Expr::CONST_TRUE || e->kind == Expr::CONST_FALSE) return 0;
    return count_leaves(e->a) + count_leaves(e->b);
}

// registers the expression needs (Sethi–Ullman / Strahler number)
int need(const ExprP& e) {
    if (e->kind == Expr::LEAF) return 1;
    const int l = need(e->a), r = need(e->b);
    return l == r ? l + 1 : std::max(l, r);
}

// Emit postfix. For AND/OR the heavier child goes first; ANDNOT with a heavier right child
// is rewritten as AND(~b-side-first) via a reverse op: we keep a & ~b by emitting b first
// and using AND with the complement pushed into b when b is a leaf, otherwise the order is
// kept (depth checked by the caller).
struct Emitter {
    EvalProgram prog{};
    int n_ops = 0;
    int depth = 0, max_depth = 0;
    bool ok = true;
    void leaf(const Leaf& l, bool neg) {
        if (prog.n_leaves >= (uint32_t)kMaxLeaves) {
            ok = false;
            return;
        }
        const uint32_t k = prog.n_leaves++;
        prog.leaf[k] = l.bv;
        if (neg) prog.negate |= 1u << k;
        max_depth = std::max(max_depth, ++depth);
    }
    void op(uint32_t o) {
        const uint32_t k = prog.n_leaves - 1;
        if (prog.n_leaves == 0 || n_ops >= kMaxOps || prog_nops(prog, (int)k) == 15) {
            ok = false;
            return;
        }
        prog.ops |= o << (2 * n_ops++);
        prog.nops += 1u << (4 * k);
        --depth;
    }
    // a conjunction of (possibly complemented) leaves: AND nodes, ANDNOT with a leaf on the right
    static bool conj_leaves(const ExprP& e, std::vector<std::pair<Leaf, bool>>& out) {
        switch (e->kind) {
        case Expr::LEAF: out.push_back({e->leaf, e->neg}); return true;
        case Expr::AND: return conj_leaves(e->a, out) && conj_leaves(e->b, out);
        case Expr::ANDNOT:
            if (e->b->kind != Expr::LEAF) return false;
            if (!conj_leaves(e->a, out)) return false;
            out.push_back({e->b->leaf, !e->b->neg});
            return true;
        default: return false;
        }
    }
    using Lits = std::vector<std::pair<Leaf, bool>>;
    static bool or_literals(const ExprP& e, Lits& out) {
        if (e->kind == Expr::LEAF) {
            out.push_back({e->leaf, e->neg});
            return true;
        }
        if (e->kind == Expr::OR) return or_literals(e->a, out) && or_literals(e->b, out);
        return false;
    }
    static void or_parts(const ExprP& e, std::vector<ExprP>& out) {
        if (e->kind == Expr::OR) {
            or_parts(e->a, out);
            or_parts(e->b, out);
        } else {
            out.push_back(e);
        }
    }
    // AND-ed parts; a & ~leaf contributes the complemented leaf as a part of its own
    static bool and_parts(const ExprP& e, std::vector<Lits>& groups) {
        if (e->kind == Expr::AND) return and_parts(e->a, groups) && and_parts(e->b, groups);
        if (e->kind == Expr::ANDNOT) {
            if (e->b->kind != Expr::LEAF) return false;
            if (!and_parts(e->a, groups)) return false;
            groups.push_back({{e->b->leaf, !e->b->neg}});
            return true;
        }
        Lits g;
        if (!or_literals(e, g)) return false;
        groups.push_back(std::move(g));
        return true;
    }
    // two-level program: groups of literals combined by `inner`, groups combined by `outer`;
    // the postfix encoding of the same program is emitted alongside (interpreter fallback)
    bool emit_groups(const std::vector<Lits>& groups, uint32_t inner, uint32_t outer, uint32_t form) {
        size_t total = 0;
        for (const auto& g : groups) total += g.size();
        if (groups.empty() || total > (size_t)kMaxLeaves) return false;
        uint32_t gstart = 0;
        for (size_t gi = 0; gi < groups.size(); ++gi) {
            gstart |= 1u << prog.n_leaves;
            for (size_t i = 0; i < groups[gi].size(); ++i) {
                leaf(groups[gi][i].first, groups[gi][i].second);
                if (i) op(inner);
            }
            if (gi) op(outer);
        }
        prog.form = form;
        prog.gstart = gstart;
        return ok;
    }
    // top level: a pure conjunction is emitted as a left-deep AND chain (branch-free CONJ
    // form, is_conjunction in cubit_kernels.hip); an OR of conjunctions (DNF) or an AND of
    // ORs of literals (CNF) as a branch-free two-level program; anything else as postfix
    void emit_top(const ExprP& e) {
        Lits c;
        if (e->kind != Expr::LEAF && conj_leaves(e, c)) {
            leaf(c[0].first, c[0].second);
            for (size_t i = 1; i < c.size(); ++i) {
                leaf(c[i].first, c[i].second);
                op(OP_AND);
            }
            return;
        }
        if (e->kind == Expr::OR) {
            std::vector<ExprP> parts;
            or_parts(e, parts);
            std::vector<Lits> groups;
            bool dnf = true;
            for (const auto& p : parts) {
                Lits g;
                if (!conj_leaves(p, g)) {
                    dnf = false;
                    break;
                }
                groups.push_back(std::move(g));
            }
            if (dnf) {
                Emitter trial;
                if (trial.emit_groups(groups, OP_AND, OP_OR, FORM_DNF)) {
                    *this = trial;
                    return;
                }
            }
        }
        if (e->kind == Expr::AND || e->kind == Expr::ANDNOT) {
            std::vector<Lits> groups;
            if (and_parts(e, groups)) {
                Emitter trial;
                if (trial.emit_groups(groups, OP_OR, OP_AND, FORM_CNF)) {
                    *this = trial;
                    return;
                }
            }
        }
        emit(e);
    }
    void emit(const ExprP& e) {
        switch (e->kind) {
        case Expr::LEAF: leaf(e->leaf, e->neg); return;
        case Expr::AND:
        case Expr::OR: {
            const uint32_t o = e->kind == Expr::AND ? OP_AND : OP_OR;
            if (need(e->b) > need(e->a)) {
                emit(e->b);
                emit(e->a);
            } else {
                emit(e->a);
                emit(e->b);
            }
            op(o);
            return;
        }
        case Expr::ANDNOT: {
            if (need(e->b) > need(e->a) && e->b->kind == Expr::LEAF) {
                // a & ~b == (~b) & a with b a leaf: emit complemented leaf first
                leaf(e->b->leaf, !e->b->neg);
                emit(e->a);
                op(OP_AND);
            } else {
                emit(e->a);
                emit(e->b);
                op(OP_ANDNOT);
            }
            return;
        }
        default: ok = false; return;
        }
    }
};

}  // namespace

extern "C" int cubit_bitvector_eval(cubit_ctx* ctx, const uint64_t* const* d_leaves, uint32_t n_leaves,
                                    uint32_t leaf_negate, const int32_t* prog, uint32_t n_prog, uint64_t n_rows,
                                    int64_t row_base, int64_t* d_rowids, uint64_t capacity, uint64_t* d_count,
                                    uint64_t* d_result_words, uint32_t flags) {
    if (!ctx || !d_leaves || !prog || !d_count) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(ctx);
    if (n_rows == 0) {  // no rows: nothing qualifies, nothing to launch
        if (int rc = set_device(ctx)) return rc;
        ctx->last_tiles = 0;
        HIP_CHECK(hipMemsetAsync(d_count, 0, sizeof(uint64_t), ctx->stream));
        return CUBIT_OK;
    }
    const bool count_only = (flags & CUBIT_SCAN_COUNT_ONLY) != 0;
    if (!count_only && !d_rowids) return fail(CUBIT_ERR_INVALID, "d_rowids is null without COUNT_ONLY");
    // postfix → expression (validates arity), then the emitter re-linearises it
    std::vector<ExprP> st;
    for (uint32_t i = 0; i < n_prog; ++i) {
        const int32_t x = prog[i];
        if (x >= 0) {
            if ((uint32_t)x >= n_leaves) return fail(CUBIT_ERR_INVALID, "leaf %d out of range", x);
            Leaf l;
            l.bv = d_leaves[x];
            st.push_back(mk_leaf(l, ((leaf_negate >> x) & 1u) != 0));
        } else {
            if (st.size() < 2) return fail(CUBIT_ERR_INVALID, "program underflow at %u", i);
            ExprP b = st.back();
            st.pop_back();
            ExprP a = st.back();
            st.pop_back();
            Expr::Kind k = x == CUBIT_OP_AND ? Expr::AND : x == CUBIT_OP_OR ? Expr::OR : x == CUBIT_OP_ANDNOT
                                                                                         ? Expr::ANDNOT
                                                                                         : Expr::CONST_FALSE;
            if (k == Expr::CONST_FALSE) return fail(CUBIT_ERR_INVALID, "bad opcode %d", x);
            auto e = std::make_shared<Expr>();
            e->kind = k;
            e->a = a;
            e->b = b;
            st.push_back(e);
        }
    }
    if (st.size() != 1) return fail(CUBIT_ERR_INVALID, "program leaves %zu values on the stack", st.size());
    Emitter em;
    em.emit_top(st[0]);
    if (!em.ok || em.max_depth > 4)
        return fail(CUBIT_ERR_UNSUPPORTED, "program needs %d leaves / depth %d (max %d / 4)", count_leaves(st[0]),
                    em.max_depth, kMaxLeaves);
    return run_eval(ctx, em.prog, n_rows, row_base, count_only ? nullptr : d_rowids, capacity, d_count, d_result_words,
                    count_only ? RunMode::kCount : RunMode::kDecode, true, (flags & CUBIT_SCAN_ORDERED) != 0,
                    (flags & CUBIT_SCAN_CHECK_CAPACITY) != 0);
}

extern "C" int cubit_gather(cubit_ctx* ctx, const void* d_col, int type, const int64_t* d_rowids,
                            const uint64_t* d_count, uint64_t max_n, int64_t row_base, int64_t* d_out) {
    if (!ctx || !d_col || !d_rowids || !d_count || !d_out) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(ctx);
    if (type != CUBIT_TYPE_INT32 && type != CUBIT_TYPE_INT64 && !type_is_keyed(type))
        return fail(CUBIT_ERR_UNSUPPORTED, "type %d", type);
    HIP_CHECK(launch_gather(d_col, type, d_rowids, d_count, max_n, row_base, d_out, ctx->stream));
    return CUBIT_OK;
}

extern "C" int cubit_narrow_i32(cubit_ctx* ctx, const int64_t* d_in, const uint64_t* d_count, uint64_t max_n,
                                int64_t offset, int32_t* d_out) {
    if (!ctx || !d_in || !d_count || !d_out) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(ctx);
    HIP_CHECK(launch_narrow_i32(d_in, d_count, max_n, offset, d_out, ctx->stream));
    return CUBIT_OK;
}

extern "C" int cubit_narrow_checked(cubit_ctx* ctx, const int64_t* d_in, const uint64_t* d_count, uint64_t max_n,
                                    int64_t offset, int width, void* d_out, uint32_t* d_overflow) {
    if (!ctx || !d_in || !d_count || !d_out || !d_overflow) return fail(CUBIT_ERR_INVALID, "null argument");
    if (width < 1 || width > 4) return fail(CUBIT_ERR_INVALID, "width %d: 1, 2, 3 or 4 bytes", width);
    CUBIT_LOCK(ctx);
    HIP_CHECK(launch_narrow_unsigned(d_in, d_count, max_n, offset, width, d_out, d_overflow, ctx->stream));
    return CUBIT_OK;
}

extern "C" int cubit_narrow_i32_checked(cubit_ctx* ctx, const int64_t* d_in, const uint64_t* d_count, uint64_t max_n,
                                        int64_t offset, int32_t* d_out, uint32_t* d_overflow) {
    if (!ctx || !d_in || !d_count || !d_out || !d_overflow) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(ctx);
    HIP_CHECK(launch_narrow_i32(d_in, d_count, max_n, offset, d_out, ctx->stream, d_overflow));
    return CUBIT_OK;
}

extern "C" int cubit_gather_sum_product(cubit_ctx* ctx, const int64_t* d_a, const int64_t* d_b,
                                        const int64_t* d_rowids, const uint64_t* d_count, uint64_t max_n,
                                        int64_t row_base, int64_t* d_out) {
    if (!ctx || !d_a || !d_b || !d_rowids || !d_count || !d_out) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(ctx);
    HIP_CHECK(launch_gather_sum_product(d_a, d_b, d_rowids, d_count, max_n, row_base, ctx->partials, d_out,
                                        ctx->stream));
    return CUBIT_OK;
}

// ------------------------------------------------------------------ table partition

namespace {

struct DevBuf {
    void* p = nullptr;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

// A VARCHAR column's dictionary: its distinct strings in DuckDB's string order
// (string_type.hpp:143-206: the bytes as unsigned — std::string_view's order — then the length,
// a prefix before its extensions), string `code` = bytes[offs[code], offs[code + 1]).
struct DictData {
    std::vector<char> bytes;
    std::vector<uint64_t> offs{0};
    uint64_t fingerprint = 0;  // FNV-1a over the entries and their lengths: an index file names its dictionary
    uint64_t size() const { return offs.size() - 1; }
    std::string_view at(uint64_t code) const {
        return std::string_view(bytes.data() + offs[code], offs[code + 1] - offs[code]);
    }
    // the first code whose string is >= s (size() when none), and whether it is s
    uint64_t lower_bound(std::string_view s, bool* present) const {
        uint64_t lo = 0, hi = size();
        while (lo < hi) {
            const uint64_t mid = (lo + hi) / 2;
            if (at(mid) < s) lo = mid + 1;
            else hi = mid;
        }
        *present = lo < size() && at(lo) == s;
        return lo;
    }
};

struct Column {
    int type = 0;
    std::shared_ptr<const DictData> dict;  // VARCHAR: the dictionary its codes index
    // FLOAT / DOUBLE: `data` holds the comparison keys (an INT32 / INT64 column to every compare
    // kernel, key_type) and `raw` the bit patterns as registered (probes, downloads), both owned and
    // kept in step by appends and merges; raw = data for every other type
    const void* raw = nullptr;
    std::unique_ptr<DevBuf> raw_buf;
    const void* data = nullptr;        // device
    const uint64_t* validity = nullptr;  // device, padded to the table's cap_words (null = no NULLs)
    uint64_t cap_rows = 0;  // rows the owned data buffer holds (0 = caller-owned device data)
    std::vector<std::unique_ptr<DevBuf>> owned;
    // a column registered as BITPACKING segments keeps them on the device (packed bytes + the
    // group table): constant comparisons on it unpack and compare in one pass
    // (bitpacked_compare_kernel) instead of reading the plain column. Dropped when the values
    // change (appends, merges).
    std::unique_ptr<DevBuf> bp_bytes, bp_groups;
    std::unique_ptr<DevBuf> bp_vgroup;  // per 2,048-row vector: the group holding its first row
    uint64_t bp_n_groups = 0;
    // every group FOR ≤ 32 bits / CONSTANT / CONSTANT_DELTA: the widest FOR group's bits (≥ 1);
    // else 0 (launch_bitpacked_compare)
    int bp_simple_width = 0;
    void drop_packed() {
        bp_bytes.reset();
        bp_groups.reset();
        bp_vgroup.reset();
        bp_n_groups = 0;
    }
};

// the type and values the compare kernels read for a column, and the values its probes read
int ktype(const Column& c) { return key_type(c.type); }
const void* raw_of(const Column& c) { return type_is_fp(c.type) ? c.raw : c.data; }

struct Index {
    int encoding = CUBIT_INDEX_RANGE;
    bool exact_all = false;  // keys = every distinct value
    int64_t vmin = 0, vmax = 0;
    bool empty = true;       // no valid rows
    std::vector<int64_t> keys;
    std::vector<uint64_t*> bvs;  // parallel to keys
    std::vector<std::unique_ptr<DevBuf>> owned;
    uint64_t bytes = 0;
};

struct Updates {
    std::unique_ptr<DevBuf> rows, values, versions;
    std::vector<int64_t> h_rows, h_values;
    std::vector<uint64_t> h_versions;
    // NULL-ness per record (the validity column's update chain, InitializeUpdateValidity,
    // update_segment.cpp:588-600): 1 = the record's value, 0 = SET NULL. Empty / null when every
    // record carries a value.
    std::vector<uint8_t> h_valids;
    std::unique_ptr<DevBuf> valids;
    bool any_null = false;
    const uint8_t* d_valids() const { return valids ? static_cast<const uint8_t*>(valids->p) : nullptr; }
    bool valid_at(uint64_t i) const { return h_valids.empty() || h_valids[i]; }
    std::vector<uint64_t> distinct_versions;  // sorted
    uint64_t n = 0;
    bool unique_rows = true;  // one record per row (the checkpoint fast path merges the list as is)
    // distinct updated values, sorted: the update statistics the planner widens the index
    // statistics with (DuckDB's zonemaps consult update statistics the same way,
    // standard_column_data.cpp:50-57)
    std::vector<int64_t> stat_values;
    // does any record pass TransactionVersionOperator::UseInsertedVersion for this
    // transaction (id < start_time || id == transaction_id)? If not, the transaction sees
    // the base values and no patch is needed.
    bool any_visible(const cubit_txn* txn) const {
        if (!txn || distinct_versions.empty()) return false;
        if (distinct_versions.front() < txn->start_time) return true;
        return std::binary_search(distinct_versions.begin(), distinct_versions.end(), txn->transaction_id);
    }
    // Patched leaves kept across scans. A leaf's content is fixed by its predicate on this
    // column (index leaf or K0 bitvector alike), and for a reader without updates of its own
    // the visible records are a version prefix, so (predicate, prefix) names the patched
    // copy. Dropped whenever the column, its indexes or the update list change.
    struct PatchKey {
        int pred, cmp;
        int64_t c, c2;
        bool operator<(const PatchKey& o) const {
            return std::tie(pred, cmp, c, c2) < std::tie(o.pred, o.cmp, o.c, o.c2);
        }
    };
    struct Patched {
        int64_t prefix = -1;
        std::unique_ptr<DevBuf> bv;
    };
    std::map<PatchKey, Patched> cache;
    // zones holding an update record of any version (bit per zone), for the zone classes of
    // patched leaves; computed on first use for dirty_nz zones
    std::vector<uint64_t> dirty;
    uint32_t dirty_nz = 0;
};

}  // namespace

struct cubit_table {
    cubit_ctx* ctx = nullptr;
    uint64_t n_rows = 0;
    int64_t row_base = 0;
    uint64_t nwp = 0;  // padded words
    // words allocated per table-owned bitvector (index leaves, validity): ≥ nwp, zero past the
    // rows; appends grow the table in place until nwp would exceed it (cubit_table_append)
    uint64_t cap_words = 0;
    std::map<int, Column> cols;
    std::map<int, Index> idx;
    std::map<int, Index> bins;  // CUBIT_INDEX_BINS (secondary)
    // MVCC delta
    std::unique_ptr<DevBuf> del_rows, del_ids;
    uint64_t n_del = 0;
    // Committed-delete visibility bitvector, kept across scans (CUBIT keeps deletions as a
    // maintained bitvector rather than re-deriving them per query). For a transaction with no
    // deletes of its own, the deletes in effect are exactly those with id < start_time — a
    // prefix of the id-sorted list — so the bitvector is reused while that prefix length is
    // unchanged. vis_prefix = -1: not built.
    std::vector<uint64_t> del_ids_sorted;
    std::unique_ptr<DevBuf> vis_cache;
    int64_t vis_prefix = -1;
    // Insert versions: row ranges [begin, end) appended by one transaction with its insert
    // id (ChunkConstantInfo::insert_id / ChunkVectorInfo::inserted, chunk_info.cpp); rows
    // outside every range were inserted before any snapshot. Sorted by id: for a reader
    // without inserts of its own the visible ranges are an id prefix, which also keys the
    // cached visibility bitvector (vis_ins_prefix).
    struct InsRange {
        int64_t begin, end;
        uint64_t id;
    };
    std::vector<InsRange> ins;
    std::unique_ptr<DevBuf> hidden_dev;  // invisible ranges of the last visibility build
    std::vector<int64_t> hidden_host;
    int64_t vis_ins_prefix = -1;
    std::map<int, Updates> upd;
    // scratch bitvectors (reused across scans)
    std::vector<std::unique_ptr<DevBuf>> scratch;
    size_t scratch_used = 0;
    std::unique_ptr<DevBuf> ones;  // all valid rows
    uint32_t last_leaves = 0, last_passes = 0;
    // the last planned program, when it is one table-owned index bitvector as it stands (no
    // complement, no patch): its per-zone counts give the decode its offsets up front
    const uint64_t* single_leaf = nullptr;
    // CUBIT_HOST_TIMING: host time of cubit_table_scan split into planning, tile offsets and
    // launch (ns, summed), printed when the table is destroyed (diagnostic)
    uint64_t host_ns[3] = {0, 0, 0};
    uint64_t host_scans = 0;
    uint32_t last_decoded = 0;  // sum_product: values of b decoded from its index (0 = gathered)
    uint64_t* dummy_count = nullptr;
    std::unique_ptr<DevBuf> dummy;
    // Zonemaps (RowGroup::CheckZonemap / CheckZonemapSegments, row_group.cpp:361-371, 407-445,
    // over bitvector zones of kZoneRows rows): per table-owned bitvector (index leaf, bin,
    // validity) a bit per zone for "no row set" (z) and "every row set" (o). Computed on the
    // first scan that reads the bitvector; dropped (drop_zones) whenever a table-owned
    // bitvector is written, grown or freed, so an entry always describes the current bits.
    struct ZoneMap {
        std::vector<uint64_t> z, o;
        bool informative = false;  // some zone is all-zero or all-one
        std::vector<uint32_t> cnt;  // set rows per zone
        // exclusive prefix of cnt on the device (nz + 1 entries), built the first time a scan of
        // this bitvector alone decodes (EvalArgs::tile_prefix); dropped with the zone map
        std::shared_ptr<DevBuf> prefix;
        std::vector<uint64_t> prefix_host;
    };
    std::unordered_map<const uint64_t*, ZoneMap> zones;
    std::unique_ptr<DevBuf> zone_dev;  // class bytes of the bitvectors being summarised
    uint64_t zone_dev_bytes = 0;
    // per-zone statistics of raw columns (min / max of the valid rows, any / every row valid),
    // for leaves built from the column values (K0, candidate check), and the zone maps derived
    // from them per predicate; dropped with the bitvector zone maps
    struct ColZones {
        std::vector<int64_t> mn, mx;
        std::vector<uint8_t> fl;  // bit 0 = some row valid, bit 1 = every row valid
    };
    std::map<int, ColZones> col_zones;
    std::map<std::tuple<int, int, int, int64_t, int64_t>, ZoneMap> pred_zones;
    uint32_t last_live = 0, last_zones = 0;  // zones the last scan evaluated / the partition has
    bool use_packed = false;  // cubit_table_use_packed_filter (off by default: slower than K0)
    uint32_t last_packed = 0;  // leaves the last plan built straight from packed segments
    bool use_narrowing = true;  // cubit_table_use_narrowing
    uint32_t last_narrowed = 0;  // K0 leaves the last plan built only at the rows a mask kept
    std::vector<int32_t> last_narrow_cols;  // columns of the last plan's K0 leaves, in build order
    bool last_sum_packed = false;  // the last sum_product read a from its BITPACKING segments
};

namespace {

// A table-owned bitvector is about to be written, grown or freed: every zone map goes (they
// are recomputed on the next scan that needs them).
void drop_zones(cubit_table* t) {
    t->zones.clear();
    t->col_zones.clear();
    t->pred_zones.clear();
}

// The column's values or indexes changed: its patched leaves are stale.
void drop_patches(cubit_table* t, int col) {
    drop_zones(t);
    auto it = t->upd.find(col);
    if (it != t->upd.end()) it->second.cache.clear();
}

// a table-owned bitvector of cap_words words, all zero (the kernels that fill it write nwp
// words; the rest must stay zero for appends that grow into it)
int alloc_table_bv(cubit_table* t, DevBuf& b) {
    if (hipMalloc(&b.p, std::max<uint64_t>(t->cap_words, 1) * 8) != hipSuccess) return CUBIT_ERR_OOM;
    if (hipMemsetAsync(b.p, 0, std::max<uint64_t>(t->cap_words, 1) * 8, t->ctx->stream) != hipSuccess) return CUBIT_ERR_HIP;
    return CUBIT_OK;
}

// Everything derived from the row count (scratch / ones / visibility / patched leaves, all
// nwp words): dropped when the table grows or its base changes.
void drop_derived(cubit_table* t) {
    drop_zones(t);
    t->scratch.clear();
    t->scratch_used = 0;
    t->ones.reset();
    t->vis_cache.reset();
    t->vis_prefix = -1;
    t->vis_ins_prefix = -1;
    for (auto& kv : t->upd) kv.second.cache.clear();
}

int scratch_bv(cubit_table* t, uint64_t** out) {
    if (t->scratch_used < t->scratch.size()) {
        *out = static_cast<uint64_t*>(t->scratch[t->scratch_used++]->p);
        return CUBIT_OK;
    }
    auto b = std::make_unique<DevBuf>();
    if (hipMalloc(&b->p, t->nwp * sizeof(uint64_t)) != hipSuccess)
        return fail(CUBIT_ERR_OOM, "scratch bitvector allocation failed");
    *out = static_cast<uint64_t*>(b->p);
    t->scratch.push_back(std::move(b));
    t->scratch_used++;
    return CUBIT_OK;
}

int ones_bv(cubit_table* t, const uint64_t** out) {
    if (!t->ones) {
        t->ones = std::make_unique<DevBuf>();
        if (hipMalloc(&t->ones->p, t->nwp * sizeof(uint64_t)) != hipSuccess)
            return fail(CUBIT_ERR_OOM, "ones bitvector allocation failed");
        HIP_CHECK(launch_fill_valid(static_cast<uint64_t*>(t->ones->p), t->n_rows, t->ctx->stream));
    }
    *out = static_cast<const uint64_t*>(t->ones->p);
    return CUBIT_OK;
}

// padded device copy of a validity mask (the NN bitvector: kernels read whole tiles), bits
// past n_rows cleared
int copy_validity(cubit_table* t, Column& c, const uint64_t* validity, int on_device) {
    hipStream_t s = t->ctx->stream;
    auto b = std::make_unique<DevBuf>();
    if (hipMalloc(&b->p, t->cap_words * 8) != hipSuccess) return fail(CUBIT_ERR_OOM, "validity allocation failed");
    HIP_CHECK(hipMemsetAsync(b->p, 0, t->cap_words * 8, s));
    const uint64_t nw = (t->n_rows + 63) / 64;
    HIP_CHECK(hipMemcpyAsync(b->p, validity, nw * 8, on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
    if (t->n_rows & 63) {
        uint64_t last = 0;
        HIP_CHECK(hipMemcpyAsync(&last, static_cast<uint64_t*>(b->p) + nw - 1, 8, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        last &= (1ull << (t->n_rows & 63)) - 1;
        HIP_CHECK(hipMemcpyAsync(static_cast<uint64_t*>(b->p) + nw - 1, &last, 8, hipMemcpyHostToDevice, s));
    }
    c.validity = static_cast<const uint64_t*>(b->p);
    c.owned.push_back(std::move(b));
    return CUBIT_OK;
}

int value_stats(cubit_table* t, const void* data, int type, const uint64_t* validity, uint64_t n,
                std::vector<int64_t>& distinct, bool want_distinct, int64_t& vmin, int64_t& vmax, bool& any);

// The INT32 / INT64 column type a type code's values are held as (INT8, INT16, UINT8, UINT16 →
// INT32; UINT32, UINT64 → INT64), and the code's value size; false for an unknown code.
bool storage_of(int type, int& col_type, uint64_t& src_size) {
    switch (type) {
    case CUBIT_TYPE_INT32: col_type = CUBIT_TYPE_INT32, src_size = 4; return true;
    case CUBIT_TYPE_INT64: col_type = CUBIT_TYPE_INT64, src_size = 8; return true;
    case CUBIT_TYPE_INT8: case CUBIT_TYPE_UINT8: col_type = CUBIT_TYPE_INT32, src_size = 1; return true;
    case CUBIT_TYPE_INT16: case CUBIT_TYPE_UINT16: col_type = CUBIT_TYPE_INT32, src_size = 2; return true;
    case CUBIT_TYPE_UINT32: col_type = CUBIT_TYPE_INT64, src_size = 4; return true;
    case CUBIT_TYPE_UINT64: col_type = CUBIT_TYPE_UINT64, src_size = 8; return true;  // the bits, keyed
    case CUBIT_TYPE_FLOAT: col_type = CUBIT_TYPE_FLOAT, src_size = 4; return true;
    case CUBIT_TYPE_DOUBLE: col_type = CUBIT_TYPE_DOUBLE, src_size = 8; return true;
    case CUBIT_TYPE_VARCHAR: col_type = CUBIT_TYPE_VARCHAR, src_size = 4; return true;  // codes
    default: return false;
    }
}

// A column of a narrower or unsigned type code: its values (host or device) widened on the
// device into an owned INT32 / INT64 column (UINT64 columns are held as their bits, keyed).
int widen_column(cubit_table* t, Column& c, int type, const void* data, const uint64_t* validity, int on_device) {
    int col_type = 0;
    uint64_t ssz = 0;
    storage_of(type, col_type, ssz);
    const uint64_t esz = col_type == CUBIT_TYPE_INT32 ? 4 : 8;
    c.type = col_type;
    if (t->n_rows == 0) return CUBIT_OK;
    hipStream_t s = t->ctx->stream;
    DevBuf staged;
    const void* src = data;
    if (!on_device) {
        if (hipMalloc(&staged.p, t->n_rows * ssz) != hipSuccess) return fail(CUBIT_ERR_OOM, "column staging failed");
        HIP_CHECK(hipMemcpyAsync(staged.p, data, t->n_rows * ssz, hipMemcpyHostToDevice, s));
        src = staged.p;
    }
    auto b = std::make_unique<DevBuf>();
    if (hipMalloc(&b->p, std::max<uint64_t>(t->n_rows * esz, 16)) != hipSuccess)
        return fail(CUBIT_ERR_OOM, "column allocation failed");
    HIP_CHECK(launch_widen(src, type, t->n_rows, b->p, s));
    c.data = b->p;
    c.cap_rows = t->n_rows;
    c.owned.push_back(std::move(b));
    if (validity) {
        if (int rc = copy_validity(t, c, validity, on_device)) return rc;
    }
    HIP_CHECK(hipStreamSynchronize(s));
    return CUBIT_OK;
}

// A FLOAT / DOUBLE column: the patterns copied into an owned buffer (from host or device memory) and
// their keys computed beside them into `data`.
int fp_column(cubit_table* t, Column& c, int type, const void* data, const uint64_t* validity, int on_device) {
    const uint64_t esz = type_is32(type) ? 4 : 8;
    hipStream_t s = t->ctx->stream;
    c.type = type;
    c.raw_buf = std::make_unique<DevBuf>();
    auto keys = std::make_unique<DevBuf>();
    if (hipMalloc(&c.raw_buf->p, std::max<uint64_t>(t->n_rows * esz, 16)) != hipSuccess ||
        hipMalloc(&keys->p, std::max<uint64_t>(t->n_rows * esz, 16)) != hipSuccess)
        return fail(CUBIT_ERR_OOM, "column allocation failed");
    if (t->n_rows)
        HIP_CHECK(hipMemcpyAsync(c.raw_buf->p, data, t->n_rows * esz, on_device ? hipMemcpyDeviceToDevice
                                                                                : hipMemcpyHostToDevice, s));
    HIP_CHECK(launch_fp_keys(c.raw_buf->p, type, t->n_rows, keys->p, s));
    c.raw = c.raw_buf->p;
    c.data = keys->p;
    c.cap_rows = t->n_rows;
    c.owned.push_back(std::move(keys));
    if (validity) {
        if (int rc = copy_validity(t, c, validity, on_device)) return rc;
    }
    HIP_CHECK(hipStreamSynchronize(s));
    return CUBIT_OK;
}

int copy_column(cubit_table* t, Column& c, int type, const void* data, const uint64_t* validity, int on_device) {
    if (type_is_fp(type)) return fp_column(t, c, type, data, validity, on_device);
    if (type != CUBIT_TYPE_INT32 && type != CUBIT_TYPE_INT64 && type != CUBIT_TYPE_VARCHAR && !type_is_keyed(type))
        return widen_column(t, c, type, data, validity, on_device);
    const uint64_t esz = type_is32(type) ? 4 : 8;  // FLOAT / DOUBLE: the bit patterns as they are
    if (t->n_rows == 0) {  // empty partition: nothing to copy
        c.type = type;
        c.data = on_device ? data : nullptr;
        return CUBIT_OK;
    }
    hipStream_t s = t->ctx->stream;
    if (on_device) {
        c.data = data;
    } else {
        auto b = std::make_unique<DevBuf>();
        if (hipMalloc(&b->p, std::max<uint64_t>(t->n_rows * esz, 16)) != hipSuccess)
            return fail(CUBIT_ERR_OOM, "column allocation failed");
        HIP_CHECK(hipMemcpyAsync(b->p, data, t->n_rows * esz, hipMemcpyHostToDevice, s));
        c.data = b->p;
        c.cap_rows = t->n_rows;
        c.owned.push_back(std::move(b));
    }
    if (validity) {
        if (int rc = copy_validity(t, c, validity, on_device)) return rc;
    }
    HIP_CHECK(hipStreamSynchronize(s));
    c.type = type;
    return CUBIT_OK;
}

std::vector<int64_t> distinct_sorted(const int64_t* v, uint64_t n);

// an exact index over a span ≥ 2^32 keeps at most this many keys (one bitvector each)
constexpr size_t kMaxWideDistinct = 1 << 16;

// Index-build statistics on the device: min / max / any valid, and (want_distinct) the
// distinct valid values through a presence bitmap of vmax - vmin + 1 bits when the span is
// below 2^32, else by sorting the valid values on the host.
int value_stats(cubit_table* t, const void* data, int type, const uint64_t* validity, uint64_t n,
                std::vector<int64_t>& distinct, bool want_distinct, int64_t& vmin, int64_t& vmax, bool& any) {
    Column c;
    c.type = type;
    c.data = data;
    c.validity = validity;
    DevBuf stats;
    if (hipMalloc(&stats.p, 3 * sizeof(int64_t)) != hipSuccess) return fail(CUBIT_ERR_OOM, "stats allocation failed");
    int64_t h[3] = {INT64_MAX, INT64_MIN, 0};
    HIP_CHECK(hipMemcpyAsync(stats.p, h, sizeof(h), hipMemcpyHostToDevice, t->ctx->stream));
    HIP_CHECK(launch_column_minmax(c.data, c.type, c.validity, n, static_cast<int64_t*>(stats.p), t->ctx->stream));
    HIP_CHECK(hipMemcpyAsync(h, stats.p, sizeof(h), hipMemcpyDeviceToHost, t->ctx->stream));
    HIP_CHECK(hipStreamSynchronize(t->ctx->stream));
    any = h[2] > 0;
    vmin = h[0];
    vmax = h[1];
    if (!want_distinct) return CUBIT_OK;
    distinct.clear();
    if (!any) return CUBIT_OK;
    const uint64_t span = (uint64_t)vmax - (uint64_t)vmin;  // no signed overflow
    if (span >= (1ull << 32)) {
        // a wide span (TIMESTAMP microseconds, BIGINT ids) over few distinct values: sort the
        // valid values on the host instead (only INT64 and DOUBLE columns get here: a DOUBLE's
        // patterns become their keys first)
        std::vector<int64_t> hv(n);
        std::vector<uint64_t> hvalid(validity ? (n + 63) / 64 : 0);
        HIP_CHECK(hipMemcpyAsync(hv.data(), data, n * 8, hipMemcpyDeviceToHost, t->ctx->stream));
        if (validity)
            HIP_CHECK(hipMemcpyAsync(hvalid.data(), validity, hvalid.size() * 8, hipMemcpyDeviceToHost,
                                     t->ctx->stream));
        HIP_CHECK(hipStreamSynchronize(t->ctx->stream));
        if (validity) {
            uint64_t k = 0;
            for (uint64_t i = 0; i < n; ++i)
                if ((hvalid[i >> 6] >> (i & 63)) & 1) hv[k++] = hv[i];
            hv.resize(k);
        }
        if (type == CUBIT_TYPE_UINT64)  // (a DOUBLE column's `data` already holds keys)
            for (int64_t& v : hv) v = value_key(type, v);
        distinct = distinct_sorted(hv.data(), hv.size());
        if (distinct.size() > kMaxWideDistinct)
            return fail(CUBIT_ERR_UNSUPPORTED, "%zu distinct values over a span of 2^32 or more; give keys",
                        distinct.size());
        return CUBIT_OK;
    }
    const uint64_t range = span + 1;
    const uint64_t nw = (range + 63) / 64;
    DevBuf bits;
    if (hipMalloc(&bits.p, nw * 8) != hipSuccess) return fail(CUBIT_ERR_OOM, "presence bitmap allocation failed");
    HIP_CHECK(hipMemsetAsync(bits.p, 0, nw * 8, t->ctx->stream));
    HIP_CHECK(launch_presence(c.data, c.type, c.validity, n, vmin, range, static_cast<uint64_t*>(bits.p),
                              t->ctx->stream));
    std::vector<uint64_t> hb(nw);
    HIP_CHECK(hipMemcpyAsync(hb.data(), bits.p, nw * 8, hipMemcpyDeviceToHost, t->ctx->stream));
    HIP_CHECK(hipStreamSynchronize(t->ctx->stream));
    for (uint64_t w = 0; w < nw; ++w)
        for (uint64_t x = hb[w]; x; x &= x - 1) distinct.push_back(vmin + (int64_t)(w * 64 + __builtin_ctzll(x)));
    return CUBIT_OK;
}

int column_stats(cubit_table* t, const Column& c, std::vector<int64_t>& distinct, bool want_distinct,
                 int64_t& vmin, int64_t& vmax, bool& any) {
    return value_stats(t, c.data, ktype(c), c.validity, t->n_rows, distinct, want_distinct, vmin, vmax, any);
}

}  // namespace

extern "C" int cubit_table_create(cubit_ctx* ctx, uint64_t n_rows, int64_t row_base, cubit_table** out) {
    if (!ctx || !out) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(ctx);
    // n_rows = 0 is an empty partition (an empty table, or a rank with no rows): every scan
    // of it returns no rows without a launch
    if (n_rows >= (1ull << 47)) return fail(CUBIT_ERR_INVALID, "%llu rows exceed 2^47", (unsigned long long)n_rows);
    if (int rc = set_device(ctx)) return rc;
    auto* t = new cubit_table();
    t->ctx = ctx;
    t->n_rows = n_rows;
    t->row_base = row_base;
    t->nwp = padded_words(n_rows);
    t->cap_words = t->nwp;
    t->dummy = std::make_unique<DevBuf>();
    if (hipMalloc(&t->dummy->p, 64) != hipSuccess) {
        delete t;
        return fail(CUBIT_ERR_OOM, "allocation failed");
    }
    t->dummy_count = static_cast<uint64_t*>(t->dummy->p);
    *out = t;
    return CUBIT_OK;
}

bool host_timing() {
    static const bool on = std::getenv("CUBIT_HOST_TIMING") != nullptr;
    return on;
}
uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

extern "C" int cubit_table_destroy(cubit_table* t) {
    if (!t) return CUBIT_OK;
    CUBIT_LOCK(t->ctx);
    if (host_timing() && t->host_scans)
        std::fprintf(stderr, "cubit host timing: %llu scans; per scan plan %.2f us, tile offsets %.2f us, launch %.2f us\n",
                     (unsigned long long)t->host_scans, t->host_ns[0] * 1e-3 / t->host_scans,
                     t->host_ns[1] * 1e-3 / t->host_scans, t->host_ns[2] * 1e-3 / t->host_scans);
    (void)hipSetDevice(t->ctx->device);
    (void)hipStreamSynchronize(t->ctx->stream);
    delete t;
    return CUBIT_OK;
}

extern "C" int cubit_table_add_column(cubit_table* t, int col, int type, const void* data, const uint64_t* validity,
                                      int on_device) {
    if (!t || !data) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    int col_type = 0;
    uint64_t src_size = 0;
    if (!storage_of(type, col_type, src_size)) return fail(CUBIT_ERR_UNSUPPORTED, "type %d", type);
    if (type == CUBIT_TYPE_VARCHAR)
        return fail(CUBIT_ERR_INVALID, "a VARCHAR column is registered with its dictionary (cubit_table_add_dict_column)");
    if (col < 0) return fail(CUBIT_ERR_INVALID, "column %d", col);
    if (int rc = set_device(t->ctx)) return rc;
    Column c;
    if (int rc = copy_column(t, c, type, data, validity, on_device)) return rc;
    t->cols[col] = std::move(c);
    drop_patches(t, col);
    t->idx.erase(col);
    t->bins.erase(col);
    return CUBIT_OK;
}

// ------------------------------------------------------------------ VARCHAR dictionaries

struct cubit_dict {
    std::shared_ptr<const DictData> d;
};

extern "C" int cubit_dict_create(const char* bytes, const uint64_t* offsets, uint64_t n, cubit_dict** out) {
    if (!out || (n && (!offsets || (!bytes && offsets[n] > offsets[0])))) return fail(CUBIT_ERR_INVALID, "null argument");
    std::vector<std::string_view> v;
    v.reserve(n);
    for (uint64_t i = 0; i < n; ++i) {
        if (offsets[i + 1] < offsets[i]) return fail(CUBIT_ERR_INVALID, "offsets descend at string %llu", (unsigned long long)i);
        v.emplace_back(bytes + offsets[i], offsets[i + 1] - offsets[i]);
    }
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    if (v.size() > (uint64_t)INT32_MAX) return fail(CUBIT_ERR_UNSUPPORTED, "%zu distinct strings exceed 2^31 - 1", v.size());
    auto d = std::make_shared<DictData>();
    uint64_t total = 0;
    for (auto sv : v) total += sv.size();
    d->bytes.reserve(total);
    d->offs.reserve(v.size() + 1);
    for (auto sv : v) {
        d->bytes.insert(d->bytes.end(), sv.begin(), sv.end());
        d->offs.push_back(d->bytes.size());
    }
    uint64_t h = 1469598103934665603ull;
    auto mix = [&h](uint64_t b) { h = (h ^ b) * 1099511628211ull; };
    for (auto sv : v) {
        mix(sv.size());
        for (char c : sv) mix((unsigned char)c);
    }
    d->fingerprint = h;
    *out = new cubit_dict{std::move(d)};
    return CUBIT_OK;
}

extern "C" int cubit_dict_destroy(cubit_dict* d) {
    delete d;
    return CUBIT_OK;
}

extern "C" int cubit_dict_size(const cubit_dict* d, uint64_t* n) {
    if (!d || !n) return fail(CUBIT_ERR_INVALID, "null argument");
    *n = d->d->size();
    return CUBIT_OK;
}

extern "C" int cubit_dict_entry(const cubit_dict* d, uint64_t code, const char** data, uint64_t* size) {
    if (!d || !data || !size) return fail(CUBIT_ERR_INVALID, "null argument");
    if (code >= d->d->size()) return fail(CUBIT_ERR_INVALID, "code %llu past the dictionary's %llu strings",
                                          (unsigned long long)code, (unsigned long long)d->d->size());
    const std::string_view sv = d->d->at(code);
    *data = sv.data();
    *size = sv.size();
    return CUBIT_OK;
}

extern "C" int cubit_dict_encode(const cubit_dict* d, const char* bytes, const uint64_t* offsets, uint64_t n,
                                 const uint64_t* validity, int32_t* codes) {
    if (!d || (n && (!offsets || !codes))) return fail(CUBIT_ERR_INVALID, "null argument");
    for (uint64_t i = 0; i < n; ++i) {
        if (validity && !((validity[i >> 6] >> (i & 63)) & 1ull)) {
            codes[i] = 0;
            continue;
        }
        if (offsets[i + 1] < offsets[i]) return fail(CUBIT_ERR_INVALID, "offsets descend at string %llu", (unsigned long long)i);
        bool present = false;
        const uint64_t c = d->d->lower_bound(std::string_view(bytes + offsets[i], offsets[i + 1] - offsets[i]), &present);
        if (!present) return fail(CUBIT_ERR_UNSUPPORTED, "string %llu is not in the dictionary", (unsigned long long)i);
        codes[i] = (int32_t)c;
    }
    return CUBIT_OK;
}

// cubit_dict_encode on the device: the dictionary's entries are copied to the context's device
// for the call, one lane per string searches them (dict_encode_kernel).
extern "C" int cubit_dict_encode_device(cubit_ctx* ctx, const cubit_dict* d, const char* d_bytes,
                                        const uint64_t* d_offsets, uint64_t n, const uint64_t* d_validity,
                                        int32_t* d_codes) {
    if (!ctx || !d || (n && (!d_offsets || !d_codes))) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(ctx);
    if (n == 0) return CUBIT_OK;
    if (int rc = set_device(ctx)) return rc;
    const DictData& dd = *d->d;
    hipStream_t s = ctx->stream;
    DevBuf db, doffs, miss;
    if (hipMalloc(&db.p, std::max<uint64_t>(dd.bytes.size(), 16)) != hipSuccess ||
        hipMalloc(&doffs.p, dd.offs.size() * 8) != hipSuccess || hipMalloc(&miss.p, 8) != hipSuccess)
        return fail(CUBIT_ERR_OOM, "dictionary upload failed");
    if (!dd.bytes.empty()) HIP_CHECK(hipMemcpyAsync(db.p, dd.bytes.data(), dd.bytes.size(), hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(doffs.p, dd.offs.data(), dd.offs.size() * 8, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemsetAsync(miss.p, 0, 8, s));
    HIP_CHECK(launch_dict_encode(reinterpret_cast<const uint8_t*>(d_bytes), d_offsets, n, d_validity,
                                 static_cast<const uint8_t*>(db.p), static_cast<const uint64_t*>(doffs.p), dd.size(),
                                 d_codes, static_cast<unsigned long long*>(miss.p), s));
    unsigned long long missing = 0;
    HIP_CHECK(hipMemcpyAsync(&missing, miss.p, 8, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (missing)
        return fail(CUBIT_ERR_UNSUPPORTED, "%llu strings are not in the dictionary (their codes are -1)", missing);
    return CUBIT_OK;
}

extern "C" int cubit_dict_lookup(const cubit_dict* d, const char* data, uint64_t size, uint64_t* lower_bound,
                                 int* present) {
    if (!d || !lower_bound || (size && !data)) return fail(CUBIT_ERR_INVALID, "null argument");
    bool p = false;
    *lower_bound = d->d->lower_bound(std::string_view(data ? data : "", size), &p);
    if (present) *present = p ? 1 : 0;
    return CUBIT_OK;
}

extern "C" int cubit_table_add_dict_column(cubit_table* t, int col, cubit_dict* d, const int32_t* codes,
                                           const uint64_t* validity, int on_device) {
    if (!t || !d || (!codes && t->n_rows)) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    if (col < 0) return fail(CUBIT_ERR_INVALID, "column %d", col);
    if (int rc = set_device(t->ctx)) return rc;
    Column c;
    if (int rc = copy_column(t, c, CUBIT_TYPE_VARCHAR, codes, validity, on_device)) return rc;
    c.dict = d->d;
    if (t->n_rows) {  // every valid code names a dictionary string
        std::vector<int64_t> unused;
        int64_t vmin = 0, vmax = 0;
        bool any = false;
        if (int rc = value_stats(t, c.data, CUBIT_TYPE_VARCHAR, c.validity, t->n_rows, unused, false, vmin, vmax, any))
            return rc;
        if (any && (vmin < 0 || (uint64_t)vmax >= c.dict->size()))
            return fail(CUBIT_ERR_INVALID, "code %lld outside the dictionary's %llu strings",
                        (long long)(vmin < 0 ? vmin : vmax), (unsigned long long)c.dict->size());
    }
    t->cols[col] = std::move(c);
    drop_patches(t, col);
    t->idx.erase(col);
    t->bins.erase(col);
    return CUBIT_OK;
}

namespace {
// codes handed to a VARCHAR column (updates, appends): each valid one must name a dictionary string
int check_codes(const Column& c, const int64_t* v, const uint8_t* valid, uint64_t n) {
    if (c.type != CUBIT_TYPE_VARCHAR) return CUBIT_OK;
    for (uint64_t i = 0; i < n; ++i)
        if ((!valid || valid[i]) && (v[i] < 0 || (uint64_t)v[i] >= c.dict->size()))
            return fail(CUBIT_ERR_INVALID, "code %lld outside the dictionary's %llu strings", (long long)v[i],
                        (unsigned long long)c.dict->size());
    return CUBIT_OK;
}
}  // namespace

// The segments' T (a CUBIT_TYPE_* code): its byte size and signedness, the column type its
// values widen to and the BpGroup::tnorm that carries T's arithmetic there.
struct SegType {
    uint32_t tsz;
    bool sgn;
    int col_type;
    uint8_t tnorm;
};
bool seg_type_of(int type, SegType& st) {
    switch (type) {
    case CUBIT_TYPE_INT32: st = {4, true, CUBIT_TYPE_INT32, 0}; return true;
    case CUBIT_TYPE_INT64: st = {8, true, CUBIT_TYPE_INT64, 0}; return true;
    case CUBIT_TYPE_INT8: st = {1, true, CUBIT_TYPE_INT32, 8 | 0x80}; return true;
    case CUBIT_TYPE_INT16: st = {2, true, CUBIT_TYPE_INT32, 16 | 0x80}; return true;
    case CUBIT_TYPE_UINT8: st = {1, false, CUBIT_TYPE_INT32, 8}; return true;
    case CUBIT_TYPE_UINT16: st = {2, false, CUBIT_TYPE_INT32, 16}; return true;
    case CUBIT_TYPE_UINT32: st = {4, false, CUBIT_TYPE_INT64, 32}; return true;
    case CUBIT_TYPE_UINT64: st = {8, false, CUBIT_TYPE_UINT64, 0}; return true;
    default: return false;
    }
}

// The groups of one BITPACKING segment (at byte `base`, `rows` rows from partition row `row`):
// each group's mode, header fields and packed words, bounds-checked; packed runs off the 4-byte
// alignment are copied behind the bytes (`moved`, at bytes_padded + …).
int parse_bp_segment(const uint8_t* bytes, uint64_t n_bytes, uint64_t base, uint64_t rows, uint64_t row,
                     const SegType& st, uint64_t bytes_padded, std::vector<BpGroup>& groups,
                     std::vector<uint8_t>& moved, uint32_t sg) {
    const uint64_t tsz = st.tsz;
    if (base % 8 || base + 8 > n_bytes) return fail(CUBIT_ERR_INVALID, "segment %u: bad offset", sg);
    uint64_t meta_end;
    std::memcpy(&meta_end, bytes + base, 8);
    const uint64_t n_groups = (rows + 2047) / 2048;
    if (meta_end > n_bytes - base || meta_end < 8 + 4 * n_groups)
        return fail(CUBIT_ERR_INVALID, "segment %u: bad metadata offset", sg);
    for (uint64_t g = 0; g < n_groups; ++g) {
        uint32_t enc;
        std::memcpy(&enc, bytes + base + meta_end - 4 * (g + 1), 4);
        BpGroup bg{};
        const uint32_t mode = enc >> 24;
        const uint64_t data_off = base + (enc & 0x00ffffffu);
        bg.mode = (uint8_t)mode;
        bg.tnorm = st.tnorm;
        bg.row_start = row + g * 2048;
        bg.count = (uint32_t)std::min<uint64_t>(2048, rows - g * 2048);
        // header fields (BitpackingScanState::LoadNextGroup, bitpacking.cpp:620-690)
        const uint64_t n_fields = mode == 2 ? 1 : (mode == 3 || mode == 5) ? 2 : mode == 4 ? 3 : 0;
        if (n_fields == 0)
            return fail(CUBIT_ERR_INVALID, "segment %u group %llu: mode %u", sg, (unsigned long long)g, mode);
        if (data_off < base + 8 || data_off + n_fields * tsz > n_bytes)
            return fail(CUBIT_ERR_INVALID, "segment %u group %llu: out of bounds", sg, (unsigned long long)g);
        auto field = [&](uint64_t i) {
            uint64_t v = 0;  // T's bits, zero-extended (the kernels work mod 2^bits: bp_norm)
            std::memcpy(&v, bytes + data_off + i * tsz, tsz);
            return v;
        };
        bg.base = field(0);
        uint64_t packed = 0;
        if (mode == 3) {
            bg.aux = field(1);
        } else if (mode == 4 || mode == 5) {
            const uint64_t w = field(1) & 0xff;  // the reference reads the width as a T, uses its low byte
            if (w > 8 * tsz) return fail(CUBIT_ERR_INVALID, "segment %u group %llu: width %u", sg, (unsigned long long)g, (unsigned)w);
            bg.width = (uint16_t)w;
            if (mode == 4) bg.aux = field(2);
            packed = ((uint64_t)bg.count + 31) / 32 * 32 * w / 8;
        }
        bg.words_off = data_off + n_fields * tsz;
        if (bg.words_off + packed > n_bytes)
            return fail(CUBIT_ERR_INVALID, "segment %u group %llu: out of bounds", sg, (unsigned long long)g);
        if (packed && bg.words_off % 4) {
            const uint64_t at = moved.size();
            moved.resize(at + (packed + 15) / 16 * 16, 0);
            std::memcpy(moved.data() + at, bytes + bg.words_off, packed);
            bg.words_off = bytes_padded + at;
        }
        groups.push_back(bg);
    }
    return CUBIT_OK;
}

// DuckDB BITPACKING segments → device column (K5). The host walks each segment's metadata
// (header = end of the metadata words, one word per 2,048-row group, highest address first:
// BitpackingScanState / LoadNextGroup, bitpacking.cpp:620-690), checks every group's bounds,
// and the GPU unpacks all groups in parallel. A T of 1 or 2 bytes leaves its groups' packed
// runs off the 4-byte alignment the kernels' word loads need (the header fields are T-sized,
// WriteData, :448-451): those runs are copied behind the segment bytes, 16-aligned.
extern "C" int cubit_table_add_bitpacked_column(cubit_table* t, int col, int type, const uint8_t* bytes,
                                                uint64_t n_bytes, const uint64_t* seg_offsets,
                                                const uint64_t* seg_rows, uint32_t n_segments,
                                                const uint64_t* validity) {
    if (!t) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    SegType st;
    if (!seg_type_of(type, st)) return fail(CUBIT_ERR_UNSUPPORTED, "type %d", type);
    if (col < 0) return fail(CUBIT_ERR_INVALID, "column %d", col);
    if (t->n_rows == 0 && n_segments == 0) {  // empty partition, no segments
        Column c;
        c.type = st.col_type;
        t->cols[col] = std::move(c);
        drop_patches(t, col);
        t->idx.erase(col);
        t->bins.erase(col);
        return CUBIT_OK;
    }
    if (!bytes || !seg_offsets || !seg_rows || n_segments == 0) return fail(CUBIT_ERR_INVALID, "null argument");
    if (int rc = set_device(t->ctx)) return rc;
    const uint64_t esz = st.col_type == CUBIT_TYPE_INT32 ? 4 : 8;
    const uint64_t bytes_padded = (n_bytes + 15) / 16 * 16;
    std::vector<BpGroup> groups;
    std::vector<uint8_t> moved;  // packed runs copied to 16-aligned offsets behind the bytes
    uint64_t row = 0;
    for (uint32_t sg = 0; sg < n_segments; ++sg) {
        if (int rc = parse_bp_segment(bytes, n_bytes, seg_offsets[sg], seg_rows[sg], row, st, bytes_padded, groups,
                                      moved, sg))
            return rc;
        row += seg_rows[sg];
    }
    if (row != t->n_rows)
        return fail(CUBIT_ERR_INVALID, "segments hold %llu rows, partition has %llu", (unsigned long long)row,
                    (unsigned long long)t->n_rows);
    // the probe's random access (SumArgs::a_vgroup): the group of each vector's first row
    const uint64_t n_vec = (t->n_rows + 2047) / 2048;
    std::vector<uint32_t> vgroup(std::max<uint64_t>(n_vec, 1), 0);
    for (uint64_t v = 0, g = 0; v < n_vec; ++v) {
        while (g + 1 < groups.size() && groups[g].row_start + groups[g].count <= v * 2048) ++g;
        vgroup[v] = (uint32_t)g;
    }
    hipStream_t s = t->ctx->stream;
    DevBuf d_bytes, d_groups, d_vgroup;
    auto out = std::make_unique<DevBuf>();
    // +16: the kernels stage packed words with 16-byte-aligned loads that may run past the end
    if (hipMalloc(&d_bytes.p, bytes_padded + moved.size() + 16) != hipSuccess ||
        hipMalloc(&d_groups.p, groups.size() * sizeof(BpGroup)) != hipSuccess ||
        hipMalloc(&out->p, std::max<uint64_t>(t->n_rows * esz, 16)) != hipSuccess ||
        hipMalloc(&d_vgroup.p, vgroup.size() * 4) != hipSuccess)
        return fail(CUBIT_ERR_OOM, "bitpacked column allocation failed");
    HIP_CHECK(hipMemcpyAsync(d_bytes.p, bytes, n_bytes, hipMemcpyHostToDevice, s));
    if (!moved.empty())
        HIP_CHECK(hipMemcpyAsync(static_cast<uint8_t*>(d_bytes.p) + bytes_padded, moved.data(), moved.size(),
                                 hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(d_vgroup.p, vgroup.data(), vgroup.size() * 4, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(d_groups.p, groups.data(), groups.size() * sizeof(BpGroup), hipMemcpyHostToDevice, s));
    hipEvent_t e0, e1;
    if (int rc = timing_events(t->ctx, e0, e1)) return rc;
    HIP_CHECK(launch_bitunpack(static_cast<const uint8_t*>(d_bytes.p), static_cast<const BpGroup*>(d_groups.p),
                               groups.size(), st.col_type, out->p, s, e0, e1));
    HIP_CHECK(hipStreamSynchronize(s));
    Column c;
    c.type = st.col_type;
    c.data = out->p;
    c.cap_rows = t->n_rows;
    c.owned.push_back(std::move(out));
    c.bp_bytes = std::make_unique<DevBuf>();
    c.bp_groups = std::make_unique<DevBuf>();
    std::swap(c.bp_bytes->p, d_bytes.p);
    std::swap(c.bp_groups->p, d_groups.p);
    c.bp_vgroup = std::make_unique<DevBuf>();
    std::swap(c.bp_vgroup->p, d_vgroup.p);
    c.bp_n_groups = groups.size();
    c.bp_simple_width = 0;
    if (std::all_of(groups.begin(), groups.end(), [](const BpGroup& g) {
            return g.mode == 2 || g.mode == 3 || (g.mode == 5 && g.width <= 32);
        })) {
        int wmax = 1;
        for (const BpGroup& g : groups)
            if (g.mode == 5) wmax = std::max<int>(wmax, g.width);
        c.bp_simple_width = wmax;
    }
    if (validity) {
        if (int rc = copy_validity(t, c, validity, 0)) return rc;
        HIP_CHECK(hipStreamSynchronize(s));
    }
    t->cols[col] = std::move(c);
    drop_patches(t, col);
    t->idx.erase(col);
    t->bins.erase(col);
    return CUBIT_OK;
}

// The runs of one RLE segment (at byte `base`, `rows` rows from partition row `row`): values as
// T widened to int64 (T's sign), each run's end row appended to `ends`.
int parse_rle_segment(const uint8_t* bytes, uint64_t n_bytes, uint64_t base, uint64_t rows, uint64_t row,
                      const SegType& st, std::vector<int64_t>& vals, std::vector<uint64_t>& ends, uint32_t sg) {
    const uint64_t tsz = st.tsz;
    if (base + 8 > n_bytes) return fail(CUBIT_ERR_INVALID, "segment %u: bad offset", sg);
    uint64_t off;
    std::memcpy(&off, bytes + base, 8);
    if (off < 8 || off > n_bytes - base) return fail(CUBIT_ERR_INVALID, "segment %u: bad run-length offset", sg);
    uint64_t covered = 0;
    for (uint64_t k = 0; covered < rows; ++k) {
        if (8 + (k + 1) * tsz > off || off + 2 * (k + 1) > n_bytes - base)
            return fail(CUBIT_ERR_INVALID, "segment %u: runs cover %llu of %llu rows", sg, (unsigned long long)covered,
                        (unsigned long long)rows);
        uint16_t len;
        std::memcpy(&len, bytes + base + off + 2 * k, 2);
        uint64_t raw = 0;  // T's bits, zero-extended, then widened as T
        std::memcpy(&raw, bytes + base + 8 + k * tsz, tsz);
        int64_t v = (int64_t)raw;
        if (st.sgn && tsz < 8) v = (int64_t)(raw << (64 - 8 * tsz)) >> (64 - 8 * tsz);
        covered += len;
        if (covered > rows) return fail(CUBIT_ERR_INVALID, "segment %u: runs overrun its rows", sg);
        vals.push_back(v);
        ends.push_back(row + covered);
    }
    return CUBIT_OK;
}

// DuckDB RLE segments → device column. Each segment (rle.cpp RLECompressState::FlushSegment,
// :190-205: 8-byte header = offset of the uint16 run lengths, the run values as T from byte 8,
// the lengths after them) is walked on the host: run lengths are read until they cover the
// segment's rows (RLEScanState, :248-277 — zero-length runs, which a run of exactly 65,535 rows
// leaves behind, included), each value widened to the column's type as the BITPACKING path does.
// Only the runs cross to the device, and rle_expand_kernel writes the column.
extern "C" int cubit_table_add_rle_column(cubit_table* t, int col, int type, const uint8_t* bytes, uint64_t n_bytes,
                                          const uint64_t* seg_offsets, const uint64_t* seg_rows, uint32_t n_segments,
                                          const uint64_t* validity) {
    if (!t) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    SegType st;
    if (!seg_type_of(type, st)) return fail(CUBIT_ERR_UNSUPPORTED, "type %d", type);
    if (col < 0) return fail(CUBIT_ERR_INVALID, "column %d", col);
    if (n_segments && (!bytes || !seg_offsets || !seg_rows)) return fail(CUBIT_ERR_INVALID, "null argument");
    const bool wide = st.col_type != CUBIT_TYPE_INT32;
    std::vector<int64_t> vals;
    std::vector<uint64_t> ends;
    uint64_t row = 0;
    for (uint32_t sg = 0; sg < n_segments; ++sg) {
        if (int rc = parse_rle_segment(bytes, n_bytes, seg_offsets[sg], seg_rows[sg], row, st, vals, ends, sg)) return rc;
        row += seg_rows[sg];
    }
    if (row != t->n_rows)
        return fail(CUBIT_ERR_INVALID, "segments hold %llu rows, partition has %llu", (unsigned long long)row,
                    (unsigned long long)t->n_rows);
    if (int rc = set_device(t->ctx)) return rc;
    hipStream_t s = t->ctx->stream;
    const uint64_t esz = wide ? 8 : 4;
    std::vector<int32_t> narrow;
    if (!wide) narrow.assign(vals.begin(), vals.end());
    DevBuf d_vals, d_ends, d_tiles;
    auto out = std::make_unique<DevBuf>();
    const uint64_t n_tiles = (t->n_rows + 2047) / 2048;
    if (hipMalloc(&d_vals.p, std::max<uint64_t>(vals.size() * esz, 16)) != hipSuccess ||
        hipMalloc(&d_ends.p, std::max<uint64_t>(ends.size() * 8, 16)) != hipSuccess ||
        hipMalloc(&d_tiles.p, (n_tiles + 1) * 8) != hipSuccess ||
        hipMalloc(&out->p, std::max<uint64_t>(t->n_rows * esz, 16)) != hipSuccess)
        return fail(CUBIT_ERR_OOM, "RLE column allocation failed");
    if (!vals.empty()) {
        HIP_CHECK(hipMemcpyAsync(d_vals.p, wide ? (const void*)vals.data() : (const void*)narrow.data(),
                                 vals.size() * esz, hipMemcpyHostToDevice, s));
        HIP_CHECK(hipMemcpyAsync(d_ends.p, ends.data(), ends.size() * 8, hipMemcpyHostToDevice, s));
    }
    hipEvent_t e0, e1;
    if (int rc = timing_events(t->ctx, e0, e1)) return rc;
    HIP_CHECK(launch_rle_expand(d_vals.p, static_cast<const uint64_t*>(d_ends.p), ends.size(), t->n_rows, wide ? 1 : 0,
                                static_cast<uint64_t*>(d_tiles.p), out->p, s, e0, e1));
    HIP_CHECK(hipStreamSynchronize(s));
    Column c;
    c.type = st.col_type;
    c.data = out->p;
    c.cap_rows = t->n_rows;
    c.owned.push_back(std::move(out));
    if (validity) {
        if (int rc = copy_validity(t, c, validity, 0)) return rc;
        HIP_CHECK(hipStreamSynchronize(s));
    }
    t->cols[col] = std::move(c);
    drop_patches(t, col);
    t->idx.erase(col);
    t->bins.erase(col);
    return CUBIT_OK;
}

// A column given as DuckDB segments of mixed codecs, one per row group as DuckDB's checkpoint chose
// (UNCOMPRESSED, CONSTANT, RLE, BITPACKING). One run list covers every row: CONSTANT segments
// are one run of their value, RLE segments their runs, the others a placeholder run; the GPU
// expands it (rle_expand_kernel), then unpacks the BITPACKING groups over their rows
// (bitunpack_kernel) and copies / widens the UNCOMPRESSED values over theirs, in stream order.
extern "C" int cubit_table_add_segment_column(cubit_table* t, int col, int type, const uint8_t* bytes, uint64_t n_bytes,
                                              const uint64_t* seg_offsets, const uint64_t* seg_rows,
                                              const int32_t* seg_codecs, const int64_t* seg_constants,
                                              uint32_t n_segments, const uint64_t* validity) {
    if (!t) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    SegType st;
    if (!seg_type_of(type, st)) return fail(CUBIT_ERR_UNSUPPORTED, "type %d", type);
    if (col < 0) return fail(CUBIT_ERR_INVALID, "column %d", col);
    if (n_segments && (!seg_offsets || !seg_rows || !seg_codecs)) return fail(CUBIT_ERR_INVALID, "null argument");
    const bool wide = st.col_type != CUBIT_TYPE_INT32;
    const uint64_t esz = wide ? 8 : 4;
    const uint64_t bytes_padded = (n_bytes + 15) / 16 * 16;
    std::vector<int64_t> vals;
    std::vector<uint64_t> ends;
    std::vector<BpGroup> groups;
    std::vector<uint8_t> moved;
    struct Plain {
        uint64_t off, rows, row;
    };
    std::vector<Plain> plain;
    uint64_t row = 0;
    for (uint32_t sg = 0; sg < n_segments; ++sg) {
        const uint64_t rows = seg_rows[sg];
        const int codec = seg_codecs[sg];
        const bool needs_bytes = codec != CUBIT_CODEC_CONSTANT;
        if (needs_bytes && (!bytes || seg_offsets[sg] > n_bytes)) return fail(CUBIT_ERR_INVALID, "segment %u: bad offset", sg);
        switch (codec) {
        case CUBIT_CODEC_CONSTANT:
            if (!seg_constants) return fail(CUBIT_ERR_INVALID, "segment %u: CONSTANT without a value", sg);
            vals.push_back(seg_constants[sg]);
            ends.push_back(row + rows);
            break;
        case CUBIT_CODEC_RLE:
            if (int rc = parse_rle_segment(bytes, n_bytes, seg_offsets[sg], rows, row, st, vals, ends, sg)) return rc;
            break;
        case CUBIT_CODEC_BITPACKING:
            if (int rc = parse_bp_segment(bytes, n_bytes, seg_offsets[sg], rows, row, st, bytes_padded, groups, moved, sg))
                return rc;
            vals.push_back(0);  // placeholder, unpacked over below
            ends.push_back(row + rows);
            break;
        case CUBIT_CODEC_UNCOMPRESSED:
            if (seg_offsets[sg] % st.tsz || rows * st.tsz > n_bytes - seg_offsets[sg])
                return fail(CUBIT_ERR_INVALID, "segment %u: %llu values past the bytes", sg, (unsigned long long)rows);
            plain.push_back({seg_offsets[sg], rows, row});
            vals.push_back(0);  // placeholder, copied over below
            ends.push_back(row + rows);
            break;
        default:
            return fail(CUBIT_ERR_UNSUPPORTED, "segment %u: codec %d", sg, codec);
        }
        row += rows;
    }
    if (row != t->n_rows)
        return fail(CUBIT_ERR_INVALID, "segments hold %llu rows, partition has %llu", (unsigned long long)row,
                    (unsigned long long)t->n_rows);
    if (int rc = set_device(t->ctx)) return rc;
    hipStream_t s = t->ctx->stream;
    std::vector<int32_t> narrow;
    if (!wide) narrow.assign(vals.begin(), vals.end());
    const bool has_bytes = !groups.empty() || !plain.empty();
    DevBuf d_vals, d_ends, d_tiles, d_bytes, d_groups;
    auto out = std::make_unique<DevBuf>();
    const uint64_t n_tiles = (t->n_rows + 2047) / 2048;
    if (hipMalloc(&d_vals.p, std::max<uint64_t>(vals.size() * esz, 16)) != hipSuccess ||
        hipMalloc(&d_ends.p, std::max<uint64_t>(ends.size() * 8, 16)) != hipSuccess ||
        hipMalloc(&d_tiles.p, (n_tiles + 1) * 8) != hipSuccess ||
        hipMalloc(&out->p, std::max<uint64_t>(t->n_rows * esz, 16)) != hipSuccess ||
        (has_bytes && hipMalloc(&d_bytes.p, bytes_padded + moved.size() + 16) != hipSuccess) ||
        (!groups.empty() && hipMalloc(&d_groups.p, groups.size() * sizeof(BpGroup)) != hipSuccess))
        return fail(CUBIT_ERR_OOM, "segment column allocation failed");
    if (!vals.empty()) {
        HIP_CHECK(hipMemcpyAsync(d_vals.p, wide ? (const void*)vals.data() : (const void*)narrow.data(),
                                 vals.size() * esz, hipMemcpyHostToDevice, s));
        HIP_CHECK(hipMemcpyAsync(d_ends.p, ends.data(), ends.size() * 8, hipMemcpyHostToDevice, s));
    }
    if (has_bytes) {
        HIP_CHECK(hipMemcpyAsync(d_bytes.p, bytes, n_bytes, hipMemcpyHostToDevice, s));
        if (!moved.empty())
            HIP_CHECK(hipMemcpyAsync(static_cast<uint8_t*>(d_bytes.p) + bytes_padded, moved.data(), moved.size(),
                                     hipMemcpyHostToDevice, s));
    }
    hipEvent_t e0, e1;
    if (int rc = timing_events(t->ctx, e0, e1)) return rc;
    HIP_CHECK(launch_rle_expand(d_vals.p, static_cast<const uint64_t*>(d_ends.p), ends.size(), t->n_rows, wide ? 1 : 0,
                                static_cast<uint64_t*>(d_tiles.p), out->p, s, e0, groups.empty() && plain.empty() ? e1 : nullptr));
    if (!groups.empty()) {
        HIP_CHECK(hipMemcpyAsync(d_groups.p, groups.data(), groups.size() * sizeof(BpGroup), hipMemcpyHostToDevice, s));
        HIP_CHECK(launch_bitunpack(static_cast<const uint8_t*>(d_bytes.p), static_cast<const BpGroup*>(d_groups.p),
                                   groups.size(), st.col_type, out->p, s, nullptr, plain.empty() ? e1 : nullptr));
    }
    for (size_t i = 0; i < plain.size(); ++i) {
        const Plain& pl = plain[i];
        const uint8_t* src = static_cast<const uint8_t*>(d_bytes.p) + pl.off;
        uint8_t* dst = static_cast<uint8_t*>(out->p) + pl.row * esz;
        if (st.tsz == esz)  // INT32, INT64, UINT64: the values as held
            HIP_CHECK(hipMemcpyAsync(dst, src, pl.rows * esz, hipMemcpyDeviceToDevice, s));
        else
            HIP_CHECK(launch_widen(src, type, pl.rows, dst, s));
    }
    if (e1 && !plain.empty()) HIP_CHECK(hipEventRecord(e1, s));
    HIP_CHECK(hipStreamSynchronize(s));
    Column c;
    c.type = st.col_type;
    c.data = out->p;
    c.cap_rows = t->n_rows;
    c.owned.push_back(std::move(out));
    if (validity) {
        if (int rc = copy_validity(t, c, validity, 0)) return rc;
        HIP_CHECK(hipStreamSynchronize(s));
    }
    t->cols[col] = std::move(c);
    drop_patches(t, col);
    t->idx.erase(col);
    t->bins.erase(col);
    return CUBIT_OK;
}

extern "C" int cubit_table_build_index(cubit_table* t, int col, int encoding, const int64_t* values, uint32_t n) {
    if (!t) return fail(CUBIT_ERR_INVALID, "null table");
    CUBIT_LOCK(t->ctx);
    auto it = t->cols.find(col);
    if (it == t->cols.end()) return fail(CUBIT_ERR_INVALID, "column %d not registered", col);
    if (encoding != CUBIT_INDEX_RANGE && encoding != CUBIT_INDEX_EQUALITY && encoding != CUBIT_INDEX_BINS)
        return fail(CUBIT_ERR_INVALID, "encoding %d", encoding);
    if (encoding == CUBIT_INDEX_BINS && (n < 2 || !values)) return fail(CUBIT_ERR_INVALID, "bins need >= 2 edges");
    if (n && !values) return fail(CUBIT_ERR_INVALID, "values is null");
    if (int rc = set_device(t->ctx)) return rc;
    const Column& c = it->second;
    // a FLOAT / DOUBLE column's keys are given as bit patterns and held as their comparison keys
    // (-0.0 and +0.0, or two NaNs, become one key)
    std::vector<int64_t> keyed;
    if (n && type_is_keyed(c.type)) {
        keyed.resize(n);
        for (uint32_t k = 0; k < n; ++k) keyed[k] = value_key(c.type, values[k]);
        values = keyed.data();
    }
    // a VARCHAR column's keys are given as addresses of cubit_strings and held as the code bound
    // each names (the first code whose string is >= the key: exact for every key of RANGE and BINS,
    // and an EQUALITY key absent from the dictionary becomes a bitvector of its neighbour's code)
    if (n && c.type == CUBIT_TYPE_VARCHAR) {
        keyed.resize(n);
        for (uint32_t k = 0; k < n; ++k) {
            const cubit_string* str = reinterpret_cast<const cubit_string*>((intptr_t)values[k]);
            if (!str || (str->size && !str->data)) return fail(CUBIT_ERR_INVALID, "VARCHAR key %u is not a cubit_string", k);
            bool present = false;
            keyed[k] = (int64_t)c.dict->lower_bound(std::string_view(str->data ? str->data : "", str->size), &present);
        }
        values = keyed.data();
    }
    Index ix;
    ix.encoding = encoding;
    if (t->n_rows == 0) {  // empty partition: an empty index (scans of it launch nothing)
        ix.empty = true;
        ix.exact_all = n == 0;  // every distinct value of no rows; appends keep it exact
        if (n) ix.keys.assign(values, values + n);
        if (n && !std::is_sorted(ix.keys.begin(), ix.keys.end()))
            return fail(CUBIT_ERR_INVALID, "index keys must be sorted ascending");
        ix.keys.erase(std::unique(ix.keys.begin(), ix.keys.end()), ix.keys.end());
        if (encoding == CUBIT_INDEX_BINS && ix.keys.size() < 2) return fail(CUBIT_ERR_INVALID, "bins need >= 2 edges");
        drop_patches(t, col);
        if (encoding == CUBIT_INDEX_BINS) t->bins[col] = std::move(ix);
        else t->idx[col] = std::move(ix);
        return CUBIT_OK;
    }
    std::vector<int64_t> distinct;
    bool any = false;
    if (int rc = column_stats(t, c, distinct, n == 0, ix.vmin, ix.vmax, any)) return rc;
    ix.empty = !any;
    if (n == 0) {
        ix.exact_all = true;
        ix.keys = distinct;
        // range encoding: L(min) is empty, keep keys above the minimum
        if (encoding == CUBIT_INDEX_RANGE && !ix.keys.empty()) ix.keys.erase(ix.keys.begin());
    } else {
        ix.keys.assign(values, values + n);
        if (!std::is_sorted(ix.keys.begin(), ix.keys.end()))
            return fail(CUBIT_ERR_INVALID, "index keys must be sorted ascending");
        ix.keys.erase(std::unique(ix.keys.begin(), ix.keys.end()), ix.keys.end());
        if (encoding == CUBIT_INDEX_BINS && ix.keys.size() < 2) return fail(CUBIT_ERR_INVALID, "bins need >= 2 edges");
    }
    const size_t n_bv = encoding == CUBIT_INDEX_BINS ? ix.keys.size() - 1 : ix.keys.size();
    // one pass of the column per kMultiKeys bitvectors
    const int cmp = encoding == CUBIT_INDEX_BINS ? kCmpBetween : encoding == CUBIT_INDEX_RANGE ? CUBIT_CMP_LT : CUBIT_CMP_EQ;
    for (size_t k0 = 0; k0 < n_bv; k0 += kMultiKeys) {
        MultiKeyArgs mk{};
        for (size_t k = k0; k < std::min(n_bv, k0 + kMultiKeys); ++k) {
            auto b = std::make_unique<DevBuf>();
            if (int rc = alloc_table_bv(t, *b))
                return fail(rc, "index bitvector allocation failed after %zu of %zu", ix.bvs.size(), n_bv);
            mk.c[mk.m] = ix.keys[k];
            mk.c2[mk.m] = encoding == CUBIT_INDEX_BINS ? ix.keys[k + 1] : 0;
            mk.out[mk.m] = static_cast<uint64_t*>(b->p);
            ++mk.m;
            ix.bvs.push_back(static_cast<uint64_t*>(b->p));
            ix.owned.push_back(std::move(b));
            ix.bytes += t->cap_words * 8;
        }
        HIP_CHECK(launch_compare_bitvectors(c.data, ktype(c), c.validity, t->n_rows, cmp, mk, t->ctx->stream));
    }
    HIP_CHECK(hipStreamSynchronize(t->ctx->stream));
    drop_patches(t, col);
    if (encoding == CUBIT_INDEX_BINS) t->bins[col] = std::move(ix);
    else t->idx[col] = std::move(ix);
    return CUBIT_OK;
}

extern "C" int cubit_table_index_info(cubit_table* t, int col, uint32_t* n_bitvectors, uint64_t* bytes) {
    if (!t) return fail(CUBIT_ERR_INVALID, "null table");
    CUBIT_LOCK(t->ctx);
    uint32_t nb = 0;
    uint64_t by = 0;
    for (auto* m : {&t->idx, &t->bins}) {
        auto it = m->find(col);
        if (it != m->end()) {
            nb += (uint32_t)it->second.bvs.size();
            by += it->second.bytes;
        }
    }
    if (n_bitvectors) *n_bitvectors = nb;
    if (bytes) *bytes = by;
    return CUBIT_OK;
}

// ------------------------------------------------------------------ index persistence

namespace {

constexpr char kIndexMagic[8] = {'C', 'U', 'B', 'I', 'T', 'I', 'X', '1'};

struct IndexFileHeader {
    char magic[8];
    uint32_t version;
    uint32_t encoding;
    uint64_t n_rows;
    uint64_t nwp;
    uint32_t exact_all;
    uint32_t empty;
    int64_t vmin;
    int64_t vmax;
    uint64_t n_keys;
    uint64_t n_bv;
};
static_assert(sizeof(IndexFileHeader) == 72, "stable on-disk header");
// version 2 appends what the keys and leaves are relative to: the column's type (keys of FLOAT /
// DOUBLE are comparison keys, of VARCHAR / HUGEINT codes) and, for a dictionary column, its
// dictionary's fingerprint — codes of another dictionary would name other strings. A version-1
// file (no tail) loads onto a column that is not a dictionary column.
struct IndexFileTail {
    int32_t col_type;
    uint32_t reserved;
    uint64_t dict_fingerprint;
};
static_assert(sizeof(IndexFileTail) == 16, "stable on-disk tail");

}  // namespace

extern "C" int cubit_table_save_index(cubit_table* t, int col, int encoding, const char* path) {
    if (!t || !path) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    const Index* ix = nullptr;
    if (encoding == CUBIT_INDEX_BINS) {
        auto it = t->bins.find(col);
        if (it != t->bins.end()) ix = &it->second;
    } else {
        auto it = t->idx.find(col);
        if (it != t->idx.end() && it->second.encoding == encoding) ix = &it->second;
    }
    if (!ix) return fail(CUBIT_ERR_INVALID, "column %d has no index of encoding %d", col, encoding);
    if (int rc = set_device(t->ctx)) return rc;
    HIP_CHECK(hipStreamSynchronize(t->ctx->stream));
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(CUBIT_ERR_INVALID, "cannot open %s for writing", path);
    IndexFileHeader h{};
    std::memcpy(h.magic, kIndexMagic, 8);
    h.version = 2;
    const Column& sc = t->cols.at(col);
    const IndexFileTail tail{sc.type, 0u, sc.dict ? sc.dict->fingerprint : 0ull};
    h.encoding = (uint32_t)ix->encoding;
    h.n_rows = t->n_rows;
    h.nwp = t->nwp;
    h.exact_all = ix->exact_all ? 1u : 0u;
    h.empty = ix->empty ? 1u : 0u;
    h.vmin = ix->vmin;
    h.vmax = ix->vmax;
    h.n_keys = ix->keys.size();
    h.n_bv = ix->bvs.size();
    bool ok = std::fwrite(&h, sizeof(h), 1, f) == 1 && std::fwrite(&tail, sizeof(tail), 1, f) == 1 &&
              (h.n_keys == 0 || std::fwrite(ix->keys.data(), 8, h.n_keys, f) == h.n_keys);
    std::vector<uint64_t> host(ok ? t->nwp : 0);
    for (size_t k = 0; ok && k < ix->bvs.size(); ++k) {
        if (hipMemcpy(host.data(), ix->bvs[k], t->nwp * 8, hipMemcpyDeviceToHost) != hipSuccess) {
            std::fclose(f);
            return fail(CUBIT_ERR_HIP, "index download failed");
        }
        ok = std::fwrite(host.data(), 8, t->nwp, f) == t->nwp;
    }
    ok = (std::fclose(f) == 0) && ok;
    return ok ? CUBIT_OK : fail(CUBIT_ERR_INVALID, "short write to %s", path);
}

extern "C" int cubit_table_load_index(cubit_table* t, int col, const char* path) {
    if (!t || !path) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    if (!t->cols.count(col)) return fail(CUBIT_ERR_INVALID, "column %d not registered", col);
    if (int rc = set_device(t->ctx)) return rc;
    FILE* f = std::fopen(path, "rb");
    if (!f) return fail(CUBIT_ERR_INVALID, "cannot open %s", path);
    auto bad = [&](const char* why) {
        std::fclose(f);
        return fail(CUBIT_ERR_INVALID, "%s: %s", path, why);
    };
    IndexFileHeader h{};
    if (std::fread(&h, sizeof(h), 1, f) != 1 || std::memcmp(h.magic, kIndexMagic, 8) != 0 ||
        (h.version != 1 && h.version != 2))
        return bad("not a cubit index file");
    const Column& lc = t->cols.at(col);
    if (h.version == 2) {
        IndexFileTail tail{};
        if (std::fread(&tail, sizeof(tail), 1, f) != 1) return bad("truncated header");
        if (tail.col_type != lc.type) return bad("index was built on a column of another type");
        if (tail.dict_fingerprint != (lc.dict ? lc.dict->fingerprint : 0ull))
            return bad("index was built against another dictionary");
    } else if (lc.dict) {
        return bad("a version-1 index file does not name its dictionary");
    }
    if (h.n_rows != t->n_rows || h.nwp != t->nwp) return bad("index was built for a partition of another size");
    if (h.encoding > CUBIT_INDEX_BINS) return bad("unknown encoding");
    const uint64_t want_bv = h.encoding == CUBIT_INDEX_BINS ? (h.n_keys ? h.n_keys - 1 : 0) : h.n_keys;
    if (h.n_bv != want_bv || h.n_keys > (1ull << 32)) return bad("inconsistent header");
    Index ix;
    ix.encoding = (int)h.encoding;
    ix.exact_all = h.exact_all != 0;
    ix.empty = h.empty != 0;
    ix.vmin = h.vmin;
    ix.vmax = h.vmax;
    ix.keys.resize(h.n_keys);
    if (h.n_keys && std::fread(ix.keys.data(), 8, h.n_keys, f) != h.n_keys) return bad("truncated keys");
    if (!std::is_sorted(ix.keys.begin(), ix.keys.end())) return bad("keys not sorted");
    std::vector<uint64_t> host(t->nwp);
    for (uint64_t k = 0; k < h.n_bv; ++k) {
        if (std::fread(host.data(), 8, t->nwp, f) != t->nwp) return bad("truncated bitvectors");
        auto b = std::make_unique<DevBuf>();
        if (alloc_table_bv(t, *b)) {
            std::fclose(f);
            return fail(CUBIT_ERR_OOM, "index bitvector allocation failed");
        }
        if (hipMemcpy(b->p, host.data(), t->nwp * 8, hipMemcpyHostToDevice) != hipSuccess) {
            std::fclose(f);
            return fail(CUBIT_ERR_HIP, "index upload failed");
        }
        ix.bvs.push_back(static_cast<uint64_t*>(b->p));
        ix.owned.push_back(std::move(b));
        ix.bytes += t->cap_words * 8;
    }
    std::fclose(f);
    drop_patches(t, col);
    if (ix.encoding == CUBIT_INDEX_BINS) t->bins[col] = std::move(ix);
    else t->idx[col] = std::move(ix);
    return CUBIT_OK;
}

extern "C" int cubit_table_set_deletes(cubit_table* t, const int64_t* rows, const uint64_t* ids, uint64_t n) {
    if (!t || (n && (!rows || !ids))) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    if (int rc = set_device(t->ctx)) return rc;
    for (uint64_t i = 0; i < n; ++i)
        if (rows[i] < 0 || (uint64_t)rows[i] >= t->n_rows) return fail(CUBIT_ERR_INVALID, "delete row out of range");
    t->del_rows = std::make_unique<DevBuf>();
    t->del_ids = std::make_unique<DevBuf>();
    if (hipMalloc(&t->del_rows->p, std::max<uint64_t>(n, 1) * 8) != hipSuccess ||
        hipMalloc(&t->del_ids->p, std::max<uint64_t>(n, 1) * 8) != hipSuccess)
        return fail(CUBIT_ERR_OOM, "delete list allocation failed");
    if (n) {
        HIP_CHECK(hipMemcpy(t->del_rows->p, rows, n * 8, hipMemcpyHostToDevice));
        HIP_CHECK(hipMemcpy(t->del_ids->p, ids, n * 8, hipMemcpyHostToDevice));
    }
    t->n_del = n;
    t->del_ids_sorted.assign(ids, ids + n);
    std::sort(t->del_ids_sorted.begin(), t->del_ids_sorted.end());
    t->vis_prefix = -1;
    return CUBIT_OK;
}

extern "C" int cubit_table_set_inserts(cubit_table* t, const int64_t* row_begin, const int64_t* row_end,
                                       const uint64_t* ids, uint64_t n) {
    if (!t || (n && (!row_begin || !row_end || !ids))) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    std::vector<cubit_table::InsRange> r(n);
    for (uint64_t i = 0; i < n; ++i) {
        if (row_begin[i] < 0 || row_begin[i] >= row_end[i] || (uint64_t)row_end[i] > t->n_rows)
            return fail(CUBIT_ERR_INVALID, "insert range %llu out of range", (unsigned long long)i);
        r[i] = {row_begin[i], row_end[i], ids[i]};
    }
    std::sort(r.begin(), r.end(), [](const auto& a, const auto& b) { return a.begin < b.begin; });
    for (uint64_t i = 1; i < n; ++i)
        if (r[i].begin < r[i - 1].end) return fail(CUBIT_ERR_INVALID, "insert ranges overlap");
    std::stable_sort(r.begin(), r.end(), [](const auto& a, const auto& b) { return a.id < b.id; });
    t->ins = std::move(r);
    t->vis_prefix = -1;
    t->vis_ins_prefix = -1;
    return CUBIT_OK;
}

namespace {

// The distinct values of v, ascending. Update lists hold millions of records over few
// distinct values: a presence bitmap over [min, max] when that span is small, else sort.
std::vector<int64_t> distinct_sorted(const int64_t* v, uint64_t n) {
    std::vector<int64_t> out;
    if (n == 0) return out;
    const auto mm = std::minmax_element(v, v + n);
    const uint64_t span = (uint64_t)*mm.second - (uint64_t)*mm.first;
    if (span < (1ull << 26)) {
        std::vector<uint64_t> bits(span / 64 + 1, 0);
        for (uint64_t i = 0; i < n; ++i) {
            const uint64_t d = (uint64_t)v[i] - (uint64_t)*mm.first;
            bits[d >> 6] |= 1ull << (d & 63);
        }
        for (uint64_t w = 0; w < bits.size(); ++w)
            for (uint64_t x = bits[w]; x; x &= x - 1)
                out.push_back((int64_t)((uint64_t)*mm.first + w * 64 + (uint64_t)__builtin_ctzll(x)));
        return out;
    }
    out.assign(v, v + n);
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
}

// store an update list (rows, values, versions, and NULL-ness when valids is not null) for col:
// records grouped by row, each row's records kept in chronological order (UpdateInfo chains,
// update_info.hpp)
int store_updates(cubit_table* t, int col, const int64_t* rows, const int64_t* values, const uint64_t* versions,
                  uint64_t n, const uint8_t* valids = nullptr) {
    std::vector<uint64_t> order(n);
    for (uint64_t i = 0; i < n; ++i) order[i] = i;
    if (!std::is_sorted(rows, rows + n))  // grouping keeps each row's records in list order
        std::stable_sort(order.begin(), order.end(), [&](uint64_t x, uint64_t y) { return rows[x] < rows[y]; });
    Updates u;
    u.n = n;
    const int type = t->cols.at(col).type;
    for (uint64_t i = 0; valids && i < n; ++i) u.any_null |= valids[i] == 0;
    u.h_rows.reserve(n);
    u.h_values.reserve(n);
    u.h_versions.reserve(n);
    for (uint64_t i : order) {
        if (!u.h_rows.empty() && u.h_rows.back() == rows[i]) u.unique_rows = false;
        u.h_rows.push_back(rows[i]);
        // a FLOAT value is its 32-bit pattern, zero-extended (as the probe hands it back)
        u.h_values.push_back(type == CUBIT_TYPE_FLOAT ? (int64_t)(uint32_t)values[i] : values[i]);
        u.h_versions.push_back(versions[i]);
        if (u.any_null) u.h_valids.push_back(valids[i] ? 1 : 0);
    }
    {
        const auto dv = distinct_sorted(reinterpret_cast<const int64_t*>(u.h_versions.data()), n);
        // versions are unsigned: distinct_sorted ordered them as signed, restore unsigned order
        u.distinct_versions.assign(dv.begin(), dv.end());
        std::sort(u.distinct_versions.begin(), u.distinct_versions.end());
    }
    {  // the statistics cover the records that carry a value (FLOAT / DOUBLE: their keys)
        std::vector<int64_t> vv;
        vv.reserve(n);
        for (uint64_t i = 0; i < n; ++i)
            if (u.valid_at(i)) vv.push_back(value_key(type, u.h_values[i]));
        u.stat_values = distinct_sorted(vv.data(), vv.size());
    }
    u.rows = std::make_unique<DevBuf>();
    u.values = std::make_unique<DevBuf>();
    u.versions = std::make_unique<DevBuf>();
    if (hipMalloc(&u.rows->p, std::max<uint64_t>(n, 1) * 8) != hipSuccess ||
        hipMalloc(&u.values->p, std::max<uint64_t>(n, 1) * 8) != hipSuccess ||
        hipMalloc(&u.versions->p, std::max<uint64_t>(n, 1) * 8) != hipSuccess)
        return fail(CUBIT_ERR_OOM, "update list allocation failed");
    if (n) {
        HIP_CHECK(hipMemcpy(u.rows->p, u.h_rows.data(), n * 8, hipMemcpyHostToDevice));
        HIP_CHECK(hipMemcpy(u.values->p, u.h_values.data(), n * 8, hipMemcpyHostToDevice));
        HIP_CHECK(hipMemcpy(u.versions->p, u.h_versions.data(), n * 8, hipMemcpyHostToDevice));
    }
    if (u.any_null) {
        u.valids = std::make_unique<DevBuf>();
        if (hipMalloc(&u.valids->p, n) != hipSuccess) return fail(CUBIT_ERR_OOM, "update list allocation failed");
        HIP_CHECK(hipMemcpy(u.valids->p, u.h_valids.data(), n, hipMemcpyHostToDevice));
    }
    t->upd[col] = std::move(u);
    return CUBIT_OK;
}

}  // namespace

extern "C" int cubit_table_set_updates(cubit_table* t, int col, const int64_t* rows, const int64_t* values,
                                       const uint64_t* versions, uint64_t n) {
    if (!t || (n && (!rows || !values || !versions))) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    if (!t->cols.count(col)) return fail(CUBIT_ERR_INVALID, "column %d not registered", col);
    if (int rc = set_device(t->ctx)) return rc;
    for (uint64_t i = 0; i < n; ++i)
        if (rows[i] < 0 || (uint64_t)rows[i] >= t->n_rows) return fail(CUBIT_ERR_INVALID, "update row out of range");
    if (int rc = check_codes(t->cols.at(col), values, nullptr, n)) return rc;
    return store_updates(t, col, rows, values, versions, n);
}

namespace {

// A validity bitvector for a column registered without one (every row valid): a SET NULL
// record, visible or merged, needs the NN leaf to patch or flip (the planner folds IS NOT NULL on
// a column without validity to TRUE).
int ensure_validity(cubit_table* t, Column& c) {
    if (c.validity) return CUBIT_OK;
    auto b = std::make_unique<DevBuf>();
    if (int rc = alloc_table_bv(t, *b)) return fail(rc, "validity allocation failed");
    if (t->n_rows) HIP_CHECK(launch_fill_valid(static_cast<uint64_t*>(b->p), t->n_rows, t->ctx->stream));
    c.validity = static_cast<const uint64_t*>(b->p);
    c.owned.push_back(std::move(b));
    drop_zones(t);
    return CUBIT_OK;
}

}  // namespace

extern "C" int cubit_table_set_updates_nullable(cubit_table* t, int col, const int64_t* rows, const int64_t* values,
                                                const uint8_t* valid, const uint64_t* versions, uint64_t n) {
    if (!t || (n && (!rows || !values || !versions))) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    auto cit = t->cols.find(col);
    if (cit == t->cols.end()) return fail(CUBIT_ERR_INVALID, "column %d not registered", col);
    if (int rc = set_device(t->ctx)) return rc;
    bool any_null = false;
    for (uint64_t i = 0; i < n; ++i) {
        if (rows[i] < 0 || (uint64_t)rows[i] >= t->n_rows) return fail(CUBIT_ERR_INVALID, "update row out of range");
        any_null |= valid && !valid[i];
    }
    if (int rc = check_codes(cit->second, values, valid, n)) return rc;
    if (any_null)
        if (int rc = ensure_validity(t, cit->second)) return rc;
    return store_updates(t, col, rows, values, versions, n, any_null ? valid : nullptr);
}

// ------------------------------------------------------------------ index maintenance

namespace {

// Every table-owned bitvector (index leaves, bins, validity) grown to `words` words: copy the
// nwp words in use, zero the rest. Index leaf pointers change, so everything derived from them
// (patched leaves, scratch) is dropped by the caller.
int grow_bitvectors(cubit_table* t, uint64_t words) {
    drop_zones(t);
    hipStream_t s = t->ctx->stream;
    auto regrow = [&](void*& p) -> int {
        void* np = nullptr;
        if (hipMalloc(&np, words * 8) != hipSuccess) return fail(CUBIT_ERR_OOM, "bitvector growth failed");
        HIP_CHECK(hipMemsetAsync(np, 0, words * 8, s));
        if (p && t->nwp) HIP_CHECK(hipMemcpyAsync(np, p, t->nwp * 8, hipMemcpyDeviceToDevice, s));
        HIP_CHECK(hipStreamSynchronize(s));
        if (p) (void)hipFree(p);
        p = np;
        return CUBIT_OK;
    };
    for (auto* m : {&t->idx, &t->bins}) {
        for (auto& kv : *m) {
            Index& ix = kv.second;
            for (size_t k = 0; k < ix.owned.size(); ++k) {
                if (int rc = regrow(ix.owned[k]->p)) return rc;
                ix.bvs[k] = static_cast<uint64_t*>(ix.owned[k]->p);
            }
            ix.bytes = ix.owned.size() * words * 8;
        }
    }
    for (auto& kv : t->cols) {
        Column& c = kv.second;
        if (!c.validity) continue;
        for (auto& b : c.owned) {
            if (b->p != (const void*)c.validity) continue;
            if (int rc = regrow(b->p)) return rc;
            c.validity = static_cast<const uint64_t*>(b->p);
            break;
        }
    }
    t->cap_words = words;
    return CUBIT_OK;
}

// an owned data buffer of at least `rows` rows holding the column's first n_rows values
int own_column(cubit_table* t, Column& c, uint64_t rows) {
    if (c.cap_rows >= rows && c.cap_rows) return CUBIT_OK;
    const uint64_t esz = type_is32(c.type) ? 4 : 8;
    auto b = std::make_unique<DevBuf>();
    if (hipMalloc(&b->p, std::max<uint64_t>(rows * esz, 16)) != hipSuccess)
        return fail(CUBIT_ERR_OOM, "column allocation failed");
    if (c.data && t->n_rows)
        HIP_CHECK(hipMemcpyAsync(b->p, c.data, t->n_rows * esz, hipMemcpyDeviceToDevice, t->ctx->stream));
    HIP_CHECK(hipStreamSynchronize(t->ctx->stream));
    // release the old owned data buffer (not the validity buffer)
    for (auto it = c.owned.begin(); it != c.owned.end(); ++it)
        if ((*it)->p == c.data) {
            c.owned.erase(it);
            break;
        }
    c.data = b->p;
    c.cap_rows = rows;
    c.owned.push_back(std::move(b));
    if (type_is_fp(c.type)) {  // the patterns grow beside the keys
        auto r = std::make_unique<DevBuf>();
        if (hipMalloc(&r->p, std::max<uint64_t>(rows * esz, 16)) != hipSuccess)
            return fail(CUBIT_ERR_OOM, "column allocation failed");
        if (t->n_rows)
            HIP_CHECK(hipMemcpyAsync(r->p, c.raw, t->n_rows * esz, hipMemcpyDeviceToDevice, t->ctx->stream));
        HIP_CHECK(hipStreamSynchronize(t->ctx->stream));
        c.raw_buf = std::move(r);
        c.raw = c.raw_buf->p;
    }
    return CUBIT_OK;
}

// The keys an exact_all index must hold after the column gained the values `added` (sorted,
// distinct, all valid): RANGE keeps every distinct value but the minimum, EQUALITY every
// distinct value. Missing keys get full-column bitvectors (the column already holds its new
// values); more than kMaxNewKeys missing keys turn the index into an edges index instead
// (exact for its keys, the candidate check for other constants).
constexpr size_t kMaxNewKeys = 64;
int maintain_exact_keys(cubit_table* t, int col, Index& ix, const std::vector<int64_t>& added, int64_t old_min,
                        bool was_empty) {
    if (!ix.exact_all || ix.encoding == CUBIT_INDEX_BINS || added.empty()) return CUBIT_OK;
    std::vector<int64_t> want;  // keys the index must hold
    if (ix.encoding == CUBIT_INDEX_RANGE) {
        // old distinct values ⊆ keys ∪ {old_min}; the new minimum needs no key
        if (!was_empty && old_min > ix.vmin) want.push_back(old_min);
        for (int64_t v : added)
            if (v > ix.vmin) want.push_back(v);
    } else {
        want = added;
    }
    std::vector<int64_t> missing;
    for (int64_t v : want)
        if (!std::binary_search(ix.keys.begin(), ix.keys.end(), v)) missing.push_back(v);
    std::sort(missing.begin(), missing.end());
    missing.erase(std::unique(missing.begin(), missing.end()), missing.end());
    if (missing.empty()) return CUBIT_OK;
    if (missing.size() > kMaxNewKeys) {
        ix.exact_all = false;
        return CUBIT_OK;
    }
    const Column& c = t->cols.at(col);
    const int cmp = ix.encoding == CUBIT_INDEX_RANGE ? CUBIT_CMP_LT : CUBIT_CMP_EQ;
    std::vector<std::pair<int64_t, std::unique_ptr<DevBuf>>> fresh;
    for (size_t k0 = 0; k0 < missing.size(); k0 += kMultiKeys) {
        MultiKeyArgs mk{};
        for (size_t k = k0; k < std::min(missing.size(), k0 + kMultiKeys); ++k) {
            auto b = std::make_unique<DevBuf>();
            if (int rc = alloc_table_bv(t, *b)) return fail(rc, "index bitvector allocation failed");
            mk.c[mk.m] = missing[k];
            mk.out[mk.m] = static_cast<uint64_t*>(b->p);
            ++mk.m;
            fresh.emplace_back(missing[k], std::move(b));
        }
        HIP_CHECK(launch_compare_bitvectors(c.data, ktype(c), c.validity, t->n_rows, cmp, mk, t->ctx->stream));
    }
    HIP_CHECK(hipStreamSynchronize(t->ctx->stream));
    // merge into the sorted key list (keys, bvs and owned stay parallel)
    std::vector<int64_t> keys;
    std::vector<uint64_t*> bvs;
    std::vector<std::unique_ptr<DevBuf>> owned;
    size_t i = 0, j = 0;
    std::vector<std::unique_ptr<DevBuf>> old_owned = std::move(ix.owned);
    while (i < ix.keys.size() || j < fresh.size()) {
        if (j == fresh.size() || (i < ix.keys.size() && ix.keys[i] < fresh[j].first)) {
            keys.push_back(ix.keys[i]);
            bvs.push_back(ix.bvs[i]);
            owned.push_back(std::move(old_owned[i]));
            ++i;
        } else {
            keys.push_back(fresh[j].first);
            bvs.push_back(static_cast<uint64_t*>(fresh[j].second->p));
            owned.push_back(std::move(fresh[j].second));
            ++j;
        }
    }
    ix.keys = std::move(keys);
    ix.bvs = std::move(bvs);
    ix.owned = std::move(owned);
    ix.bytes = ix.owned.size() * t->cap_words * 8;
    return CUBIT_OK;
}

// bitvectors an index of this encoding holds for its keys
size_t index_bv_count(const Index& ix) {
    return ix.encoding == CUBIT_INDEX_BINS ? (ix.keys.size() >= 2 ? ix.keys.size() - 1 : 0) : ix.keys.size();
}

}  // namespace

// Append rows to the partition (RowGroupCollection::Append + every BoundIndex::Append,
// bound_index.hpp:67-70): the new rows get local ids n_rows … n_rows + n_new - 1. Values are
// host arrays, one per registered column (cols[i] names the column of data[i]); validity[i]
// (LSB-first words for the appended rows, bit 0 = first appended row) may be null = all valid.
// Every index of every column is maintained incrementally: the index-build compare kernel runs
// over the appended slice only and its words are spliced into each bitvector at bit n_rows;
// statistics widen, and an index over every distinct value gains keys for new values.
// insert_id ≠ 0 records the rows as an insert range of that transaction (ChunkVectorInfo
// inserted ids): readers with start_time ≤ insert_id (other than the inserting transaction)
// do not see them. Storage grows in place, geometrically, when the padding is exhausted.
extern "C" int cubit_table_append(cubit_table* t, uint64_t n_new, const int* cols, const void* const* data,
                                  const uint64_t* const* validity, uint32_t n_cols, uint64_t insert_id) {
    if (!t || (n_cols && (!cols || !data))) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    if (n_new == 0) return CUBIT_OK;
    const uint64_t n_old = t->n_rows, n_total = n_old + n_new;
    if (n_total >= (1ull << 47) || n_total < n_old)
        return fail(CUBIT_ERR_INVALID, "%llu rows exceed 2^47", (unsigned long long)n_total);
    if (n_cols != t->cols.size())
        return fail(CUBIT_ERR_INVALID, "append gives %u columns, the table has %zu", n_cols, t->cols.size());
    std::map<int, uint32_t> at;
    for (uint32_t i = 0; i < n_cols; ++i) {
        if (!t->cols.count(cols[i])) return fail(CUBIT_ERR_INVALID, "column %d not registered", cols[i]);
        if (!data[i]) return fail(CUBIT_ERR_INVALID, "column %d: null data", cols[i]);
        if (!at.emplace(cols[i], i).second) return fail(CUBIT_ERR_INVALID, "column %d given twice", cols[i]);
        const Column& c = t->cols.at(cols[i]);
        if (c.type == CUBIT_TYPE_VARCHAR) {  // the appended codes name dictionary strings (NULL rows: any)
            const int32_t* codes = static_cast<const int32_t*>(data[i]);
            const uint64_t* vw = validity ? validity[i] : nullptr;
            for (uint64_t r = 0; r < n_new; ++r)
                if ((!vw || ((vw[r >> 6] >> (r & 63)) & 1ull)) && (codes[r] < 0 || (uint64_t)codes[r] >= c.dict->size()))
                    return fail(CUBIT_ERR_INVALID, "column %d: appended code %d outside the dictionary", cols[i], codes[r]);
        }
    }
    if (int rc = set_device(t->ctx)) return rc;
    hipStream_t s = t->ctx->stream;
    HIP_CHECK(hipStreamSynchronize(s));
    drop_zones(t);  // every bitvector gains the appended rows
    // 1. capacity: bitvectors and columns grow together (×1.25 at least)
    const uint64_t need_words = padded_words(n_total);
    if (need_words > t->cap_words) {
        const uint64_t words = std::max(need_words, padded_words(n_old + n_old / 4));
        if (int rc = grow_bitvectors(t, words)) return rc;
    }
    for (auto& kv : t->cols)
        if (int rc = own_column(t, kv.second, std::max(n_total, kv.second.cap_rows >= n_total ? kv.second.cap_rows
                                                                                          : t->cap_words * 64)))
            return rc;
    // 2. per column: values, validity, then every index on it
    const uint64_t slice_words = padded_words(n_new);
    DevBuf tmp_col, tmp_valid, tmp_bits;
    const uint32_t n_tmp_bv = (uint32_t)kMultiKeys;
    if (hipMalloc(&tmp_col.p, n_new * 8 + 16) != hipSuccess || hipMalloc(&tmp_valid.p, slice_words * 8) != hipSuccess ||
        hipMalloc(&tmp_bits.p, slice_words * 8 * n_tmp_bv) != hipSuccess)
        return fail(CUBIT_ERR_OOM, "append staging allocation failed");
    for (auto& kv : t->cols) {
        const int col = kv.first;
        Column& c = kv.second;
        c.drop_packed();  // the segments do not hold the appended rows
        const uint32_t i = at[col];
        const uint64_t esz = type_is32(c.type) ? 4 : 8;
        HIP_CHECK(hipMemcpyAsync(tmp_col.p, data[i], n_new * esz, hipMemcpyHostToDevice, s));
        if (type_is_fp(c.type)) {  // the patterns appended as given, the slice keyed in place for the rest
            HIP_CHECK(hipMemcpyAsync(static_cast<char*>(const_cast<void*>(c.raw)) + n_old * esz, tmp_col.p,
                                     n_new * esz, hipMemcpyDeviceToDevice, s));
            HIP_CHECK(launch_fp_keys(tmp_col.p, c.type, n_new, tmp_col.p, s));
        }
        HIP_CHECK(hipMemcpyAsync(static_cast<char*>(const_cast<void*>(c.data)) + n_old * esz, tmp_col.p, n_new * esz,
                                 hipMemcpyDeviceToDevice, s));
        const uint64_t* slice_valid = nullptr;
        if (validity && validity[i]) {
            HIP_CHECK(hipMemsetAsync(tmp_valid.p, 0, slice_words * 8, s));
            HIP_CHECK(hipMemcpyAsync(tmp_valid.p, validity[i], (n_new + 63) / 64 * 8, hipMemcpyHostToDevice, s));
            if (n_new & 63) {  // bits past the appended rows are not rows
                uint64_t last = validity[i][(n_new - 1) / 64] & ((1ull << (n_new & 63)) - 1);
                HIP_CHECK(hipMemcpyAsync(static_cast<uint64_t*>(tmp_valid.p) + (n_new - 1) / 64, &last, 8,
                                         hipMemcpyHostToDevice, s));
                HIP_CHECK(hipStreamSynchronize(s));
            }
            slice_valid = static_cast<const uint64_t*>(tmp_valid.p);
            if (!c.validity) {  // first NULLs of the column: the old rows are all valid
                auto b = std::make_unique<DevBuf>();
                if (int rc = alloc_table_bv(t, *b)) return fail(rc, "validity allocation failed");
                if (n_old) HIP_CHECK(launch_fill_valid(static_cast<uint64_t*>(b->p), n_old, s));
                c.validity = static_cast<const uint64_t*>(b->p);
                c.owned.push_back(std::move(b));
            }
            HIP_CHECK(launch_splice_bits(const_cast<uint64_t*>(c.validity), slice_valid, n_old, n_new, s));
        } else if (c.validity) {  // a column with NULLs gets all-valid rows
            HIP_CHECK(launch_fill_valid(static_cast<uint64_t*>(tmp_valid.p), n_new, s));
            HIP_CHECK(launch_splice_bits(const_cast<uint64_t*>(c.validity), static_cast<const uint64_t*>(tmp_valid.p),
                                         n_old, n_new, s));
        }
        Index* ixs[2] = {t->idx.count(col) ? &t->idx[col] : nullptr, t->bins.count(col) ? &t->bins[col] : nullptr};
        if (!ixs[0] && !ixs[1]) continue;
        // statistics of the appended slice (+ its distinct values for an every-distinct-value index)
        bool want_distinct = ixs[0] && ixs[0]->exact_all;
        std::vector<int64_t> added;
        int64_t smin = 0, smax = 0;
        bool sany = false;
        int rc = value_stats(t, tmp_col.p, ktype(c), slice_valid, n_new, added, want_distinct, smin, smax, sany);
        if (rc == CUBIT_ERR_UNSUPPORTED && want_distinct) {  // too wide a span for a presence bitmap
            ixs[0]->exact_all = false;
            want_distinct = false;
            rc = value_stats(t, tmp_col.p, ktype(c), slice_valid, n_new, added, false, smin, smax, sany);
        }
        if (rc) return rc;
        for (Index* ix : ixs) {
            if (!ix) continue;
            const int enc = ix->encoding;
            const size_t n_bv = index_bv_count(*ix);
            while (ix->owned.size() < n_bv) {  // an index built on an empty partition has no bitvectors yet
                auto b = std::make_unique<DevBuf>();
                if (int rc2 = alloc_table_bv(t, *b)) return fail(rc2, "index bitvector allocation failed");
                ix->owned.push_back(std::move(b));
            }
            ix->bvs.resize(n_bv);
            for (size_t k = 0; k < n_bv; ++k) ix->bvs[k] = static_cast<uint64_t*>(ix->owned[k]->p);
            ix->bytes = ix->owned.size() * t->cap_words * 8;
            const int cmp = enc == CUBIT_INDEX_BINS ? kCmpBetween : enc == CUBIT_INDEX_RANGE ? CUBIT_CMP_LT : CUBIT_CMP_EQ;
            for (size_t k0 = 0; k0 < n_bv; k0 += kMultiKeys) {
                MultiKeyArgs mk{};
                for (size_t k = k0; k < std::min(n_bv, k0 + kMultiKeys); ++k) {
                    mk.c[mk.m] = ix->keys[k];
                    mk.c2[mk.m] = enc == CUBIT_INDEX_BINS ? ix->keys[k + 1] : 0;
                    mk.out[mk.m] = static_cast<uint64_t*>(tmp_bits.p) + (uint64_t)mk.m * slice_words;
                    ++mk.m;
                }
                HIP_CHECK(launch_compare_bitvectors(tmp_col.p, ktype(c), slice_valid, n_new, cmp, mk, s));
                for (uint32_t m = 0; m < mk.m; ++m)
                    HIP_CHECK(launch_splice_bits(ix->bvs[k0 + m], mk.out[m], n_old, n_new, s));
            }
            if (sany) {
                const bool was_empty = ix->empty;
                const int64_t old_min = ix->vmin;
                ix->vmin = was_empty ? smin : std::min(ix->vmin, smin);
                ix->vmax = was_empty ? smax : std::max(ix->vmax, smax);
                ix->empty = false;
                // the new keys' bitvectors span the whole column: counted with the new rows
                t->n_rows = n_total;
                t->nwp = need_words;
                rc = maintain_exact_keys(t, col, *ix, added, old_min, was_empty);
                t->n_rows = n_old;
                t->nwp = padded_words(n_old);
                if (rc) return rc;
            }
        }
        HIP_CHECK(hipStreamSynchronize(s));  // tmp_col / tmp_valid reused by the next column
    }
    HIP_CHECK(hipStreamSynchronize(s));
    t->n_rows = n_total;
    t->nwp = need_words;
    if (insert_id) {
        t->ins.push_back({(int64_t)n_old, (int64_t)n_total, insert_id});
        std::stable_sort(t->ins.begin(), t->ins.end(), [](const auto& a, const auto& b) { return a.id < b.id; });
    }
    drop_derived(t);
    return CUBIT_OK;
}

// Merge committed updates of one column into its base values and indexes (the checkpoint of
// update chains; CUBIT folds its update bitvectors into the index the same way). Every record
// with version < horizon — visible to every snapshot the caller still serves (start_time ≥
// horizon, as DuckDB's lowest active start bounds what a checkpoint may fold) — leaves the
// update list: each row takes its newest such value (records of a row are chronological; the
// merged records are the row's prefix below horizon) and its NULL-ness, and every index bitvector
// of the column whose membership can change is rewritten for each 64-row word holding a merged
// row (merge_words_kernel). Records
// at or past horizon stay in the list. *n_merged (optional) = rows whose base changed.
extern "C" int cubit_table_merge_updates(cubit_table* t, int col, uint64_t horizon, uint64_t* n_merged) {
    if (!t) return fail(CUBIT_ERR_INVALID, "null table");
    CUBIT_LOCK(t->ctx);
    if (n_merged) *n_merged = 0;
    auto cit = t->cols.find(col);
    if (cit == t->cols.end()) return fail(CUBIT_ERR_INVALID, "column %d not registered", col);
    auto uit = t->upd.find(col);
    if (uit == t->upd.end() || uit->second.n == 0) return CUBIT_OK;
    if (int rc = set_device(t->ctx)) return rc;
    hipStream_t s = t->ctx->stream;
    Column& c = cit->second;
    const Updates& u = uit->second;
    // The merged records: each row's newest record below horizon. When every record is below it
    // and each row has one record (a checkpoint after the writers committed: the common case),
    // that is the update list itself, already on the device, and nothing is left.
    const bool all = u.unique_rows && u.distinct_versions.back() < horizon;
    std::vector<int64_t> m_rows, m_vals, k_rows, k_vals;
    std::vector<uint8_t> m_valid, k_valid;
    std::vector<uint64_t> k_vers;
    bool m_null = all && u.any_null;
    uint64_t m = all ? u.n : 0;
    if (!all) {
        for (uint64_t i = 0; i < u.n;) {
            uint64_t j = i;
            while (j < u.n && u.h_rows[j] == u.h_rows[i]) ++j;
            uint64_t p = i;  // merged prefix [i, p)
            while (p < j && u.h_versions[p] < horizon) ++p;
            if (p > i) {
                const int64_t v = u.h_values[p - 1];
                const bool ok = u.valid_at(p - 1);  // the newest merged record decides value and NULL-ness
                m_rows.push_back(u.h_rows[i]);
                m_vals.push_back(ok ? v : 0);
                m_valid.push_back(ok ? 1 : 0);
                m_null |= !ok;
            }
            for (uint64_t q = p; q < j; ++q) {
                k_rows.push_back(u.h_rows[q]);
                k_vals.push_back(u.h_values[q]);
                k_vers.push_back(u.h_versions[q]);
                k_valid.push_back(u.valid_at(q) ? 1 : 0);
            }
            i = j;
        }
        m = m_rows.size();
    }
    if (m == 0) return CUBIT_OK;
    // the merged values' distinct valid values: the statistics and exact keys they add
    std::vector<int64_t> added;
    if (all) {
        added = u.stat_values;  // the records' distinct valid values, computed when they were set
    } else {
        std::vector<int64_t> valid_vals;
        for (uint64_t i = 0; i < m; ++i)
            if (m_valid[i]) valid_vals.push_back(value_key(c.type, m_vals[i]));
        added = distinct_sorted(valid_vals.data(), valid_vals.size());
    }
    if (c.type == CUBIT_TYPE_INT32 && !added.empty() && (added.front() < INT32_MIN || added.back() > INT32_MAX))
        return fail(CUBIT_ERR_INVALID, "merged value %lld does not fit an INT32 column",
                    (long long)(added.front() < INT32_MIN ? added.front() : added.back()));
    HIP_CHECK(hipStreamSynchronize(s));
    drop_zones(t);  // the merge rewrites index words in place
    if (int rc = own_column(t, c, std::max<uint64_t>(t->n_rows, c.cap_rows))) return rc;
    if (m_null)
        if (int rc = ensure_validity(t, c)) return rc;
    c.drop_packed();  // merged values are not in the segments
    DevBuf d_rows, d_vals, d_valid;
    const int64_t* rows_p;
    const int64_t* vals_p;
    const uint8_t* valid_p;
    if (all) {
        rows_p = static_cast<const int64_t*>(u.rows->p);
        vals_p = static_cast<const int64_t*>(u.values->p);
        valid_p = u.any_null ? u.d_valids() : nullptr;  // a NULL record holds value 0 (store_updates)
    } else {
        if (hipMalloc(&d_rows.p, m * 8) != hipSuccess || hipMalloc(&d_vals.p, m * 8) != hipSuccess ||
            (m_null && hipMalloc(&d_valid.p, m) != hipSuccess))
            return fail(CUBIT_ERR_OOM, "merge list allocation failed");
        HIP_CHECK(hipMemcpyAsync(d_rows.p, m_rows.data(), m * 8, hipMemcpyHostToDevice, s));
        HIP_CHECK(hipMemcpyAsync(d_vals.p, m_vals.data(), m * 8, hipMemcpyHostToDevice, s));
        if (m_null) HIP_CHECK(hipMemcpyAsync(d_valid.p, m_valid.data(), m, hipMemcpyHostToDevice, s));
        rows_p = static_cast<const int64_t*>(d_rows.p);
        vals_p = static_cast<const int64_t*>(d_vals.p);
        valid_p = m_null ? static_cast<const uint8_t*>(d_valid.p) : nullptr;
    }
    Index* ixs[2] = {t->idx.count(col) ? &t->idx[col] : nullptr, t->bins.count(col) ? &t->bins[col] : nullptr};
    MergeIndex mi[2] = {};
    DevBuf d_keys[2], d_bvs[2];
    for (int x = 0; x < 2; ++x) {
        Index* ix = ixs[x];
        if (!ix || index_bv_count(*ix) == 0 || ix->bvs.size() != index_bv_count(*ix)) continue;
        if (hipMalloc(&d_keys[x].p, ix->keys.size() * 8) != hipSuccess ||
            hipMalloc(&d_bvs[x].p, ix->bvs.size() * sizeof(uint64_t*)) != hipSuccess)
            return fail(CUBIT_ERR_OOM, "merge index descriptor allocation failed");
        HIP_CHECK(hipMemcpyAsync(d_keys[x].p, ix->keys.data(), ix->keys.size() * 8, hipMemcpyHostToDevice, s));
        HIP_CHECK(hipMemcpyAsync(d_bvs[x].p, ix->bvs.data(), ix->bvs.size() * sizeof(uint64_t*), hipMemcpyHostToDevice, s));
        mi[x].keys = static_cast<const int64_t*>(d_keys[x].p);
        mi[x].bvs = static_cast<uint64_t* const*>(d_bvs[x].p);
        mi[x].n_keys = (uint32_t)ix->keys.size();
        mi[x].encoding = ix->encoding == CUBIT_INDEX_RANGE ? 0 : ix->encoding == CUBIT_INDEX_EQUALITY ? 1 : 2;
    }
    // every 64-row word holding merged rows, rewritten by one wave (rows ascend, each once)
    // FLOAT / DOUBLE: the merge compares and writes keys (the key column is what the indexes were built
    // from); the patterns are scattered into the pattern column beside it
    DevBuf d_keys_of;
    const int64_t* merge_vals = vals_p;
    if (type_is_fp(c.type)) {
        if (hipMalloc(&d_keys_of.p, m * 8) != hipSuccess) return fail(CUBIT_ERR_OOM, "merge key allocation failed");
        HIP_CHECK(launch_value_keys(vals_p, m, c.type, static_cast<int64_t*>(d_keys_of.p), s));
        merge_vals = static_cast<const int64_t*>(d_keys_of.p);
    }
    HIP_CHECK(launch_merge_words(rows_p, merge_vals, valid_p, m, t->n_rows, const_cast<void*>(c.data), ktype(c),
                                 const_cast<uint64_t*>(c.validity), mi[0], mi[1], s));
    if (type_is_fp(c.type))
        HIP_CHECK(launch_scatter_raw(rows_p, vals_p, valid_p, m, c.type, const_cast<void*>(c.raw), s));
    HIP_CHECK(hipStreamSynchronize(s));
    // statistics and exact keys for the merged values (a merged NULL leaves the index bounds:
    // they only have to contain the valid values)
    for (Index* ix : ixs) {
        if (!ix || added.empty()) continue;
        const bool was_empty = ix->empty;
        const int64_t old_min = ix->vmin;
        ix->vmin = was_empty ? added.front() : std::min(ix->vmin, added.front());
        ix->vmax = was_empty ? added.back() : std::max(ix->vmax, added.back());
        ix->empty = false;
        if (int rc = maintain_exact_keys(t, col, *ix, added, old_min, was_empty)) return rc;
    }
    // the records left (each row's suffix at or past horizon), still grouped and chronological
    if (k_rows.empty()) {
        t->upd.erase(col);
    } else if (int rc = store_updates(t, col, k_rows.data(), k_vals.data(), k_vers.data(), k_rows.size(),
                                      k_valid.data())) {
        return rc;
    }
    drop_derived(t);
    if (n_merged) *n_merged = m;
    return CUBIT_OK;
}

// ------------------------------------------------------------------ planner

namespace {

// An index as the planner may use it: its keys and bitvectors with statistics widened by the
// column's update records (any version: wider bounds are always safe). Folding a constant
// against the base statistics alone would drop rows whose visible updated value lies outside
// them, and "every distinct value" exactness holds only while every updated value is a key.
struct IndexView {
    int encoding;
    bool exact_all, empty;
    int64_t vmin, vmax;
    const std::vector<int64_t>& keys;
    const std::vector<uint64_t*>& bvs;
};

IndexView view_of(const cubit_table* t, int col, const Index& ix) {
    IndexView v{ix.encoding, ix.exact_all, ix.empty, ix.vmin, ix.vmax, ix.keys, ix.bvs};
    auto uit = t->upd.find(col);
    if (uit == t->upd.end() || uit->second.stat_values.empty()) return v;
    const std::vector<int64_t>& uv = uit->second.stat_values;
    v.vmin = ix.empty ? uv.front() : std::min(ix.vmin, uv.front());
    v.vmax = ix.empty ? uv.back() : std::max(ix.vmax, uv.back());
    v.empty = false;
    if (v.exact_all) {
        auto is_key = [&](int64_t x) { return std::binary_search(ix.keys.begin(), ix.keys.end(), x); };
        if (ix.encoding == CUBIT_INDEX_RANGE) {
            // values ⊆ keys ∪ {vmin}: the base minimum and every updated value
            if (!ix.empty && ix.vmin != v.vmin && !is_key(ix.vmin)) v.exact_all = false;
            for (int64_t x : uv)
                if (x != v.vmin && !is_key(x)) {
                    v.exact_all = false;
                    break;
                }
        } else {
            for (int64_t x : uv)
                if (!is_key(x)) {
                    v.exact_all = false;
                    break;
                }
        }
    }
    return v;
}

// A K0 leaf whose bitvector is not built yet: {valid rows: v cmp c} of column col into bv.
struct PendingK0 {
    uint64_t* bv;
    int col, cmp;
    int64_t c;
};

// Build a K0 leaf over the whole column (from the BITPACKING segments when enabled).
int compute_k0(cubit_table* t, const PendingK0& k) {
    const Column& cl = t->cols.at(k.col);
    hipError_t e;
    // (UBIGINT segments: the packed compare orders values as signed; such columns compare unpacked)
    if (cl.bp_n_groups && t->use_packed && cl.type != CUBIT_TYPE_UINT64) {
        // straight from the BITPACKING segments: w/8 bytes per row instead of sizeof(T)
        e = hipMemsetAsync(k.bv, 0, t->nwp * 8, t->ctx->stream);
        if (e == hipSuccess)
            e = launch_bitpacked_compare(static_cast<const uint8_t*>(cl.bp_bytes->p),
                                         static_cast<const BpGroup*>(cl.bp_groups->p), cl.bp_n_groups, cl.type,
                                         cl.validity, k.cmp, k.c, 0, k.bv, t->ctx->stream, cl.bp_simple_width);
        t->last_packed++;
    } else {
        e = launch_compare_bitvector(cl.data, ktype(cl), cl.validity, t->n_rows, k.cmp, k.c, k.bv, t->ctx->stream);
    }
    if (e != hipSuccess) return fail(CUBIT_ERR_HIP, "compare kernel: %s", hipGetErrorString(e));
    return CUBIT_OK;
}

struct Planner {
    cubit_table* t;
    const cubit_filter_node* nodes;
    uint32_t n_nodes;
    int rc = CUBIT_OK;

    int subtree_end(uint32_t i) {
        if (i >= n_nodes) return -1;
        uint32_t j = i + 1;
        for (int k = 0; k < nodes[i].n_children; ++k) {
            int e = subtree_end(j);
            if (e < 0) return -1;
            j = (uint32_t)e;
        }
        return (int)j;
    }

    ExprP nn(int col) {
        const Column& c = t->cols.at(col);
        if (!c.validity) return mk_true();
        Leaf l;
        l.bv = c.validity;
        l.column = col;
        l.pred = 1;
        l.zsrc = kZoneBits;
        return mk_leaf(l);
    }

    // K0 fallback: the comparison from the raw column into a scratch bitvector. The launch is
    // deferred (pending) until the plan is complete: inside a conjunction it may be narrowed to
    // the rows the other filters keep (narrow_k0), as the reference's filter loop does.
    std::vector<PendingK0> pending;
    ExprP raw_compare(int col, int cmp, int64_t c) {
        uint64_t* bv = nullptr;
        if ((rc = scratch_bv(t, &bv))) return nullptr;
        pending.push_back({bv, col, cmp, c});
        Leaf l;
        l.bv = bv;
        l.column = col;
        l.cmp = cmp;
        l.constant = c;
        l.zsrc = kZoneStats;
        return mk_leaf(l);
    }

    // {v < c} from a range index; nullptr when the index cannot answer exactly
    ExprP range_lt(int col, const IndexView& ix, int64_t c) {
        if (ix.empty || c <= ix.vmin) return mk_false();
        if (c > ix.vmax) return nn(col);
        auto it = std::lower_bound(ix.keys.begin(), ix.keys.end(), c);
        if (it != ix.keys.end() && (*it == c || ix.exact_all)) {
            Leaf l;
            l.bv = ix.bvs[it - ix.keys.begin()];
            l.column = col;
            l.cmp = CUBIT_CMP_LT;
            l.constant = *it;
            l.zsrc = kZoneBits;
            return mk_leaf(l);
        }
        return nullptr;
    }

    // {v < c} (cmp LT) or {v == c} (cmp EQ) for a constant that is not a key of the range
    // index: the constant lies in one bin [k_lo, k_hi) between neighbouring keys, and only that
    // bin's rows are checked on the raw column (launch_candidate_check). This is the binned
    // bitmap index's candidate check: reads L(k_lo), L(k_hi) and the column at the bin's rows
    // instead of K0's whole column. nullptr when the bin is estimated (uniform values over
    // [vmin, vmax]) to hold more than a quarter of the rows, where K0's sequential read of the
    // column is cheaper; rc is set on a launch or allocation failure.
    ExprP candidate(int col, const IndexView& ix, int cmp, int64_t c) {
        auto hi_it = std::upper_bound(ix.keys.begin(), ix.keys.end(), c);  // first key > c
        const bool has_lo = hi_it != ix.keys.begin(), has_hi = hi_it != ix.keys.end();
        const double lo_v = has_lo ? (double)*(hi_it - 1) : (double)ix.vmin;
        const double hi_v = has_hi ? (double)*hi_it : (double)ix.vmax + 1.0;
        const double span = (double)ix.vmax - (double)ix.vmin + 1.0;
        if ((std::min(hi_v, (double)ix.vmax + 1.0) - std::max(lo_v, (double)ix.vmin)) > 0.25 * span) return nullptr;
        const Column& cl = t->cols.at(col);
        uint64_t* bv = nullptr;
        if ((rc = scratch_bv(t, &bv))) return nullptr;
        const uint64_t* lo_bv = has_lo ? ix.bvs[hi_it - 1 - ix.keys.begin()] : nullptr;
        const uint64_t* hi_bv = has_hi ? ix.bvs[hi_it - ix.keys.begin()] : nullptr;
        hipError_t e = launch_candidate_check(cl.data, ktype(cl), cl.validity, lo_bv, hi_bv, t->n_rows, cmp, c, bv,
                                              t->ctx->stream);
        if (e != hipSuccess) {
            rc = fail(CUBIT_ERR_HIP, "candidate check kernel: %s", hipGetErrorString(e));
            return nullptr;
        }
        Leaf l;
        l.bv = bv;
        l.column = col;
        l.cmp = cmp;
        l.constant = c;
        l.zsrc = kZoneStats;
        return mk_leaf(l);
    }

    // lo <= v < hi (either side open) on a column whose equality index holds every distinct
    // value (exact_all): the union of the keys' bitvectors inside, or the valid rows minus the
    // union of those outside — the fewer leaves; nullptr when both exceed 16.
    ExprP eq_interval(int col, const IndexView& ix, int64_t lo, int64_t hi, bool has_lo, bool has_hi) {
        const size_t b = has_lo ? (size_t)(std::lower_bound(ix.keys.begin(), ix.keys.end(), lo) - ix.keys.begin()) : 0;
        const size_t e = has_hi ? (size_t)(std::lower_bound(ix.keys.begin(), ix.keys.end(), hi) - ix.keys.begin())
                                : ix.keys.size();
        auto leaf = [&](size_t k) {
            Leaf l;
            l.bv = ix.bvs[k];
            l.column = col;
            l.cmp = CUBIT_CMP_EQ;
            l.constant = ix.keys[k];
            l.zsrc = kZoneBits;
            return mk_leaf(l);
        };
        const size_t inside = e > b ? e - b : 0, outside = ix.keys.size() - inside;
        if (inside <= 16 && inside <= outside + 1) {
            ExprP acc = mk_false();
            for (size_t k = b; k < e; ++k) acc = mk_bin(Expr::OR, acc, leaf(k));
            return acc;
        }
        if (outside > 16) return nullptr;
        ExprP out = mk_false();
        for (size_t k = 0; k < ix.keys.size(); ++k)
            if (k < b || k >= e) out = mk_bin(Expr::OR, out, leaf(k));
        return mk_bin(Expr::ANDNOT, nn(col), out);
    }

    // the column's equality index when it holds every distinct value (an interval over it is a
    // union of its bitvectors), else null
    const Index* exact_equality(int col) const {
        auto it = t->idx.find(col);
        return it != t->idx.end() && it->second.encoding == CUBIT_INDEX_EQUALITY && it->second.exact_all &&
                       !it->second.empty
                   ? &it->second
                   : nullptr;
    }

    ExprP eq_leaf(int col, const IndexView& ix, int64_t c, bool& exact) {
        exact = true;
        auto it = std::lower_bound(ix.keys.begin(), ix.keys.end(), c);
        if (it != ix.keys.end() && *it == c) {
            Leaf l;
            l.bv = ix.bvs[it - ix.keys.begin()];
            l.column = col;
            l.cmp = CUBIT_CMP_EQ;
            l.constant = c;
            l.zsrc = kZoneBits;
            return mk_leaf(l);
        }
        if (ix.exact_all || ix.empty || c < ix.vmin || c > ix.vmax) return mk_false();
        exact = false;
        return nullptr;
    }

    ExprP constant(int col, int cmp, int64_t c) {
        auto ixit = t->idx.find(col);
        if (ixit != t->idx.end()) {
            const IndexView ix = view_of(t, col, ixit->second);
            const bool top = c == INT64_MAX;
            if (ix.encoding == CUBIT_INDEX_RANGE) {
                // {v < k}: an index leaf when k is a key, else the candidate check of k's bin
                auto lt = [&](int64_t k) -> ExprP {
                    ExprP e = range_lt(col, ix, k);
                    return e ? e : candidate(col, ix, CUBIT_CMP_LT, k);
                };
                ExprP r;
                switch (cmp) {
                case CUBIT_CMP_LT: r = lt(c); break;
                case CUBIT_CMP_LE: r = top ? nn(col) : lt(c + 1); break;
                case CUBIT_CMP_GT: {
                    ExprP e = top ? nn(col) : lt(c + 1);
                    r = e ? mk_bin(Expr::ANDNOT, nn(col), e) : nullptr;
                    break;
                }
                case CUBIT_CMP_GE: {
                    ExprP e = lt(c);
                    r = e ? mk_bin(Expr::ANDNOT, nn(col), e) : nullptr;
                    break;
                }
                case CUBIT_CMP_EQ:
                case CUBIT_CMP_NE: {
                    ExprP lt_c = range_lt(col, ix, c);
                    ExprP lt_c1 = top ? nn(col) : range_lt(col, ix, c + 1);
                    if (lt_c && lt_c1) {
                        r = cmp == CUBIT_CMP_EQ ? mk_bin(Expr::ANDNOT, lt_c1, lt_c)
                                                : mk_bin(Expr::OR, mk_bin(Expr::ANDNOT, nn(col), lt_c1), lt_c);
                    } else if (ExprP eq = candidate(col, ix, CUBIT_CMP_EQ, c)) {
                        r = cmp == CUBIT_CMP_EQ ? eq : mk_bin(Expr::ANDNOT, nn(col), eq);
                    }
                    break;
                }
                default: break;
                }
                if (rc) return nullptr;
                if (r) return r;
            } else {
                bool exact = true;
                if (cmp == CUBIT_CMP_EQ) {
                    ExprP e = eq_leaf(col, ix, c, exact);
                    if (exact) return e;
                } else if (cmp == CUBIT_CMP_NE) {
                    ExprP e = eq_leaf(col, ix, c, exact);
                    if (exact) return mk_bin(Expr::ANDNOT, nn(col), e);
                } else if (ix.exact_all) {
                    // the equality bitvectors in range, or the valid rows outside the others
                    // (whichever reads fewer); wide ranges both ways go to K0
                    const bool has_lo = cmp == CUBIT_CMP_GT || cmp == CUBIT_CMP_GE;
                    int64_t lo = 0, hi = 0;
                    bool empty = false;
                    if (cmp == CUBIT_CMP_GE) lo = c;
                    else if (cmp == CUBIT_CMP_GT) empty = c == INT64_MAX, lo = empty ? c : c + 1;
                    else if (cmp == CUBIT_CMP_LT) hi = c;
                    else if (c == INT64_MAX) return nn(col);
                    else hi = c + 1;
                    if (empty) return mk_false();
                    if (ExprP e = eq_interval(col, ix, lo, hi, has_lo, !has_lo)) return e;
                }
            }
        }
        return raw_compare(col, cmp, c);
    }

    // Cheapest exact plan of lo <= v < hi (half-open, from folded constant filters) out of
    // the column's binned index, or nullptr when the bins cannot answer it in fewer leaves than
    // the range index would (2, or 1 for a one-sided bound).
    ExprP interval_from_bins(int col, int64_t lo, int64_t hi, bool has_lo, bool has_hi) {
        auto bit = t->bins.find(col);
        if (bit == t->bins.end()) return nullptr;
        const IndexView b = view_of(t, col, bit->second);
        if (b.empty) return mk_false();
        const std::vector<int64_t>& e = b.keys;
        const size_t nb = e.size() - 1;
        size_t first, last;  // bins [first, last)
        if (!has_lo || lo <= b.vmin) {
            if (e.front() > b.vmin) return nullptr;  // rows below the first edge are in no bin
            first = 0;
        } else {
            auto it = std::lower_bound(e.begin(), e.end(), lo);
            if (it == e.end() || *it != lo) return nullptr;
            first = (size_t)(it - e.begin());
        }
        if (!has_hi || hi > b.vmax) {
            if (e.back() <= b.vmax) return nullptr;  // rows at or above the last edge
            last = nb;
        } else {
            auto it = std::lower_bound(e.begin(), e.end(), hi);
            if (it == e.end() || *it != hi) return nullptr;
            last = (size_t)(it - e.begin());
        }
        if (last <= first) return mk_false();
        const size_t range_cost = (has_lo && lo > b.vmin ? 1 : 0) + (has_hi && hi <= b.vmax ? 1 : 0);
        if (last - first >= std::max<size_t>(range_cost, 1) && t->idx.count(col)) return nullptr;
        if (last - first > 16) return nullptr;
        ExprP acc = mk_false();
        for (size_t k = first; k < last; ++k) {
            Leaf l;
            l.bv = b.bvs[k];
            l.column = col;
            l.pred = 2;
            l.constant = e[k];
            l.constant2 = e[k + 1];
            l.zsrc = kZoneBits;
            acc = mk_bin(Expr::OR, acc, mk_leaf(l));
        }
        return acc;
    }

    // AND node: constant comparisons on one column fold into an interval first (DuckDB
    // pushes "a <= x AND x < b" as one ConjunctionAndFilter on x, table_filter.cpp:20-40).
    ExprP plan_and(uint32_t i) {
        const cubit_filter_node& f = nodes[i];
        struct Bounds {
            int64_t lo = INT64_MIN, hi = INT64_MAX;
            bool has_lo = false, has_hi = false, empty = false;
            std::vector<uint32_t> members;
        };
        std::map<int, Bounds> by_col;
        std::vector<uint32_t> kids;
        uint32_t j = i + 1;
        for (int k = 0; k < f.n_children; ++k) {
            kids.push_back(j);
            const cubit_filter_node& c = nodes[j];
            if (c.kind == CUBIT_FILTER_CONSTANT && c.n_children == 0 && c.cmp != CUBIT_CMP_NE && c.cmp >= 0 &&
                c.cmp <= 5 && (t->bins.count(c.column) || exact_equality(c.column))) {
                Bounds& bd = by_col[c.column];
                const int64_t v = c.constant;
                auto lower = [&](int64_t x) { bd.lo = bd.has_lo ? std::max(bd.lo, x) : x; bd.has_lo = true; };
                auto upper = [&](int64_t x) { bd.hi = bd.has_hi ? std::min(bd.hi, x) : x; bd.has_hi = true; };
                switch (c.cmp) {
                case CUBIT_CMP_GE: lower(v); break;
                case CUBIT_CMP_GT: if (v == INT64_MAX) bd.empty = true; else lower(v + 1); break;
                case CUBIT_CMP_LT: upper(v); break;
                case CUBIT_CMP_LE: if (v != INT64_MAX) upper(v + 1); break;
                case CUBIT_CMP_EQ:  // [v, v + 1); v = INT64_MAX: [v, ∞) is {v} (a UBIGINT 2^64 - 1's key)
                    lower(v);
                    if (v != INT64_MAX) upper(v + 1);
                    break;
                default: break;
                }
                bd.members.push_back(j);
            }
            j = (uint32_t)subtree_end(j);
        }
        std::vector<char> done(n_nodes, 0);
        ExprP acc = mk_true();
        for (auto& [col, bd] : by_col) {
            ExprP e;
            if (bd.empty || (bd.has_lo && bd.has_hi && bd.hi <= bd.lo)) e = mk_false();
            else if (t->bins.count(col)) e = interval_from_bins(col, bd.lo, bd.hi, bd.has_lo, bd.has_hi);
            if (!e && !rc && bd.members.size() > 1) {
                // two or more bounds on an every-value equality index: one union for the interval
                if (const Index* eq = exact_equality(col)) {
                    const IndexView v = view_of(t, col, *eq);  // exact only while every updated value is a key
                    if (v.exact_all && !v.empty) e = eq_interval(col, v, bd.lo, bd.hi, bd.has_lo, bd.has_hi);
                }
            }
            if (rc) return nullptr;
            if (!e) continue;
            for (uint32_t m : bd.members) done[m] = 1;
            acc = mk_bin(Expr::AND, acc, e);
        }
        for (uint32_t k : kids) {
            if (done[k]) continue;
            ExprP c = plan(k);
            if (!c) return nullptr;
            acc = mk_bin(Expr::AND, acc, c);
        }
        return acc;
    }

    ExprP plan(uint32_t i) {
        if (rc) return nullptr;
        const cubit_filter_node& f = nodes[i];
        switch (f.kind) {
        case CUBIT_FILTER_AND:
            return plan_and(i);
        case CUBIT_FILTER_OR: {
            ExprP acc = mk_false();
            uint32_t j = i + 1;
            for (int k = 0; k < f.n_children; ++k) {
                ExprP c = plan(j);
                if (!c) return nullptr;
                acc = mk_bin(Expr::OR, acc, c);
                j = (uint32_t)subtree_end(j);
            }
            return acc;
        }
        case CUBIT_FILTER_CONSTANT:
        case CUBIT_FILTER_IS_NULL:
        case CUBIT_FILTER_IS_NOT_NULL: {
            if (!t->cols.count(f.column)) {
                rc = fail(CUBIT_ERR_INVALID, "filter references unregistered column %d", f.column);
                return nullptr;
            }
            if (f.kind == CUBIT_FILTER_IS_NOT_NULL) return nn(f.column);
            if (f.kind == CUBIT_FILTER_IS_NULL) return mk_not(nn(f.column));
            if (f.cmp < 0 || f.cmp > 5) {
                rc = fail(CUBIT_ERR_INVALID, "comparison %d", f.cmp);
                return nullptr;
            }
            return constant(f.column, f.cmp, f.constant);
        }
        default:
            rc = fail(CUBIT_ERR_INVALID, "filter node kind %d", f.kind);
            return nullptr;
        }
    }
};

// Materialise a subexpression into a scratch bitvector (bits-only pass).
int materialize(cubit_table* t, const ExprP& e, uint64_t** out) {
    Emitter em;
    em.emit_top(e);
    if (!em.ok || em.max_depth > 4) return fail(CUBIT_ERR_UNSUPPORTED, "subexpression too deep");
    if (int rc = scratch_bv(t, out)) return rc;
    t->last_passes++;
    return run_eval(t->ctx, em.prog, t->n_rows, 0, nullptr, 0, t->dummy_count, *out, RunMode::kCount);
}

bool fits(const ExprP& e);
int fit(cubit_table* t, ExprP& e);
double literal_selectivity(cubit_table* t, const Leaf& l, bool neg, int* rc);
double conj_selectivity(cubit_table* t, const Emitter::Lits& lits, int* rc);

// top-level conjuncts of e (a & ~leaf contributes the complemented leaf as a conjunct)
void conj_parts(const ExprP& e, std::vector<ExprP>& out) {
    if (e->kind == Expr::AND) {
        conj_parts(e->a, out);
        conj_parts(e->b, out);
    } else if (e->kind == Expr::ANDNOT && e->b->kind == Expr::LEAF) {
        conj_parts(e->a, out);
        out.push_back(mk_leaf(e->b->leaf, !e->b->neg));
    } else if (e->kind != Expr::CONST_TRUE) {
        out.push_back(e);
    }
}
void leaves_of(const ExprP& e, std::vector<const uint64_t*>& out) {
    if (e->kind == Expr::LEAF) out.push_back(e->leaf.bv);
    else if (e->a) {
        leaves_of(e->a, out);
        if (e->b) leaves_of(e->b, out);
    }
}
// estimated fraction of rows a subtree keeps, from its literals' estimates
double expr_selectivity(cubit_table* t, const ExprP& e, int* rc) {
    switch (e->kind) {
    case Expr::LEAF: return literal_selectivity(t, e->leaf, e->neg, rc);
    case Expr::AND: return expr_selectivity(t, e->a, rc) * expr_selectivity(t, e->b, rc);
    case Expr::OR: return std::min(1.0, expr_selectivity(t, e->a, rc) + expr_selectivity(t, e->b, rc));
    case Expr::ANDNOT: return expr_selectivity(t, e->a, rc) * (1.0 - expr_selectivity(t, e->b, rc));
    case Expr::CONST_TRUE: return 1.0;
    default: return 0.0;
    }
}

// Selection narrowing of K0 leaves (RowGroup::TemplatedScan's filter loop, row_group.cpp:537-550:
// each filter column after the first is read only at the rows the earlier ones kept). When the
// planned expression is a conjunction of literals holding non-negated K0 leaves, the other
// literals are materialised into a mask; with none, the most selective K0 comparison is built in
// full and is the mask. Each remaining K0 leaf, most selective first, is then built by
// masked_compare_kernel — its column read only at the mask's rows, the result already the AND
// with the mask, and the next leaf's mask — and the conjunction becomes that one leaf. The order
// and the decision come from selectivity estimates of every literal over the columns' per-zone
// min / max (literal_selectivity; the statistics the zonemaps use, computed once per table
// version), the reference's AdaptiveFilter ordering its filters by observed cost
// (adaptive_filter.cpp:21-88) made up front: when the mask is estimated to keep more than one
// row in 32, the K0 leaves are built in full (gathering most lines costs more than reading the
// column in order). The other conjuncts need not be literals: a union of equality bitvectors (an
// interval on an every-value equality index) or any subtree joins the mask, its selectivity
// estimated from its literals (OR: their sum, AND: their product). No count is read back:
// planning never waits for the device. allow = false
// (visible MVCC updates, whose patches need whole leaves) builds every leaf in full. Every
// pending leaf is built on return; t->last_narrow_cols lists the K0 columns in build order.
int narrow_k0(cubit_table* t, ExprP& e, std::vector<PendingK0>& pending, bool allow) {
    t->last_narrow_cols.clear();
    auto compute_rest = [&]() -> int {
        for (const PendingK0& k : pending) {
            if (int rc = compute_k0(t, k)) return rc;
            t->last_narrow_cols.push_back(k.col);
        }
        pending.clear();
        return CUBIT_OK;
    };
    auto take = [&](const uint64_t* bv, PendingK0* out) {
        for (size_t i = 0; i < pending.size(); ++i)
            if (pending[i].bv == bv) {
                if (out) *out = pending[i];
                pending.erase(pending.begin() + (long)i);
                return true;
            }
        return false;
    };
    auto is_pending = [&](const uint64_t* bv) {
        return std::any_of(pending.begin(), pending.end(), [&](const PendingK0& k) { return k.bv == bv; });
    };
    if (pending.empty()) return CUBIT_OK;
    if (!allow || t->n_rows == 0 || e->kind == Expr::LEAF) return compute_rest();
    std::vector<ExprP> parts;
    conj_parts(e, parts);
    Emitter::Lits lits;  // the literal conjuncts
    std::vector<ExprP> others;  // the other conjuncts (unions, subtrees)
    for (const ExprP& p : parts) {
        if (p->kind == Expr::LEAF) lits.push_back({p->leaf, p->neg});
        else others.push_back(p);
    }
    std::vector<const uint64_t*> narrow_bvs;
    Emitter::Lits rest;
    for (const auto& lit : lits) {
        if (!lit.second && is_pending(lit.first.bv) &&
            std::find(narrow_bvs.begin(), narrow_bvs.end(), lit.first.bv) == narrow_bvs.end())
            narrow_bvs.push_back(lit.first.bv);
        else
            rest.push_back(lit);
    }
    std::vector<const uint64_t*> other_bvs;
    for (const ExprP& p : others) leaves_of(p, other_bvs);
    for (const auto& lit : rest)  // a narrowed leaf must not also be read whole
        if (std::find(narrow_bvs.begin(), narrow_bvs.end(), lit.first.bv) != narrow_bvs.end()) return compute_rest();
    for (const uint64_t* bv : other_bvs)
        if (std::find(narrow_bvs.begin(), narrow_bvs.end(), bv) != narrow_bvs.end()) return compute_rest();
    if (narrow_bvs.empty()) return compute_rest();
    // selectivity estimates: the mask of the other conjuncts (independent columns: the
    // product; literals on one column as one interval), each K0 comparison
    int rc = CUBIT_OK;
    double rest_sel = conj_selectivity(t, rest, &rc);
    for (const ExprP& p : others) rest_sel *= expr_selectivity(t, p, &rc);
    if (rc) return rc;
    std::vector<std::pair<double, PendingK0>> narrow;
    for (const uint64_t* bv : narrow_bvs) {
        Leaf l;
        for (const auto& lit : lits)
            if (lit.first.bv == bv) l = lit.first;
        const double s = literal_selectivity(t, l, false, &rc);
        if (rc) return rc;
        PendingK0 k;
        take(bv, &k);
        narrow.push_back({s, k});
    }
    // most selective first (ties: column order, so the plan does not depend on the text order)
    std::sort(narrow.begin(), narrow.end(), [](const auto& x, const auto& y) {
        return x.first != y.first ? x.first < y.first
                                  : (x.second.col != y.second.col ? x.second.col < y.second.col : x.second.c < y.second.c);
    });
    std::vector<const uint64_t*> rest_bvs = other_bvs;  // K0 leaves inside the other conjuncts: in full
    for (const auto& lit : rest) rest_bvs.push_back(lit.first.bv);
    for (const uint64_t* bv : rest_bvs) {
        PendingK0 k;
        if (take(bv, &k)) {
            if (int rc2 = compute_k0(t, k)) return rc2;
            t->last_narrow_cols.push_back(k.col);
        }
    }
    const bool has_rest = !rest.empty() || !others.empty();
    const double mask_sel = has_rest ? rest_sel : narrow.front().first;
    uint64_t* mask = nullptr;
    cubit_ctx* ctx = t->ctx;
    if (has_rest) {
        ExprP r = mk_true();
        for (const auto& lit : rest) r = mk_bin(Expr::AND, r, mk_leaf(lit.first, lit.second));
        for (const ExprP& p : others) r = mk_bin(Expr::AND, r, p);
        if (mask_sel * 32 > 1.0) {
            for (const auto& kv : narrow) pending.push_back(kv.second);
            return compute_rest();
        }
        if (int rc2 = fit(t, r)) return rc2;  // a mask of more leaves than one pass: split
        if (int rc2 = materialize(t, r, &mask)) return rc2;
    } else {
        const PendingK0 first = narrow.front().second;
        narrow.erase(narrow.begin());
        if (int rc2 = compute_k0(t, first)) return rc2;
        t->last_narrow_cols.push_back(first.col);
        mask = first.bv;
        if (mask_sel * 32 > 1.0) {  // too dense a mask: every other K0 leaf in full
            Leaf ml;
            ml.bv = mask;
            ExprP acc = mk_leaf(ml);
            for (const auto& kv : narrow) {
                if (int rc2 = compute_k0(t, kv.second)) return rc2;
                t->last_narrow_cols.push_back(kv.second.col);
                Leaf l;
                l.bv = kv.second.bv;
                acc = mk_bin(Expr::AND, acc, mk_leaf(l));
            }
            e = acc;
            return compute_rest();
        }
    }
    for (const auto& kv : narrow) {
        const PendingK0& k = kv.second;
        const Column& cl = t->cols.at(k.col);
        HIP_CHECK(launch_masked_compare(cl.data, ktype(cl), cl.validity, mask, t->n_rows, k.cmp, k.c, k.bv, ctx->stream));
        mask = k.bv;
        t->last_narrowed++;
        t->last_narrow_cols.push_back(k.col);
    }
    Leaf ml;
    ml.bv = mask;
    e = mk_leaf(ml);
    return compute_rest();
}

bool fits(const ExprP& e) {
    Emitter em;
    em.emit_top(e);
    return em.ok && em.max_depth <= 4;
}

// Reduce an expression until it fits one kernel pass (<= kMaxLeaves leaves, depth <= 4):
// descend into a child that does not fit; when both children fit but not together,
// materialise the larger one into a scratch bitvector (one bits-only pass).
int fit(cubit_table* t, ExprP& e) {
    for (int guard = 0; guard < 256; ++guard) {
        if (fits(e)) return CUBIT_OK;
        ExprP* cur = &e;
        for (;;) {
            if ((*cur)->kind == Expr::LEAF) return fail(CUBIT_ERR_UNSUPPORTED, "cannot split program");
            ExprP& a = (*cur)->a;
            ExprP& b = (*cur)->b;
            if (!fits(a)) {
                cur = &a;
                continue;
            }
            if (!fits(b)) {
                cur = &b;
                continue;
            }
            ExprP* m = count_leaves(a) >= count_leaves(b) ? &a : &b;
            if ((*m)->kind == Expr::LEAF) m = (m == &a) ? &b : &a;
            uint64_t* bv = nullptr;
            if (int rc = materialize(t, *m, &bv)) return rc;
            Leaf l;
            l.bv = bv;
            *m = mk_leaf(l);
            break;
        }
    }
    return fail(CUBIT_ERR_UNSUPPORTED, "program too large");
}

// Copy-on-write patch of every leaf on an updated column: rows whose update is visible to
// the transaction get the bit their visible value implies (UpdatesForTransaction,
// update_info.hpp:44-55). Done on the device: copy the leaf, clear the updated rows, then
// set the rows whose visible value passes the leaf predicate.
__global__ void patch_leaf_kernel(const int64_t* __restrict__ rows, const int64_t* __restrict__ values,
                                  const uint8_t* __restrict__ valids, const uint64_t* __restrict__ versions, uint64_t n,
                                  uint64_t start_time, uint64_t tid, int pred, int cmp, int64_t c, int64_t c2,
                                  int type, uint64_t* __restrict__ bv) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t ver = versions[i];
        if (!(ver < start_time || ver == tid)) continue;
        const int64_t r = rows[i];
        // only the newest visible update of a row decides (records are chronological and
        // grouped by row by the host)
        bool newest = true;
        for (uint64_t j = i + 1; j < n && rows[j] == r; ++j) {
            const uint64_t vj = versions[j];
            if (vj < start_time || vj == tid) {
                newest = false;
                break;
            }
        }
        if (!newest) continue;
        const int64_t v = value_key(type, values[i]);  // the leaf's constants are keys (FLOAT / DOUBLE)
        // a SET NULL record: the row leaves the validity leaf and fails every comparison
        // (UpdateMergeValidity, update_segment.cpp:94-99; NULL never passes a filter)
        const bool ok = !valids || valids[i];
        bool p;
        if (pred == 1) p = ok;
        else if (!ok) p = false;
        else if (pred == 2) p = v >= c && v < c2;
        else if (cmp == 0) p = v == c;
        else if (cmp == 1) p = v != c;
        else if (cmp == 2) p = v < c;
        else if (cmp == 3) p = v <= c;
        else if (cmp == 4) p = v > c;
        else p = v >= c;
        unsigned long long* w = reinterpret_cast<unsigned long long*>(&bv[r >> 6]);
        const uint64_t bit = 1ull << (r & 63);
        if (p) atomicOr(w, bit);
        else atomicAnd(w, ~bit);
    }
}

int patch_updates(cubit_table* t, ExprP& e, const cubit_txn* txn, std::map<const uint64_t*, uint64_t*>& patched) {
    if (e->kind == Expr::LEAF) {
        auto uit = t->upd.find(e->leaf.column);
        if (uit == t->upd.end() || !uit->second.any_visible(txn)) return CUBIT_OK;
        auto pit = patched.find(e->leaf.bv);
        uint64_t* copy = nullptr;
        Updates& u = uit->second;
        const auto& dv = u.distinct_versions;
        const bool own = txn->transaction_id >= txn->start_time &&
                         std::binary_search(dv.begin(), dv.end(), txn->transaction_id);
        const int64_t prefix = std::lower_bound(dv.begin(), dv.end(), txn->start_time) - dv.begin();
        const Updates::PatchKey key{e->leaf.pred, e->leaf.cmp, e->leaf.constant, e->leaf.constant2};
        Updates::Patched* slot = own ? nullptr : &u.cache[key];
        if (pit != patched.end()) {
            copy = pit->second;
        } else if (slot && slot->bv && slot->prefix == prefix) {
            copy = static_cast<uint64_t*>(slot->bv->p);  // patched by an earlier scan of this snapshot set
            patched[e->leaf.bv] = copy;
        } else {
            if (slot) {
                if (!slot->bv) {
                    auto b = std::make_unique<DevBuf>();
                    if (hipMalloc(&b->p, t->nwp * 8) != hipSuccess)
                        return fail(CUBIT_ERR_OOM, "patched leaf allocation failed");
                    slot->bv = std::move(b);
                }
                copy = static_cast<uint64_t*>(slot->bv->p);
                slot->prefix = prefix;
            } else if (int rc = scratch_bv(t, &copy)) {
                return rc;
            }
            HIP_CHECK(hipMemcpyAsync(copy, e->leaf.bv, t->nwp * 8, hipMemcpyDeviceToDevice, t->ctx->stream));
            const unsigned grid = (unsigned)std::min<uint64_t>((u.n + 255) / 256, 4096);
            hipLaunchKernelGGL(patch_leaf_kernel, dim3(std::max(grid, 1u)), dim3(256), 0, t->ctx->stream,
                               static_cast<const int64_t*>(u.rows->p), static_cast<const int64_t*>(u.values->p),
                               u.d_valids(), static_cast<const uint64_t*>(u.versions->p), u.n, txn->start_time,
                               txn->transaction_id, e->leaf.pred, e->leaf.cmp, e->leaf.constant, e->leaf.constant2,
                               t->cols.at(e->leaf.column).type, copy);
            HIP_CHECK(hipGetLastError());
            patched[e->leaf.bv] = copy;
        }
        Leaf l = e->leaf;
        l.bv = copy;
        // the copy differs from the base only in zones holding an update record of the column
        if (!l.zbv) l.zbv = e->leaf.bv;
        l.zdirty = e->leaf.column;
        e = mk_leaf(l, e->neg);
        return CUBIT_OK;
    }
    if (e->kind == Expr::CONST_TRUE || e->kind == Expr::CONST_FALSE) return CUBIT_OK;
    if (int rc = patch_updates(t, e->a, txn, patched)) return rc;
    return patch_updates(t, e->b, txn, patched);
}

// ---- zonemaps: the reference skips a row group (RowGroup::CheckZonemap, row_group.cpp:361-371)
// or a run of vectors (CheckZonemapSegments, row_group.cpp:407-445) when a filter's
// CheckStatistics (constant_filter.cpp:11-32) proves it false on the segment's min/max. Here the
// statistics are the bitvectors themselves: per zone, "no row set" / "every row set". The
// expression's zone classes follow three-valued logic, and zones it proves empty are skipped.

using ZoneMap = cubit_table::ZoneMap;

// zones that hold at least one row of the partition
uint32_t real_zones(const cubit_table* t) { return (uint32_t)((t->n_rows + kZoneRows - 1) / kZoneRows); }

// the table-owned bitvectors (kZoneBits) and the columns (kZoneStats) an expression's leaves
// take their zone classes from
void collect_zone_sources(const ExprP& e, std::vector<const uint64_t*>& bvs, std::vector<int>& cols) {
    if (e->kind == Expr::LEAF) {
        const uint64_t* key = e->leaf.zbv ? e->leaf.zbv : e->leaf.bv;
        if (e->leaf.zsrc == kZoneBits && std::find(bvs.begin(), bvs.end(), key) == bvs.end()) bvs.push_back(key);
        if (e->leaf.zsrc == kZoneStats && std::find(cols.begin(), cols.end(), e->leaf.column) == cols.end())
            cols.push_back(e->leaf.column);
        return;
    }
    if (e->a) collect_zone_sources(e->a, bvs, cols);
    if (e->b) collect_zone_sources(e->b, bvs, cols);
}

// device scratch for zone summaries
uint8_t* zone_scratch(cubit_table* t, uint64_t bytes) {
    if (bytes > t->zone_dev_bytes) {
        t->zone_dev = std::make_unique<DevBuf>();
        t->zone_dev_bytes = 0;
        if (hipMalloc(&t->zone_dev->p, bytes) != hipSuccess) return nullptr;
        t->zone_dev_bytes = bytes;
    }
    return static_cast<uint8_t*>(t->zone_dev->p);
}

// Zone maps for the table-owned bitvectors `bvs` and zone statistics for the columns `cols`
// that have none yet: one classification launch per bitvector (zone_class_kernel reads it
// once), one statistics launch per column, one copy back.
int ensure_zones(cubit_table* t, const std::vector<const uint64_t*>& bvs, const std::vector<int>& cols) {
    std::vector<const uint64_t*> todo;
    for (const uint64_t* b : bvs)
        if (!t->zones.count(b)) todo.push_back(b);
    std::vector<int> todo_c;
    for (int c : cols)
        if (!t->col_zones.count(c)) todo_c.push_back(c);
    if (todo.empty() && todo_c.empty()) return CUBIT_OK;
    const uint32_t nz = real_zones(t);
    // min, max (int64) + flags per zone, each column's block 8-byte aligned
    const uint64_t per_col = ((uint64_t)nz * 17 + 7) / 8 * 8;
    // class bytes of the bitvectors, then their per-zone counts (4-byte aligned), then the
    // columns' statistics (8-byte aligned)
    const uint64_t cnt_base = ((uint64_t)todo.size() * nz + 3) / 4 * 4;
    const uint64_t cbase = (cnt_base + (uint64_t)todo.size() * nz * 4 + 7) / 8 * 8;
    const uint64_t bytes = cbase + (uint64_t)todo_c.size() * per_col + 16;
    uint8_t* dev = zone_scratch(t, bytes);
    if (!dev) return fail(CUBIT_ERR_OOM, "zone classes allocation failed");
    hipStream_t s = t->ctx->stream;
    for (size_t i = 0; i < todo.size(); ++i)
        HIP_CHECK(launch_zone_classes(todo[i], t->n_rows, 0, nz, dev + i * nz, s,
                                      reinterpret_cast<uint32_t*>(dev + cnt_base) + i * nz));
    for (size_t i = 0; i < todo_c.size(); ++i) {
        const Column& c = t->cols.at(todo_c[i]);
        uint8_t* p = dev + cbase + i * per_col;
        HIP_CHECK(launch_column_zone_stats(c.data, ktype(c), c.validity, t->n_rows, nz, reinterpret_cast<int64_t*>(p),
                                           reinterpret_cast<int64_t*>(p + 8ull * nz), p + 16ull * nz, s));
    }
    std::vector<uint8_t> host(cbase + todo_c.size() * per_col);
    HIP_CHECK(hipMemcpyAsync(host.data(), dev, host.size(), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    const size_t nw = (nz + 63) / 64;
    for (size_t i = 0; i < todo.size(); ++i) {
        ZoneMap m;
        m.z.assign(nw, 0);
        m.o.assign(nw, 0);
        for (uint32_t z = 0; z < nz; ++z) {
            const uint8_t c = host[i * nz + z];
            if (c & 1) m.z[z >> 6] |= 1ull << (z & 63);
            if (c & 2) m.o[z >> 6] |= 1ull << (z & 63);
            m.informative |= c != 0;
        }
        m.cnt.resize(nz);
        std::memcpy(m.cnt.data(), host.data() + cnt_base + 4ull * i * nz, 4ull * nz);
        t->zones.emplace(todo[i], std::move(m));
    }
    for (size_t i = 0; i < todo_c.size(); ++i) {
        const uint8_t* p = host.data() + cbase + i * per_col;
        cubit_table::ColZones cz;
        cz.mn.resize(nz);
        cz.mx.resize(nz);
        std::memcpy(cz.mn.data(), p, 8ull * nz);
        std::memcpy(cz.mx.data(), p + 8ull * nz, 8ull * nz);
        cz.fl.assign(p + 16ull * nz, p + 17ull * nz);
        t->col_zones.emplace(todo_c[i], std::move(cz));
    }
    return CUBIT_OK;
}

// Zone map of the leaf {valid rows with v cmp c} of column col from the column's zone statistics:
// ConstantFilter::CheckStatistics → NumericStats::CheckZonemap (constant_filter.cpp:11-32,
// numeric_stats.cpp:157-228) — FILTER_ALWAYS_FALSE = every valid value fails (or no row is
// valid), FILTER_ALWAYS_TRUE = every value passes and every row is valid.
const ZoneMap& stats_zone_map(cubit_table* t, const Leaf& l) {
    const auto key = std::make_tuple(l.column, l.pred, l.cmp, l.constant, l.constant2);
    auto it = t->pred_zones.find(key);
    if (it != t->pred_zones.end()) return it->second;
    const cubit_table::ColZones& cz = t->col_zones.at(l.column);
    const uint32_t nz = (uint32_t)cz.fl.size();
    ZoneMap m;
    m.z.assign((nz + 63) / 64, 0);
    m.o.assign((nz + 63) / 64, 0);
    const int64_t c = l.constant;
    for (uint32_t z = 0; z < nz; ++z) {
        const int64_t lo = cz.mn[z], hi = cz.mx[z];
        bool none, all;
        if (!(cz.fl[z] & 1)) {
            none = true;
            all = false;
        } else {
            switch (l.cmp) {
            case CUBIT_CMP_EQ: none = c < lo || c > hi; all = lo == c && hi == c; break;
            case CUBIT_CMP_NE: none = lo == c && hi == c; all = c < lo || c > hi; break;
            case CUBIT_CMP_LT: none = lo >= c; all = hi < c; break;
            case CUBIT_CMP_LE: none = lo > c; all = hi <= c; break;
            case CUBIT_CMP_GT: none = hi <= c; all = lo > c; break;
            default: none = hi < c; all = lo >= c; break;  // GE
            }
            all = all && (cz.fl[z] & 2);
        }
        if (none) m.z[z >> 6] |= 1ull << (z & 63);
        if (all) m.o[z >> 6] |= 1ull << (z & 63);
        m.informative |= none || all;
    }
    return t->pred_zones.emplace(key, std::move(m)).first->second;
}

// Estimated fraction of the partition's rows whose value of column col lies in [lo, hi) (valid
// rows only), from the column's per-zone min / max (values uniform between them in each zone):
// the planner's cost model for narrowing. Exactness never depends on it.
double interval_selectivity(cubit_table* t, int col, double lo_c, double hi_c, int* rc) {
    if (!t->cols.count(col) || t->n_rows == 0) return 1.0;
    if ((*rc = ensure_zones(t, {}, {col}))) return 1.0;
    const cubit_table::ColZones& cz = t->col_zones.at(col);
    const uint32_t nz = (uint32_t)cz.fl.size();
    // FLOAT / DOUBLE: zone bounds and the interval are keys; values are taken uniform in value
    // (not key) space, so every bound is mapped back to the value it names (NaN, the greatest
    // value, and ±inf as ±inf; a zone with an infinite span counts as an outlier below)
    const int type = t->cols.at(col).type;
    const bool fp = type_is_fp(type);
    auto value_of = [type](double k) -> double {
        if (std::isinf(k)) return k;
        const int64_t key = k >= 9.2e18 ? INT64_MAX : k <= -9.2e18 ? INT64_MIN + 1 : (int64_t)k;
        const int64_t bits = cubit_fp_value(type, key);
        double v;
        if (type == CUBIT_TYPE_FLOAT) {
            float f;
            const uint32_t u = (uint32_t)bits;
            std::memcpy(&f, &u, 4);
            v = f;
        } else {
            std::memcpy(&v, &bits, 8);
        }
        return std::isnan(v) ? std::numeric_limits<double>::infinity() : v;
    };
    if (fp) {
        lo_c = value_of(lo_c);
        hi_c = value_of(hi_c);
    }
    auto zone_bounds = [&](uint32_t z, double& lo, double& hi) {
        if (fp) {
            lo = value_of((double)cz.mn[z]);
            hi = value_of((double)cz.mx[z]);
            if (hi == lo) hi = std::nextafter(hi, std::numeric_limits<double>::infinity());
        } else {
            lo = (double)cz.mn[z];
            hi = (double)cz.mx[z] + 1.0;
        }
    };
    // a zone whose value span is far wider than the typical zone's holds a few outliers (one
    // extreme value stretches the uniform assumption over the whole type range): it counts at
    // the other zones' mean fraction instead
    std::vector<double> spans;
    for (uint32_t z = 0; z < nz; ++z) {
        if (!(cz.fl[z] & 1)) continue;
        double lo, hi;
        zone_bounds(z, lo, hi);
        if (std::isfinite(hi - lo)) spans.push_back(hi - lo);
    }
    double median_span = 0.0;
    if (!spans.empty()) {
        std::nth_element(spans.begin(), spans.begin() + spans.size() / 2, spans.end());
        median_span = spans[spans.size() / 2];
    }
    double kept = 0.0, normal_rows = 0.0, outlier_rows = 0.0;
    for (uint32_t z = 0; z < nz; ++z) {
        const double rows = (double)std::min<uint64_t>(kZoneRows, t->n_rows - (uint64_t)z * kZoneRows);
        if (!(cz.fl[z] & 1)) continue;  // no valid row passes a comparison
        double lo, hi;
        zone_bounds(z, lo, hi);
        const double span = hi - lo;
        if (!std::isfinite(span) || ((median_span > 1.0 || (fp && median_span > 0.0)) && span > 8.0 * median_span)) {
            outlier_rows += rows;
            continue;
        }
        const double f = std::max(0.0, std::min(hi, hi_c) - std::max(lo, lo_c)) / span;
        kept += f * rows;  // NULL rows of a mixed zone counted as valid: an over-estimate
        normal_rows += rows;
    }
    if (outlier_rows > 0.0) kept += outlier_rows * (normal_rows > 0.0 ? kept / normal_rows : 0.5);
    return std::min(1.0, kept / (double)t->n_rows);
}

// Estimated fraction of rows a conjunction of literals keeps: the literals of one column fold
// into one interval (a range index answers `a <= v < b` as L(b) AND NOT L(a): two literals of
// one predicate, not independent ones), the columns multiply (independence), literals that
// fold into no interval (NOT (v = c), NOT of a bin) multiply as 1 - their own fraction, and
// leaves not derived from a column value (visibility, materialised subtrees) keep every row.
double conj_selectivity(cubit_table* t, const Emitter::Lits& lits, int* rc) {
    const double inf = std::numeric_limits<double>::infinity();
    std::map<int, std::pair<double, double>> iv;
    double sel = 1.0;
    for (const auto& lit : lits) {
        const Leaf& l = lit.first;
        const bool neg = lit.second;
        if (l.column < 0 || l.pred == 1) continue;
        auto& r = iv.emplace(l.column, std::make_pair(-inf, inf)).first->second;
        const double c = (double)l.constant;
        double lo = -inf, hi = inf;  // the literal as [lo, hi), when it is one interval
        bool interval = true;
        if (l.pred == 2) {
            lo = c;
            hi = (double)l.constant2;
            interval = !neg;
        } else {
            switch (l.cmp) {
            case CUBIT_CMP_EQ: lo = c; hi = c + 1; interval = !neg; break;
            case CUBIT_CMP_NE: lo = c; hi = c + 1; interval = neg; break;  // NOT (v != c) = (v = c)
            case CUBIT_CMP_LT: (neg ? lo : hi) = c; break;
            case CUBIT_CMP_LE: (neg ? lo : hi) = c + 1; break;
            case CUBIT_CMP_GT: (neg ? hi : lo) = c + 1; break;
            default: (neg ? hi : lo) = c; break;  // GE
            }
        }
        if (interval) {
            r.first = std::max(r.first, lo);
            r.second = std::min(r.second, hi);
        } else {
            sel *= 1.0 - interval_selectivity(t, l.column, lo, hi, rc);
            if (*rc) return 1.0;
        }
    }
    for (const auto& kv : iv) {
        if (kv.second.first == -inf && kv.second.second == inf) continue;
        sel *= interval_selectivity(t, kv.first, kv.second.first, kv.second.second, rc);
        if (*rc) return 1.0;
    }
    return sel;
}

double literal_selectivity(cubit_table* t, const Leaf& l, bool neg, int* rc) {
    Emitter::Lits one{{l, neg}};
    return conj_selectivity(t, one, rc);
}

struct ZoneSet {
    std::vector<uint64_t> z, o;  // zones where the expression is false / true on every row
};

// zones holding an update record of column col (any version), a bit per zone
const std::vector<uint64_t>& dirty_zones(cubit_table* t, int col) {
    static const std::vector<uint64_t> none;
    auto it = t->upd.find(col);
    if (it == t->upd.end()) return none;
    Updates& u = it->second;
    const uint32_t nz = real_zones(t);
    if (u.dirty_nz != nz) {
        u.dirty.assign((nz + 63) / 64, 0);
        for (int64_t r : u.h_rows) {
            const uint64_t z = (uint64_t)r / kZoneRows;
            if (z < nz) u.dirty[z >> 6] |= 1ull << (z & 63);
        }
        u.dirty_nz = nz;
    }
    return u.dirty;
}

// three-valued evaluation of an expression over zone classes; leaves without zone classes are
// mixed everywhere
void zone_eval(cubit_table* t, const ExprP& e, size_t nw, ZoneSet& r) {
    switch (e->kind) {
    case Expr::LEAF: {
        const ZoneMap* m = nullptr;
        if (e->leaf.zsrc == kZoneBits) {
            auto it = t->zones.find(e->leaf.zbv ? e->leaf.zbv : e->leaf.bv);
            if (it != t->zones.end()) m = &it->second;
        } else if (e->leaf.zsrc == kZoneStats) {
            m = &stats_zone_map(t, e->leaf);
        }
        if (m) {
            r.z = m->z;
            r.o = m->o;
        } else {
            r.z.assign(nw, 0);
            r.o.assign(nw, 0);
        }
        if (m && e->leaf.zdirty >= 0) {  // patched: zones with an update record are mixed
            const std::vector<uint64_t>& d = dirty_zones(t, e->leaf.zdirty);
            for (size_t w = 0; w < nw && w < d.size(); ++w) {
                r.z[w] &= ~d[w];
                r.o[w] &= ~d[w];
            }
        }
        if (e->neg) std::swap(r.z, r.o);
        return;
    }
    case Expr::CONST_TRUE:
        r.z.assign(nw, 0);
        r.o.assign(nw, ~0ull);
        return;
    case Expr::CONST_FALSE:
        r.z.assign(nw, ~0ull);
        r.o.assign(nw, 0);
        return;
    default: break;
    }
    ZoneSet b;
    zone_eval(t, e->a, nw, r);
    zone_eval(t, e->b, nw, b);
    for (size_t w = 0; w < nw; ++w) {
        const uint64_t az = r.z[w], ao = r.o[w];
        switch (e->kind) {
        case Expr::AND: r.z[w] = az | b.z[w]; r.o[w] = ao & b.o[w]; break;
        case Expr::OR: r.z[w] = az & b.z[w]; r.o[w] = ao | b.o[w]; break;
        default: r.z[w] = az | b.o[w]; r.o[w] = ao & b.z[w]; break;  // ANDNOT
        }
    }
}

// does any leaf carry a zone class other than "mixed"?
bool zone_informative(cubit_table* t, const ExprP& e) {
    if (e->kind == Expr::LEAF) {
        if (e->leaf.zsrc == kZoneBits) {
            auto it = t->zones.find(e->leaf.zbv ? e->leaf.zbv : e->leaf.bv);
            return it != t->zones.end() && it->second.informative;
        }
        if (e->leaf.zsrc == kZoneStats) return stats_zone_map(t, e->leaf).informative;
        return false;
    }
    return (e->a && zone_informative(t, e->a)) || (e->b && zone_informative(t, e->b));
}

// The zonemap skip of a planned expression. live = the zones a kernel must evaluate, when at
// least one zone in 32 provably holds no qualifying row (below that the list and the cleared
// directory cost about what the skipped reads save); left empty otherwise = every zone.
// *none = no zone can hold a qualifying row.
int zone_plan(cubit_table* t, const ExprP& e, std::vector<uint32_t>& live, bool* none) {
    live.clear();
    *none = false;
    std::vector<const uint64_t*> bvs;
    std::vector<int> cols;
    collect_zone_sources(e, bvs, cols);
    if (bvs.empty() && cols.empty()) return CUBIT_OK;
    if (int rc = ensure_zones(t, bvs, cols)) return rc;
    if (!zone_informative(t, e)) return CUBIT_OK;  // every zone of every leaf mixed: nothing to skip
    const uint32_t nz = real_zones(t);
    ZoneSet r;
    zone_eval(t, e, (nz + 63) / 64, r);
    uint32_t dead = 0;
    for (uint32_t z = 0; z < nz; ++z) dead += (uint32_t)((r.z[z >> 6] >> (z & 63)) & 1);
    if (dead == nz) {
        *none = true;
        return CUBIT_OK;
    }
    if (dead == 0 || (uint64_t)dead * 32 < nz) return CUBIT_OK;
    live.reserve(nz - dead);
    for (uint32_t z = 0; z < nz; ++z)
        if (!((r.z[z >> 6] >> (z & 63)) & 1)) live.push_back(z);
    return CUBIT_OK;
}

// [lo, hi) of the values a comparison keeps (NE: the interval it removes); false for NE.
bool cmp_interval(int cmp, int64_t c, double* lo, double* hi) {
    const double inf = std::numeric_limits<double>::infinity(), x = (double)c;
    *lo = -inf;
    *hi = inf;
    switch (cmp) {
    case CUBIT_CMP_EQ: *lo = x; *hi = x + 1; return true;
    case CUBIT_CMP_NE: *lo = x; *hi = x + 1; return false;
    case CUBIT_CMP_LT: *hi = x; return true;
    case CUBIT_CMP_LE: *hi = x + 1; return true;
    case CUBIT_CMP_GT: *lo = x + 1; return true;
    default: *lo = x; return true;  // GE
    }
}

// Filter nodes with the constants on FLOAT / DOUBLE columns replaced by their comparison keys
// (cubit_fp_key): the planner, the zone statistics, the index keys and every kernel compare keys,
// so DuckDB's floating-point operators (NaN greatest and equal to NaN, -0.0 == +0.0) become integer
// comparisons. Nodes on other columns are used as given (no copy when there are none).
struct KeyedNodes {
    std::vector<cubit_filter_node> buf;
    const cubit_filter_node* p;
    int rc = CUBIT_OK;
    KeyedNodes(const cubit_table* t, const cubit_filter_node* nodes, uint32_t n) : p(nodes) {
        for (uint32_t k = 0; k < n; ++k) {
            if (nodes[k].kind != CUBIT_FILTER_CONSTANT) continue;
            auto it = t->cols.find(nodes[k].column);
            if (it == t->cols.end() || (!type_is_keyed(it->second.type) && it->second.type != CUBIT_TYPE_VARCHAR)) continue;
            if (buf.empty()) {
                buf.assign(nodes, nodes + n);
                p = buf.data();
            }
            if (it->second.type != CUBIT_TYPE_VARCHAR) {
                buf[k].constant = value_key(it->second.type, nodes[k].constant);
                continue;
            }
            // a string constant → a comparison of codes with the same rows: lb = the first code whose
            // string is >= s; s absent: = matches nothing (code -1), != every valid row, <= is < lb,
            // > is >= lb
            const cubit_string* str = reinterpret_cast<const cubit_string*>((intptr_t)nodes[k].constant);
            if (!str || (str->size && !str->data)) {
                rc = fail(CUBIT_ERR_INVALID, "filter node %u: a VARCHAR constant must be a cubit_string", k);
                return;
            }
            bool present = false;
            const int64_t lb =
                (int64_t)it->second.dict->lower_bound(std::string_view(str->data ? str->data : "", str->size), &present);
            int cmp = nodes[k].cmp;
            int64_t c = lb;
            if (!present) {
                if (cmp == CUBIT_CMP_EQ || cmp == CUBIT_CMP_NE) c = -1;
                else if (cmp == CUBIT_CMP_LE) cmp = CUBIT_CMP_LT;
                else if (cmp == CUBIT_CMP_GT) cmp = CUBIT_CMP_GE;
            }
            buf[k].cmp = cmp;
            buf[k].constant = c;
        }
    }
};

// Estimated fraction of the partition's rows a filter tree (prefix nodes from i; i ends past the
// subtree) keeps, on the planner's cost model (interval_selectivity: per-zone min / max, values
// uniform within a zone, columns independent). An AND folds its constant children on one column
// into one interval (a pushed TableFilterSet's `a <= v AND v < b`); an OR keeps 1 - Π(1 - s);
// IS NULL counts the zones that hold a NULL. MVCC deletes only lower the true fraction.
double tree_selectivity(cubit_table* t, const cubit_filter_node* nodes, uint32_t& i, int* rc) {
    const cubit_filter_node& f = nodes[i++];
    double lo, hi;
    switch (f.kind) {
    case CUBIT_FILTER_AND: {
        std::map<int, std::pair<double, double>> iv;
        double sel = 1.0;
        for (int k = 0; k < f.n_children && !*rc; ++k) {
            const cubit_filter_node& c = nodes[i];
            if (c.kind == CUBIT_FILTER_CONSTANT && c.cmp != CUBIT_CMP_NE) {
                cmp_interval(c.cmp, c.constant, &lo, &hi);
                const double inf = std::numeric_limits<double>::infinity();
                auto& r = iv.emplace(c.column, std::make_pair(-inf, inf)).first->second;
                r.first = std::max(r.first, lo);
                r.second = std::min(r.second, hi);
                ++i;
            } else {
                sel *= tree_selectivity(t, nodes, i, rc);
            }
        }
        for (const auto& kv : iv) {
            if (*rc) break;
            sel *= kv.second.second <= kv.second.first ? 0.0
                                                       : interval_selectivity(t, kv.first, kv.second.first, kv.second.second, rc);
        }
        return sel;
    }
    case CUBIT_FILTER_OR: {
        double none = 1.0;
        for (int k = 0; k < f.n_children && !*rc; ++k) none *= 1.0 - tree_selectivity(t, nodes, i, rc);
        return 1.0 - none;
    }
    case CUBIT_FILTER_CONSTANT: {
        const bool in = cmp_interval(f.cmp, f.constant, &lo, &hi);
        const double s = interval_selectivity(t, f.column, lo, hi, rc);
        return in ? s : 1.0 - s;
    }
    case CUBIT_FILTER_IS_NULL: {
        if (!t->cols.at(f.column).validity || t->n_rows == 0) return 0.0;
        if ((*rc = ensure_zones(t, {}, {f.column}))) return 1.0;
        const auto& fl = t->col_zones.at(f.column).fl;
        double rows = 0.0;
        for (uint32_t z = 0; z < (uint32_t)fl.size(); ++z)
            if (!(fl[z] & 2)) rows += (double)std::min<uint64_t>(kZoneRows, t->n_rows - (uint64_t)z * kZoneRows);
        return std::min(1.0, rows / (double)t->n_rows);
    }
    default:  // IS NOT NULL
        return 1.0;
    }
}

}  // namespace

extern "C" int cubit_table_estimate_rows(cubit_table* t, const cubit_filter_node* nodes, uint32_t n_nodes,
                                         uint64_t* rows) {
    if (!t || !rows || (n_nodes && !nodes)) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    *rows = t->n_rows;
    if (n_nodes == 0 || t->n_rows == 0) return CUBIT_OK;
    Planner shape{t, nodes, n_nodes};
    if (shape.subtree_end(0) != (int)n_nodes) return fail(CUBIT_ERR_INVALID, "malformed filter tree");
    for (uint32_t k = 0; k < n_nodes; ++k) {
        const cubit_filter_node& f = nodes[k];
        if (f.kind < CUBIT_FILTER_CONSTANT || f.kind > CUBIT_FILTER_AND)
            return fail(CUBIT_ERR_INVALID, "filter node kind %d", f.kind);
        if (f.kind != CUBIT_FILTER_OR && f.kind != CUBIT_FILTER_AND && !t->cols.count(f.column))
            return fail(CUBIT_ERR_INVALID, "filter references unregistered column %d", f.column);
        if (f.kind == CUBIT_FILTER_CONSTANT && (f.cmp < 0 || f.cmp > 5))
            return fail(CUBIT_ERR_INVALID, "comparison %d", f.cmp);
    }
    if (int rc = set_device(t->ctx)) return rc;
    int rc = CUBIT_OK;
    uint32_t i = 0;
    const KeyedNodes keyed(t, nodes, n_nodes);
    if (keyed.rc) return keyed.rc;
    const double s = std::min(1.0, std::max(0.0, tree_selectivity(t, keyed.p, i, &rc)));
    if (rc) return rc;
    *rows = std::min<uint64_t>(t->n_rows, (uint64_t)std::ceil(s * (double)t->n_rows));
    return CUBIT_OK;
}

namespace {

// Plan a pushed filter tree for a transaction into one program (front half of every scan):
// planner → MVCC update patches → visibility leaf → constant folding → split until it fits
// one pass → emit. *empty = the filter is FALSE (no kernel needed). live (optional) receives the
// zonemap skip's live zones (empty = evaluate every zone); a filter false on every zone is
// *empty too.
int plan_program(cubit_table* t, const cubit_filter_node* nodes, uint32_t n_nodes, const cubit_txn* txn,
                 Emitter& em, bool* empty, std::vector<uint32_t>* live = nullptr) {
    *empty = false;
    if (live) live->clear();
    cubit_ctx* ctx = t->ctx;
    t->single_leaf = nullptr;
    t->scratch_used = 0;
    t->last_passes = 0;
    t->last_packed = 0;
    t->last_narrowed = 0;
    t->last_narrow_cols.clear();
    ExprP e;
    std::vector<PendingK0> pending;  // K0 leaves not built yet (narrow_k0)
    if (n_nodes == 0) {
        e = mk_true();
    } else {
        const KeyedNodes keyed(t, nodes, n_nodes);
        if (keyed.rc) return keyed.rc;
        Planner p{t, keyed.p, n_nodes};
        if (p.subtree_end(0) != (int)n_nodes) return fail(CUBIT_ERR_INVALID, "malformed filter tree");
        e = p.plan(0);
        if (!e) return p.rc ? p.rc : fail(CUBIT_ERR_INVALID, "planning failed");
        pending = std::move(p.pending);
    }
    // a transaction that sees updates patches whole leaves: build the K0 leaves in full first
    bool visible_updates = false;
    if (txn)
        for (auto& kv : t->upd) visible_updates |= kv.second.any_visible(txn);
    if (visible_updates) {
        for (const PendingK0& k : pending) {
            if (int rc = compute_k0(t, k)) return rc;
            t->last_narrow_cols.push_back(k.col);
        }
        pending.clear();
    }
    if (txn) {
        std::map<const uint64_t*, uint64_t*> patched;
        // bound the patched-leaf caches between scans (never during one: a slot freed
        // mid-plan could be reallocated to another leaf of the same plan)
        for (auto& kv : t->upd)
            if (kv.second.cache.size() >= 16) kv.second.cache.clear();
        if (!t->upd.empty()) {
            if (int rc = patch_updates(t, e, txn, patched)) return rc;
        }
        // visibility leaf: insert ranges the reader may not see, then deletes in effect
        // (ChunkVectorInfo::TemplatedGetSelVector, chunk_info.cpp:123-161)
        const auto& ids = t->del_ids_sorted;
        const int64_t prefix = std::lower_bound(ids.begin(), ids.end(), txn->start_time) - ids.begin();
        const bool own_del = t->n_del && std::binary_search(ids.begin(), ids.end(), txn->transaction_id) &&
                             txn->transaction_id >= txn->start_time;
        const int64_t ins_prefix =
            std::lower_bound(t->ins.begin(), t->ins.end(), txn->start_time,
                             [](const cubit_table::InsRange& a, uint64_t v) { return a.id < v; }) -
            t->ins.begin();
        bool own_ins = false, any_hidden = false;
        for (int64_t i = ins_prefix; i < (int64_t)t->ins.size(); ++i) {
            own_ins |= t->ins[i].id == txn->transaction_id;
            any_hidden |= t->ins[i].id != txn->transaction_id;
        }
        if (prefix > 0 || own_del || any_hidden) {
            const bool own = own_del || own_ins;
            uint64_t* vis = nullptr;
            if (!own) {
                if (!t->vis_cache) {
                    auto b = std::make_unique<DevBuf>();
                    if (hipMalloc(&b->p, t->nwp * sizeof(uint64_t)) != hipSuccess)
                        return fail(CUBIT_ERR_OOM, "visibility bitvector allocation failed");
                    t->vis_cache = std::move(b);
                }
                vis = static_cast<uint64_t*>(t->vis_cache->p);
            } else if (int rc = scratch_bv(t, &vis)) {
                return rc;
            }
            if (own || prefix != t->vis_prefix || ins_prefix != t->vis_ins_prefix) {
                // hidden insert ranges: ids at or past start_time, except the reader's own
                t->hidden_host.clear();
                for (int64_t i = ins_prefix; i < (int64_t)t->ins.size(); ++i)
                    if (t->ins[i].id != txn->transaction_id) {
                        t->hidden_host.push_back(t->ins[i].begin);
                        t->hidden_host.push_back(t->ins[i].end);
                    }
                const uint32_t n_hidden = (uint32_t)(t->hidden_host.size() / 2);
                if (n_hidden) {
                    t->hidden_dev = std::make_unique<DevBuf>();
                    if (hipMalloc(&t->hidden_dev->p, t->hidden_host.size() * 8) != hipSuccess)
                        return fail(CUBIT_ERR_OOM, "insert range allocation failed");
                    HIP_CHECK(hipMemcpyAsync(t->hidden_dev->p, t->hidden_host.data(), t->hidden_host.size() * 8,
                                             hipMemcpyHostToDevice, ctx->stream));
                }
                HIP_CHECK(launch_visibility(t->n_del ? static_cast<const int64_t*>(t->del_rows->p) : nullptr,
                                            t->n_del ? static_cast<const uint64_t*>(t->del_ids->p) : nullptr,
                                            t->n_del, t->n_rows, txn->start_time, txn->transaction_id, vis,
                                            ctx->stream,
                                            n_hidden ? static_cast<const int64_t*>(t->hidden_dev->p) : nullptr,
                                            n_hidden));
                if (n_hidden) HIP_CHECK(hipStreamSynchronize(ctx->stream));  // hidden_host / hidden_dev reuse
                if (!own) {  // a reader with its own versions builds into scratch: the cache stays
                    t->vis_prefix = prefix;
                    t->vis_ins_prefix = ins_prefix;
                }
            }
            Leaf l;
            l.bv = vis;
            e = mk_bin(Expr::AND, e, mk_leaf(l));
        }
    }
    if (e->kind == Expr::CONST_FALSE) {
        *empty = true;
        t->last_leaves = 0;
        return CUBIT_OK;
    }
    if (e->kind == Expr::CONST_TRUE) {
        const uint64_t* ones = nullptr;
        if (int rc = ones_bv(t, &ones)) return rc;
        Leaf l;
        l.bv = ones;
        e = mk_leaf(l);
    }
    if (live) {
        bool none = false;
        if (int rc = zone_plan(t, e, *live, &none)) return rc;
        if (none) {
            *empty = true;
            t->last_leaves = 0;
            return CUBIT_OK;
        }
    }
    // the K0 leaves last: narrowed to the rows the rest of a conjunction keeps, or in full
    if (int rc = narrow_k0(t, e, pending, t->use_narrowing)) return rc;
    if (int rc = fit(t, e)) return rc;
    em.emit_top(e);
    if (!em.ok) return fail(CUBIT_ERR_UNSUPPORTED, "program does not fit one pass");
    t->last_leaves = em.prog.n_leaves;
    t->last_passes++;
    t->single_leaf = e->kind == Expr::LEAF && !e->neg && e->leaf.zsrc == kZoneBits && !e->leaf.zbv &&
                             e->leaf.zdirty < 0 && em.prog.n_leaves == 1 && em.prog.negate == 0
                         ? e->leaf.bv
                         : nullptr;
    return CUBIT_OK;
}

// The device prefix of the per-zone counts of a table-owned bitvector whose zone map is built
// (null when it is not): the offsets of a decode of that bitvector alone.
const uint64_t* tile_prefix_of(cubit_table* t, const uint64_t* bv, int* rc) {
    *rc = CUBIT_OK;
    auto it = t->zones.find(bv);
    if (it == t->zones.end() || it->second.cnt.empty()) return nullptr;
    ZoneMap& m = it->second;
    if (!m.prefix) {
        m.prefix_host.assign(m.cnt.size() + 1, 0);
        for (size_t z = 0; z < m.cnt.size(); ++z) m.prefix_host[z + 1] = m.prefix_host[z] + m.cnt[z];
        auto b = std::make_shared<DevBuf>();
        if (hipMalloc(&b->p, m.prefix_host.size() * sizeof(uint64_t)) != hipSuccess) {
            *rc = fail(CUBIT_ERR_OOM, "tile prefix allocation failed");
            return nullptr;
        }
        if (hipMemcpyAsync(b->p, m.prefix_host.data(), m.prefix_host.size() * sizeof(uint64_t), hipMemcpyHostToDevice,
                           t->ctx->stream) != hipSuccess) {
            *rc = fail(CUBIT_ERR_HIP, "tile prefix upload failed");
            return nullptr;
        }
        m.prefix = std::move(b);
    }
    return static_cast<const uint64_t*>(m.prefix->p);
}

// The values `col` can take among the rows the filter keeps, when its constant filters in the
// top-level AND pin it to a short list that the column's exact range index can decode:
// v0 < v1 < … with leaves L(v_j). Returns false when it cannot (the kernel then gathers b).
bool decodable_values(cubit_table* t, const cubit_filter_node* nodes, uint32_t n_nodes, int col,
                      std::vector<int64_t>& vals, std::vector<const uint64_t*>& leaves) {
    auto ixit = t->idx.find(col);
    if (ixit == t->idx.end() || n_nodes == 0) return false;
    const IndexView ix = view_of(t, col, ixit->second);
    if (ix.encoding != CUBIT_INDEX_RANGE || !ix.exact_all || ix.empty) return false;
    int64_t lo = ix.vmin, hi = ix.vmax;  // inclusive bounds
    bool bounded = false;
    // constants on col reachable through AND nodes only
    std::vector<uint32_t> stack{0};
    Planner pl{t, nodes, n_nodes};
    while (!stack.empty()) {
        const uint32_t i = stack.back();
        stack.pop_back();
        const cubit_filter_node& f = nodes[i];
        if (f.kind == CUBIT_FILTER_AND) {
            uint32_t j = i + 1;
            for (int k = 0; k < f.n_children; ++k) {
                stack.push_back(j);
                j = (uint32_t)pl.subtree_end(j);
            }
        } else if (f.kind == CUBIT_FILTER_CONSTANT && f.column == col) {
            const int64_t c = f.constant;
            switch (f.cmp) {
            case CUBIT_CMP_EQ: lo = std::max(lo, c); hi = std::min(hi, c); break;
            case CUBIT_CMP_LT: if (c == INT64_MIN) return false; hi = std::min(hi, c - 1); break;
            case CUBIT_CMP_LE: hi = std::min(hi, c); break;
            case CUBIT_CMP_GT: if (c == INT64_MAX) return false; lo = std::max(lo, c + 1); break;
            case CUBIT_CMP_GE: lo = std::max(lo, c); break;
            default: continue;
            }
            bounded = true;
        }
    }
    if (!bounded || lo > hi) return false;
    vals.clear();
    leaves.clear();
    if (ix.vmin >= lo && ix.vmin <= hi) vals.push_back(ix.vmin);
    for (size_t k = 0; k < ix.keys.size(); ++k) {
        if (ix.keys[k] < lo || ix.keys[k] > hi) continue;
        if (!vals.empty()) leaves.push_back(ix.bvs[k]);  // L(v_j) for j >= 1
        vals.push_back(ix.keys[k]);
        if (vals.size() > (size_t)kMaxDecode + 1) return false;
    }
    return !vals.empty();
}

}  // namespace

extern "C" int cubit_table_scan(cubit_table* t, const cubit_filter_node* nodes, uint32_t n_nodes,
                                const cubit_txn* txn, int64_t* d_rowids, uint64_t capacity, uint64_t* d_count,
                                uint32_t flags) {
    if (!t || !d_count) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    const bool count_only = (flags & CUBIT_SCAN_COUNT_ONLY) != 0;
    if (!count_only && !d_rowids) return fail(CUBIT_ERR_INVALID, "d_rowids is null without COUNT_ONLY");
    if (n_nodes && !nodes) return fail(CUBIT_ERR_INVALID, "nodes is null");
    if (int rc = set_device(t->ctx)) return rc;
    t->ctx->last_tiles = 0;  // until this scan's decode is launched (a planning error leaves none)
    if (t->n_rows == 0) {  // empty partition
        t->last_leaves = t->last_passes = 0;
        t->last_live = t->last_zones = 0;
        HIP_CHECK(hipMemsetAsync(d_count, 0, sizeof(uint64_t), t->ctx->stream));
        return CUBIT_OK;
    }
    Emitter em;
    bool empty = false;
    std::vector<uint32_t> live;
    const bool zonemap = (flags & CUBIT_SCAN_NO_ZONEMAP) == 0;
    t->last_zones = real_zones(t);
    t->last_live = 0;
    const uint64_t h0 = host_timing() ? now_ns() : 0;
    if (int rc = plan_program(t, nodes, n_nodes, txn, em, &empty, zonemap ? &live : nullptr)) return rc;
    const uint64_t h1 = host_timing() ? now_ns() : 0;
    if (empty) {  // the filter folded to FALSE (or the zonemaps rule out every zone): no launch, no tiles
        t->ctx->last_tiles = 0;
        HIP_CHECK(hipMemsetAsync(d_count, 0, sizeof(uint64_t), t->ctx->stream));
        return CUBIT_OK;
    }
    t->last_live = live.empty() ? t->last_zones : (uint32_t)live.size();
    const uint64_t* prefix = nullptr;
    if (!count_only && t->single_leaf) {
        int rc = CUBIT_OK;
        prefix = tile_prefix_of(t, t->single_leaf, &rc);
        if (rc) return rc;
    }
    const uint64_t h2 = host_timing() ? now_ns() : 0;
    const int rc = run_eval(t->ctx, em.prog, t->n_rows, t->row_base, count_only ? nullptr : d_rowids, capacity, d_count,
                            nullptr, count_only ? RunMode::kCount : RunMode::kDecode, true,
                            (flags & CUBIT_SCAN_ORDERED) != 0, (flags & CUBIT_SCAN_CHECK_CAPACITY) != 0,
                            live.empty() ? nullptr : &live, prefix);
    if (host_timing()) {
        const uint64_t h3 = now_ns();
        t->host_ns[0] += h1 - h0;
        t->host_ns[1] += h2 - h1;
        t->host_ns[2] += h3 - h2;
        t->host_scans++;
    }
    return rc;
}

// cubit_table_scan and its tile directory under one hold of the context lock: the directory is
// copied on the context's stream before any other thread's scan can reuse the context's buffer
// (cubit_ctx_last_tiles read after a separate cubit_table_scan may describe another thread's
// scan when several DuckDB pipeline tasks share the context).
extern "C" int cubit_table_scan_tiles(cubit_table* t, const cubit_filter_node* nodes, uint32_t n_nodes,
                                      const cubit_txn* txn, int64_t* d_rowids, uint64_t capacity, uint64_t* d_count,
                                      uint32_t flags, uint64_t* d_dir, uint32_t dir_cap, uint32_t* n_tiles,
                                      uint64_t* rows_per_tile) {
    if (!t || !n_tiles) return fail(CUBIT_ERR_INVALID, "null argument");
    if (flags & CUBIT_SCAN_COUNT_ONLY) return fail(CUBIT_ERR_INVALID, "a count-only scan has no tile directory");
    CUBIT_LOCK(t->ctx);
    if (int rc = cubit_table_scan(t, nodes, n_nodes, txn, d_rowids, capacity, d_count, flags)) return rc;
    cubit_ctx* ctx = t->ctx;
    *n_tiles = ctx->last_tiles;
    if (rows_per_tile) *rows_per_tile = ctx->last_tile_rows;
    if (ctx->last_tiles > dir_cap)
        return fail(CUBIT_ERR_CAPACITY, "tile directory of %u tiles, room for %u", ctx->last_tiles, dir_cap);
    if (ctx->last_tiles) {
        if (!d_dir) return fail(CUBIT_ERR_INVALID, "d_dir is null");
        HIP_CHECK(hipMemcpyAsync(d_dir, ctx->dir, 2ull * ctx->last_tiles * sizeof(uint64_t), hipMemcpyDeviceToDevice,
                                 ctx->stream));
    }
    return CUBIT_OK;
}

namespace {
int probe_impl(cubit_table* t, int col, const cubit_txn* txn, const int64_t* d_rowids, const uint64_t* d_count,
               uint64_t max_n, int64_t* d_out, uint64_t* d_valid);
}  // namespace

extern "C" int cubit_table_sum_product(cubit_table* t, const cubit_filter_node* nodes, uint32_t n_nodes,
                                       const cubit_txn* txn, int col_a, int col_b, int64_t* d_out,
                                       uint64_t* d_count, uint32_t flags) {
    if (!t || !d_out) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    if (n_nodes && !nodes) return fail(CUBIT_ERR_INVALID, "nodes is null");
    auto ait = t->cols.find(col_a), bit = t->cols.find(col_b);
    if (ait == t->cols.end() || bit == t->cols.end()) return fail(CUBIT_ERR_INVALID, "column not registered");
    if (ait->second.type != CUBIT_TYPE_INT64 || bit->second.type != CUBIT_TYPE_INT64)
        return fail(CUBIT_ERR_UNSUPPORTED, "sum_product needs INT64 (DECIMAL storage) columns");
    if (int rc = set_device(t->ctx)) return rc;
    cubit_ctx* ctx = t->ctx;
    ctx->last_tiles = 0;  // writes no row ids, so no tile directory (the fallback's scan resets it below)
    uint64_t* count = d_count ? d_count : t->dummy_count;
    if (t->n_rows == 0) {  // empty partition: sum 0 over 0 rows
        HIP_CHECK(hipMemsetAsync(d_out, 0, 2 * sizeof(int64_t), ctx->stream));
        HIP_CHECK(hipMemsetAsync(count, 0, sizeof(uint64_t), ctx->stream));
        return CUBIT_OK;
    }
    auto visible_updates = [&](int col) {
        auto u = t->upd.find(col);
        return txn && u != t->upd.end() && u->second.any_visible(txn);
    };
    if (visible_updates(col_a) || visible_updates(col_b)) {
        // MVCC fallback: row ids, then the probe (which applies the visible updates, NULL-ness
        // included), then a plain sum over the two value arrays. A nullable column probes with
        // its validity, which leaves 0 at NULL rows: those rows add nothing, as SUM skips NULLs.
        const bool nullable = ait->second.validity || bit->second.validity;
        const uint64_t cap = t->n_rows;
        const uint64_t vwords = nullable ? (cap + 63) / 64 : 0;
        if (int rc = ensure_tmp(ctx, 3 * cap + vwords)) return rc;
        int64_t* ids = ctx->tmp_ids + 0;
        int64_t* xa = ctx->tmp_ids + cap;
        int64_t* xb = ctx->tmp_ids + 2 * cap;
        uint64_t* vw = nullable ? reinterpret_cast<uint64_t*>(ctx->tmp_ids + 3 * cap) : nullptr;
        // the scan's own decode must not use tmp_ids (ordered flag off)
        if (int rc = cubit_table_scan(t, nodes, n_nodes, txn, ids, cap, count, 0)) return rc;
        if (int rc = probe_impl(t, col_a, txn, ids, count, cap, xa, vw)) return rc;
        if (int rc = probe_impl(t, col_b, txn, ids, count, cap, xb, vw)) return rc;
        HIP_CHECK(launch_sum_product_arrays(xa, xb, count, cap, ctx->partials, d_out, ctx->stream));
        ctx->last_tiles = 0;  // the directory described ids in scratch, not a caller's buffer
        return CUBIT_OK;
    }
    Emitter em;
    bool empty = false;
    std::vector<uint32_t> live;
    t->last_zones = real_zones(t);
    t->last_live = 0;
    if (int rc = plan_program(t, nodes, n_nodes, txn, em, &empty, (flags & CUBIT_SUM_NO_ZONEMAP) ? nullptr : &live))
        return rc;
    if (empty) {
        HIP_CHECK(hipMemsetAsync(d_out, 0, 2 * sizeof(int64_t), ctx->stream));
        HIP_CHECK(hipMemsetAsync(count, 0, sizeof(uint64_t), ctx->stream));
        return CUBIT_OK;
    }
    t->last_live = live.empty() ? t->last_zones : (uint32_t)live.size();
    SumArgs sa{};
    sa.a = static_cast<const int64_t*>(ait->second.data);
    sa.a_valid = ait->second.validity;
    t->last_sum_packed = false;
    if (!(flags & CUBIT_SUM_PLAIN_A) && ait->second.bp_n_groups) {
        sa.a_bytes = static_cast<const uint8_t*>(ait->second.bp_bytes->p);
        sa.a_groups = static_cast<const BpGroup*>(ait->second.bp_groups->p);
        sa.a_vgroup = static_cast<const uint32_t*>(ait->second.bp_vgroup->p);
        sa.a_plain = sa.a;
        sa.a_n_groups = ait->second.bp_n_groups;
        t->last_sum_packed = true;
    }
    sa.partials = ctx->partials;
    std::vector<int64_t> vals;
    std::vector<const uint64_t*> dl;
    if (!(flags & CUBIT_SUM_GATHER_B) && decodable_values(t, nodes, n_nodes, col_b, vals, dl)) {
        sa.b = nullptr;
        sa.v0 = vals[0];
        sa.n_decode = (uint32_t)dl.size();
        for (size_t j = 0; j < dl.size(); ++j) {
            sa.dleaf[j] = dl[j];
            sa.delta[j] = (int64_t)((uint64_t)vals[j + 1] - (uint64_t)vals[j]);  // modular: no signed overflow
        }
        t->last_decoded = (uint32_t)dl.size() + 1;
    } else {
        sa.b = static_cast<const int64_t*>(bit->second.data);
        sa.b_valid = bit->second.validity;
        t->last_decoded = 0;
    }
    EvalArgs a{};
    a.prog = em.prog;
    a.n_rows = t->n_rows;
    a.n_words = (t->n_rows + 63) / 64;
    a.row_base = t->row_base;
    a.count = count;
    a.ticket = ctx->ticket;
    a.num_tiles = (uint32_t)(padded_words(t->n_rows) / decode_tile_words());
    if (!live.empty()) {  // zonemap skip: a zone is one tile of the fused kernel
        uint32_t n_live = 0;
        if (int rc = upload_live(ctx, live, 1, &a.live, &n_live)) return rc;
        a.num_tiles = n_live;
    }
    const unsigned grid = std::min<unsigned>(a.num_tiles, sum_product_grid((unsigned)ctx->n_cus));
    HIP_CHECK(launch_eval_sum_product(a, sa, std::max(grid, 1u), d_out, ctx->stream));
    return CUBIT_OK;
}

extern "C" int cubit_table_last_plan(cubit_table* t, uint32_t* n_leaves, uint32_t* n_passes) {
    if (!t) return fail(CUBIT_ERR_INVALID, "null table");
    CUBIT_LOCK(t->ctx);
    if (n_leaves) *n_leaves = t->last_leaves;
    if (n_passes) *n_passes = t->last_passes;
    return CUBIT_OK;
}

// Column statistics (DataTable::GetStatistics, behind seq_scan's `statistics` callback
// TableScanStatistics, table_scan.cpp:108-117): min / max of the valid values and whether the
// column has NULL / non-NULL rows, from the per-zone statistics the zonemaps use (computed once,
// cached until the column changes). As DuckDB's column statistics absorb every update
// (UpdateSegment merges its values into the segment statistics), the bounds widen by the
// column's update records of any version, and an updated row counts as a non-NULL one.
extern "C" int cubit_table_column_statistics(cubit_table* t, int col, int64_t* vmin, int64_t* vmax,
                                             int* has_null, int* has_no_null) {
    if (!t) return fail(CUBIT_ERR_INVALID, "null table");
    CUBIT_LOCK(t->ctx);
    if (!t->cols.count(col)) return fail(CUBIT_ERR_INVALID, "column %d not registered", col);
    if (int rc = set_device(t->ctx)) return rc;
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    bool any_null = false, any_valid = false;
    if (t->n_rows) {
        if (int rc = ensure_zones(t, {}, {col})) return rc;
        const cubit_table::ColZones& cz = t->col_zones.at(col);
        for (size_t z = 0; z < cz.fl.size(); ++z) {
            if (cz.fl[z] & 1) {
                any_valid = true;
                lo = std::min(lo, cz.mn[z]);
                hi = std::max(hi, cz.mx[z]);
            }
            if (!(cz.fl[z] & 2)) any_null = true;
        }
    }
    auto uit = t->upd.find(col);
    if (uit != t->upd.end() && !uit->second.stat_values.empty()) {
        any_valid = true;
        lo = std::min(lo, uit->second.stat_values.front());
        hi = std::max(hi, uit->second.stat_values.back());
    }
    // a SET NULL record makes the column nullable (UpdateValidityStatistics,
    // update_segment.cpp:907-918: an update vector with an invalid row sets has_null)
    if (uit != t->upd.end() && uit->second.any_null) any_null = true;
    // FLOAT / DOUBLE: the bounds are keys; handed out as the bit patterns of those values
    const int type = t->cols.at(col).type;
    if (vmin) *vmin = any_valid ? cubit_fp_value(type, lo) : 0;
    if (vmax) *vmax = any_valid ? cubit_fp_value(type, hi) : 0;
    if (has_null) *has_null = any_null ? 1 : 0;
    if (has_no_null) *has_no_null = any_valid ? 1 : 0;
    return CUBIT_OK;
}

extern "C" int cubit_table_use_packed_filter(cubit_table* t, int on) {
    if (!t) return fail(CUBIT_ERR_INVALID, "null table");
    CUBIT_LOCK(t->ctx);
    t->use_packed = on != 0;
    return CUBIT_OK;
}

extern "C" int cubit_table_use_narrowing(cubit_table* t, int on) {
    if (!t) return fail(CUBIT_ERR_INVALID, "null table");
    CUBIT_LOCK(t->ctx);
    t->use_narrowing = on != 0;
    return CUBIT_OK;
}

extern "C" int cubit_table_column_changed(cubit_table* t, int col) {
    if (!t) return fail(CUBIT_ERR_INVALID, "null table");
    CUBIT_LOCK(t->ctx);
    if (!t->cols.count(col)) return fail(CUBIT_ERR_INVALID, "column %d is not registered", col);
    // statistics and zone classes derived from the values, and leaves patched from them
    drop_patches(t, col);
    return CUBIT_OK;
}

extern "C" int cubit_table_last_k0_order(cubit_table* t, int32_t* cols, uint32_t cap, uint32_t* n) {
    if (!t || !n || (cap && !cols)) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    *n = (uint32_t)t->last_narrow_cols.size();
    for (uint32_t i = 0; i < *n && i < cap; ++i) cols[i] = t->last_narrow_cols[i];
    return CUBIT_OK;
}

extern "C" int cubit_table_last_narrowed(cubit_table* t, uint32_t* n_leaves) {
    if (!t || !n_leaves) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    *n_leaves = t->last_narrowed;
    return CUBIT_OK;
}

extern "C" int cubit_table_last_packed(cubit_table* t, uint32_t* n_leaves) {
    if (!t || !n_leaves) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    *n_leaves = t->last_packed;
    return CUBIT_OK;
}

extern "C" int cubit_table_last_zones(cubit_table* t, uint32_t* evaluated, uint32_t* zones) {
    if (!t) return fail(CUBIT_ERR_INVALID, "null table");
    CUBIT_LOCK(t->ctx);
    if (evaluated) *evaluated = t->last_live;
    if (zones) *zones = t->last_zones;
    return CUBIT_OK;
}

extern "C" int cubit_table_last_sum_packed(cubit_table* t, int* packed) {
    if (!t || !packed) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    *packed = t->last_sum_packed ? 1 : 0;
    return CUBIT_OK;
}

extern "C" int cubit_table_last_sum_decode(cubit_table* t, uint32_t* n_values) {
    if (!t || !n_values) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    *n_values = t->last_decoded;
    return CUBIT_OK;
}

namespace {

// visible value of updated rows for a probe: patch gathered values in place — and their
// NULL-ness when out_valid is given (FetchRowValidity, update_segment.cpp:357-370: the newest
// visible record of the validity chain sets the row's bit)
__global__ void patch_probe_kernel(const int64_t* __restrict__ rowids, const uint64_t* __restrict__ d_count,
                                   uint64_t max_n, int64_t row_base, const int64_t* __restrict__ urows,
                                   const int64_t* __restrict__ uvalues, const uint8_t* __restrict__ uvalids,
                                   const uint64_t* __restrict__ uversions, uint64_t nu, uint64_t start_time,
                                   uint64_t tid, int64_t* __restrict__ out, uint64_t* __restrict__ out_valid) {
    const uint64_t n = min(*d_count, max_n);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t r = rowids[i] - row_base;
        // binary search the first record of row r (records grouped by row, ascending)
        uint64_t lo = 0, hi = nu;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) / 2;
            if (urows[mid] < r) lo = mid + 1;
            else hi = mid;
        }
        int vis = -1;  // newest visible record of the row
        for (uint64_t j = lo; j < nu && urows[j] == r; ++j) {
            const uint64_t v = uversions[j];
            if (v < start_time || v == tid) vis = (int)(j - lo);
        }
        if (vis < 0) continue;
        const uint64_t j = lo + (uint64_t)vis;
        const bool ok = !uvalids || uvalids[j];
        out[i] = ok ? uvalues[j] : 0;
        if (out_valid) {
            unsigned long long* w = reinterpret_cast<unsigned long long*>(&out_valid[i >> 6]);
            if (ok) atomicOr(w, 1ull << (i & 63));
            else atomicAnd(w, ~(1ull << (i & 63)));
        }
    }
}

}  // namespace

namespace {

// K3 for cubit_table_probe (d_valid null: values only, a NULL row's slot as stored) and
// cubit_table_probe_validity (values, 0 at NULL rows, and the validity words), then the visible
// update records on top
int probe_impl(cubit_table* t, int col, const cubit_txn* txn, const int64_t* d_rowids, const uint64_t* d_count,
               uint64_t max_n, int64_t* d_out, uint64_t* d_valid) {
    auto it = t->cols.find(col);
    if (it == t->cols.end()) return fail(CUBIT_ERR_INVALID, "column %d not registered", col);
    if (int rc = set_device(t->ctx)) return rc;
    const Column& c = it->second;
    if (d_valid)
        HIP_CHECK(launch_gather_valid(raw_of(c), c.type, c.validity, d_rowids, d_count, max_n, t->row_base, d_out, d_valid,
                                      t->ctx->stream));
    else
        HIP_CHECK(launch_gather(raw_of(c), c.type, d_rowids, d_count, max_n, t->row_base, d_out, t->ctx->stream));
    auto uit = t->upd.find(col);
    if (txn && uit != t->upd.end() && uit->second.any_visible(txn)) {
        const Updates& u = uit->second;
        const unsigned grid = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((max_n + 255) / 256, 4096));
        hipLaunchKernelGGL(patch_probe_kernel, dim3(grid), dim3(256), 0, t->ctx->stream, d_rowids, d_count, max_n,
                           t->row_base, static_cast<const int64_t*>(u.rows->p),
                           static_cast<const int64_t*>(u.values->p), u.d_valids(),
                           static_cast<const uint64_t*>(u.versions->p), u.n, txn->start_time, txn->transaction_id,
                           d_out, d_valid);
        HIP_CHECK(hipGetLastError());
    }
    return CUBIT_OK;
}

}  // namespace

extern "C" int cubit_table_probe(cubit_table* t, int col, const cubit_txn* txn, const int64_t* d_rowids,
                                 const uint64_t* d_count, uint64_t max_n, int64_t* d_out) {
    if (!t || !d_rowids || !d_count || !d_out) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    return probe_impl(t, col, txn, d_rowids, d_count, max_n, d_out, nullptr);
}

extern "C" int cubit_table_probe_validity(cubit_table* t, int col, const cubit_txn* txn, const int64_t* d_rowids,
                                          const uint64_t* d_count, uint64_t max_n, int64_t* d_out,
                                          uint64_t* d_validity) {
    if (!t || !d_rowids || !d_count || !d_out || !d_validity) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    return probe_impl(t, col, txn, d_rowids, d_count, max_n, d_out, d_validity);
}

extern "C" int cubit_table_info(cubit_table* t, uint64_t* n_rows, int64_t* row_base, cubit_ctx** ctx) {
    if (!t) return fail(CUBIT_ERR_INVALID, "null table");
    if (n_rows) *n_rows = t->n_rows;
    if (row_base) *row_base = t->row_base;
    if (ctx) *ctx = t->ctx;
    return CUBIT_OK;
}

extern "C" int cubit_table_column_data(cubit_table* t, int col, const void** data, int* type) {
    if (!t || !data) return fail(CUBIT_ERR_INVALID, "null argument");
    CUBIT_LOCK(t->ctx);
    auto it = t->cols.find(col);
    if (it == t->cols.end()) return fail(CUBIT_ERR_INVALID, "column %d not registered", col);
    *data = raw_of(it->second);  // FLOAT / DOUBLE: the patterns (the keys are internal)
    if (type) *type = it->second.type;
    return CUBIT_OK;
}
