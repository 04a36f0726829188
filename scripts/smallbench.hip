// Small-partition decode microbenchmark (development tool, not shipped): steady-state time per
// launch of the evaluate + decode kernels when launches run back to back on one stream, as in
// bench.py's timed loop — at the partition sizes strong scaling produces (SF100 over 8 / 4 / 2
// GPUs, SURVEY config 2) — against floors of the same launch shape.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-atomic-optimizer-strategy=None \
//         -I duckdb-cubit_amd/csrc scripts/smallbench.hip -o scripts/smallbench
// usage: smallbench [reps]   (prints one table per size; every kernel's row ids checked against
//                             the pair kernel's through the tile directories)
#include "cubit_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

using namespace cubit;

#define CK(x)                                                                                        \
    do {                                                                                             \
        hipError_t e_ = (x);                                                                         \
        if (e_ != hipSuccess) {                                                                      \
            fprintf(stderr, "%s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                                 \
        }                                                                                            \
    } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void fill_leaf(uint64_t* w, uint64_t pw, uint64_t n_rows, uint32_t thresh, uint64_t seed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < pw; i += stride) {
        uint64_t word = 0;
        for (int b = 0; b < 64; ++b) {
            const uint64_t row = i * 64 + b;
            const uint32_t h = (uint32_t)(mix64(seed * 0x9E3779B97F4A7C15ull + row) >> 32);
            if (row < n_rows && h < thresh) word |= 1ull << b;
        }
        w[i] = word;
    }
}

__global__ void empty_kernel(int* p) {
    if (p && threadIdx.x == 9999) *p = 0;
}

// one tile per workgroup: the K leaves read (same loads as the decode), and optionally WR
// int64 written per tile as one contiguous 16-byte-per-lane run
template <int K, int WR>
__global__ __launch_bounds__(512, 6) void floor_kernel(EvalArgs a, int64_t* out) {
    constexpr int THREADS = 512, PAIRS = 2;
    constexpr uint64_t TILE_WORDS = THREADS * 2 * PAIRS;
    const int t = threadIdx.x;
    const uint32_t tile = blockIdx.x;
    u64x2 v[K][PAIRS];
    load_tile<K, PAIRS, THREADS>(a, (uint64_t)tile * TILE_WORDS, t, v);
    uint64_t x = 0;
#pragma unroll
    for (int k = 0; k < K; ++k)
#pragma unroll
        for (int p = 0; p < PAIRS; ++p) x ^= v[k][p].x ^ v[k][p].y;
    if (WR == 0) {
        if (x == 0x12345) out[t] = (int64_t)x;
        return;
    }
    typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
    i64x2* o = reinterpret_cast<i64x2*>(out + (uint64_t)tile * WR);
    for (int i = t; i < WR / 2; i += THREADS) {
        i64x2 val;
        val.x = (int64_t)(x + 2 * i);
        val.y = (int64_t)(x + 2 * i + 1);
        o[i] = val;
    }
}

// the look-back kernel as it stood before its wave sum moved to DPP, for comparison (a copy of
// the kernel text, diagnostic only)
constexpr int kFlagCntBitsR03 = 20;
template <int K, int FORM, int STAGE, int WPC, int SAUX = 16>
__global__ __launch_bounds__(512, WPC * 2) void eval_decode_lookback_r03(EvalArgs a, uint64_t* __restrict__ dir) {
    constexpr int THREADS = 512, PAIRS = 2, NW = 2 * PAIRS, NWAVES = THREADS / 64;
    constexpr uint64_t TILE_WORDS = (uint64_t)THREADS * NW;
    constexpr uint64_t kCntMask = (1ull << kFlagCntBitsR03) - 1;
    __shared__ uint32_t s_wave_tot[NWAVES];
    __shared__ uint64_t s_pre[NWAVES];
    __shared__ uint32_t s_bad;
    __shared__ uint32_t s_stage[STAGE];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t b = blockIdx.x;
    const uint32_t tile = tile_at(a, b);
    const uint64_t tile_word0 = (uint64_t)tile * TILE_WORDS;
    const bool write_ids = a.rowids != nullptr;
    if (t == 0) s_bad = 0;
    u64x2 v[K][PAIRS];
    load_tile<K, PAIRS, THREADS>(a, tile_word0, t, v);
    uint64_t r[NW];
    eval_words<K, NW, FORM>(a.prog, v, r);
    tail_mask<NW, THREADS>(a, tile_word0, t, r);
    if (a.result_words) store_words<PAIRS, THREADS>(a.result_words, tile_word0, t, r);
    uint32_t packed = 0;
#pragma unroll
    for (int p = 0; p < PAIRS; ++p)
        packed |= (uint32_t)(__popcll(r[2 * p]) + __popcll(r[2 * p + 1])) << (16 * p);
    const uint32_t incl = wave_incl_scan32(packed);
    if (lane == 63) s_wave_tot[wave] = incl;
    __syncthreads();
    uint32_t wave_pre[2] = {0, 0}, block_tot[2] = {0, 0};
#pragma unroll
    for (int w = 0; w < NWAVES; ++w) {
        const uint32_t x = s_wave_tot[w];
        const uint32_t lo = x & 0xffffu, hi = x >> 16;
        if (w < wave) {
            wave_pre[0] += lo;
            wave_pre[1] += hi;
        }
        block_tot[0] += lo;
        block_tot[1] += hi;
    }
    const uint32_t excl = incl - packed;
    uint32_t pair_off[PAIRS];
    uint32_t tile_count = 0;
#pragma unroll
    for (int p = 0; p < PAIRS; ++p) {
        pair_off[p] = tile_count + wave_pre[p] + ((excl >> (16 * p)) & 0xffffu);
        tile_count += block_tot[p];
    }
    if (t == 0)
        __hip_atomic_store(a.flags + b, (a.epoch << kFlagCntBitsR03) | (uint64_t)tile_count, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    const bool staged = tile_count <= (uint32_t)STAGE;
    if (staged && write_ids && tile_count) {
#pragma unroll
        for (int p = 0; p < PAIRS; ++p) {
            uint32_t off = pair_off[p];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                uint64_t w = r[2 * p + e];
                const uint32_t wrow = (uint32_t)((p * 2 * THREADS + 2 * t + e) * 64);
                while (w) {
                    s_stage[off++] = wrow + (uint32_t)__builtin_ctzll(w);
                    w &= w - 1;
                }
            }
        }
    }
    // look-back over every earlier workgroup's flag
    uint64_t pre = 0;
    for (uint32_t j = t; j < b; j += THREADS) {
        uint64_t f = __hip_atomic_load(a.flags + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t spins = 0;
        while ((f >> kFlagCntBitsR03) != a.epoch) {
            if (++spins == kLookbackSpins) {
                s_bad = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(2);
            f = __hip_atomic_load(a.flags + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        pre += f & kCntMask;
    }
    pre = wave_sum(pre);
    if (lane == 0) s_pre[wave] = pre;
    __syncthreads();  // also: the stage is complete
    uint64_t base = 0;
#pragma unroll
    for (int w = 0; w < NWAVES; ++w) base += s_pre[w];
    if (s_bad) {
        if (t == 0) *a.count = ~0ull;
        return;
    }
    const int64_t row0 = a.row_base + (int64_t)(tile_word0 * 64);
    if (t == 0) {
        if (dir) {
            dir[2 * tile] = tile_count ? base : 0;
            dir[2 * tile + 1] = tile_count;
        }
        if (b == gridDim.x - 1) *a.count = base + tile_count;
    }
    if (!write_ids || !tile_count) return;
    if (staged) {
        emit_ids<THREADS, SAUX>(a.rowids, a.capacity, s_stage, tile_count, base, row0, t);
        return;
    }
    // dense tile: rounds of STAGE ids through the stage
    for (uint32_t r0 = 0; r0 < tile_count; r0 += (uint32_t)STAGE) {
        const uint32_t r1 = min(tile_count, r0 + (uint32_t)STAGE);
        if (r0) __syncthreads();  // the previous round's copy-out is done
#pragma unroll
        for (int p = 0; p < PAIRS; ++p) {
            uint32_t off = pair_off[p];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                uint64_t w = r[2 * p + e];
                const uint32_t c = (uint32_t)__popcll(w);
                const uint32_t wrow = (uint32_t)((p * 2 * THREADS + 2 * t + e) * 64);
                if (off < r1 && off + c > r0) {
                    uint32_t k = off;
                    for (; k < r0; ++k) w &= w - 1;  // the word straddles the round's start
                    for (; w && k < r1; ++k) {
                        s_stage[k - r0] = wrow + (uint32_t)__builtin_ctzll(w);
                        w &= w - 1;
                    }
                }
                off += c;
            }
        }
        __syncthreads();
        emit_ids<THREADS, SAUX>(a.rowids, a.capacity, s_stage, r1 - r0, base + r0, row0, t);
    }
}


// look-back variants: the kernel's diagnostic switches (DBG: 1 no spin, 2 no ids, 4 no sleep,
// 8 no flag loads, 16 no LDS decode, 64 the staging loop without its LDS stores)
template <int K, int SAUX, int DBG>
void lookback_variant(EvalArgs& a, uint64_t* dir, hipStream_t st) {
    hipLaunchKernelGGL((eval_decode_lookback<K, FORM_CONJ, kLookbackStage, lookback_wpc(K), SAUX, DBG>), dim3(a.num_tiles),
                       dim3(512), 0, st, a, dir);
}

struct Variant {
    std::string name;
    std::function<void(EvalArgs&, hipStream_t)> launch;
    bool check;
    uint32_t tmul = 1;  // directory entries per 131,072-row tile (2: 65,536-row tiles)
};

// the look-back decode over 65,536-row tiles: 256-thread workgroups, twice the grid, a 4,096-id
// stage, up to 6 workgroups per CU
template <int K>
void lookback_t256(EvalArgs& a, uint64_t* dir, hipStream_t st) {
    a.num_tiles = (uint32_t)((a.n_words + 1023) / 1024);
    hipLaunchKernelGGL((eval_decode_lookback<K, FORM_CONJ, 4096, 6, 16, 0, 256>), dim3(a.num_tiles), dim3(256), 0, st,
                       a, dir);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 50;
    int dev = 0, cus = 256;
    CK(hipSetDevice(dev));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, dev));
    cus = prop.multiProcessorCount;
    struct Case {
        const char* name;
        uint64_t n;
        int k;
        double dens;  // per-leaf density
    };
    const Case cases[] = {
        {"SF100/8 Q6-like K4", 75004738, 4, 0.372},
        {"cfg2 1e8 K1 1%", 100000000, 1, 0.01},
        {"SF100/4 Q6-like K4", 150009476, 4, 0.372},
        {"SF100/2 Q6-like K4", 300018951, 4, 0.372},
        {"SF100 Q6-like K4", 600037902, 4, 0.372},
    };
    uint64_t* flags;
    CK(hipMalloc(&flags, kLookbackMaxTiles * 8));
    CK(hipMemset(flags, 0, kLookbackMaxTiles * 8));
    uint64_t* flags_r03;
    CK(hipMalloc(&flags_r03, kLookbackMaxTiles * 8));
    CK(hipMemset(flags_r03, 0, kLookbackMaxTiles * 8));
    uint64_t* ticket;
    CK(hipMalloc(&ticket, kTicketWords * 8));
    CK(hipMemset(ticket, 0, kTicketWords * 8));
    uint64_t epoch = 0;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (const Case& c : cases) {
        const uint64_t n = c.n, W = (n + 63) / 64, pw = padded_words(n);
        const uint32_t tiles = (uint32_t)((W + 2047) / 2048);
        std::vector<uint64_t*> leaf(c.k);
        for (int k = 0; k < c.k; ++k) {
            CK(hipMalloc(&leaf[k], pw * 8));
            hipLaunchKernelGGL(fill_leaf, dim3(4096), dim3(256), 0, s, leaf[k], pw, n, (uint32_t)(c.dens * 4294967296.0),
                               (uint64_t)(k + 1));
        }
        const uint64_t cap = n / 8 + 4096;
        int64_t *ids, *ids_ref, *fl_out;
        uint64_t *cnt, *dir, *dir_ref;
        CK(hipMalloc(&ids, cap * 8));
        CK(hipMalloc(&ids_ref, cap * 8));
        CK(hipMalloc(&fl_out, cap * 8));
        int64_t* ids_ord;
        uint64_t* dst_off;
        CK(hipMalloc(&ids_ord, cap * 8));
        CK(hipMalloc(&dst_off, (uint64_t)tiles * 8 + 64));
        CK(hipMalloc(&cnt, 16));
        CK(hipMalloc(&dir, 4 * (uint64_t)tiles * 8 + 64));
        CK(hipMalloc(&dir_ref, 2 * (uint64_t)tiles * 8 + 64));
        uint64_t* d_prefix = nullptr;
        EvalArgs base{};
        for (int k = 0; k < c.k; ++k) base.prog.leaf[k] = leaf[k];
        base.prog.n_leaves = c.k;
        base.prog.form = FORM_CONJ;
        base.n_rows = n;
        base.n_words = W;
        base.row_base = 0;
        base.rowids = ids;
        base.capacity = cap;
        base.count = cnt;
        base.num_tiles = tiles;
        base.ticket = ticket;
        base.flags = flags;
        const uint64_t max_grid = 2ull * cus;
        const unsigned grid = (unsigned)(tiles <= max_grid ? tiles : tiles <= 2 * max_grid ? (tiles + 1) / 2 : max_grid);
        std::vector<Variant> vs;
        vs.push_back({"pairs (old policy, grid " + std::to_string(grid) + ")", [&](EvalArgs& a, hipStream_t st) {
                          CK(launch_eval_decode(a, dir, grid, st, nullptr, nullptr, 1, cus));
                      }, true});
        vs.push_back({"runs", [&](EvalArgs& a, hipStream_t st) {
                          CK(launch_eval_decode(a, dir, grid, st, nullptr, nullptr, 2, cus));
                      }, true});
        vs.push_back({"runs + order pass (one ascending array)", [&](EvalArgs& a, hipStream_t st) {
                          CK(launch_eval_decode(a, dir, grid, st, nullptr, nullptr, 2, cus));
                          CK(launch_order_runs(dir, tiles, dst_off, a.rowids, a.capacity, ids_ord, st));
                      }, false});
        if (tiles <= kLookbackMaxTiles)
            vs.push_back({"lookback (grid " + std::to_string(tiles) + ")", [&](EvalArgs& a, hipStream_t st) {
                              a.epoch = ++epoch;
                              CK(launch_eval_decode(a, dir, grid, st, nullptr, nullptr, 3, cus));
                          }, true});
        if (tiles <= kLookbackMaxTiles && getenv("SMALLBENCH_LB_VARIANTS")) {
            auto add = [&](const char* nm, void (*f1)(EvalArgs&, uint64_t*, hipStream_t),
                           void (*f4)(EvalArgs&, uint64_t*, hipStream_t), bool chk) {
                vs.push_back({std::string("lookback ") + nm, [&, f1, f4](EvalArgs& a, hipStream_t st) {
                                  a.epoch = ++epoch;
                                  (c.k == 4 ? f4 : f1)(a, dir, st);
                              }, chk});
            };
            // flag copies (read copy b % R), a two-level look-back (groups of 64 tiles + group
            // totals) and flag loads issued before the LDS decode measured no faster:
            // profiles/r03e_smallbench_flag_copies_two_level.txt
            vs.push_back({"lookback r03 kernel (shfl wave sum)", [&](EvalArgs& a, hipStream_t st) {
                              a.epoch = ++epoch;
                              EvalArgs a2 = a;
                              a2.flags = flags_r03;
                              if (c.k == 4)
                                  hipLaunchKernelGGL((eval_decode_lookback_r03<4, FORM_CONJ, kLookbackStage, 3>), dim3(a.num_tiles),
                                                     dim3(512), 0, st, a2, dir);
                              else
                                  hipLaunchKernelGGL((eval_decode_lookback_r03<1, FORM_CONJ, kLookbackStage, 3>), dim3(a.num_tiles),
                                                     dim3(512), 0, st, a2, dir);
                          }, true});
            add("DBG no ids", lookback_variant<1, 16, 2>, lookback_variant<4, 16, 2>, false);
            add("DBG no flag loads, no ids", lookback_variant<1, 16, 10>, lookback_variant<4, 16, 10>, false);
            add("DBG no wait, no ids", lookback_variant<1, 16, 3>, lookback_variant<4, 16, 3>, false);
        }
        if (2 * tiles <= kLookbackMaxTiles)
            vs.push_back({"lookback 65,536-row tiles (grid " + std::to_string((W + 1023) / 1024) + ")",
                          [&](EvalArgs& a, hipStream_t st) {
                              a.epoch = ++epoch;
                              (c.k == 4 ? lookback_t256<4> : lookback_t256<1>)(a, dir, st);
                          }, true, 2});
        // K = 1: the decode with its tile offsets known (EvalArgs::tile_prefix, as a single index
        // leaf decodes from its per-zone counts), and its diagnostic cuts: no ids written (DBG 2),
        // no LDS staging of the ids (16; the copy-out still runs), the copy-out only (2|16 = 18 is
        // not a variant: 2 returns first)
        if (c.k == 1) {
            if (!d_prefix) {
                // per-tile counts from one look-back decode, exclusive prefix on the host
                EvalArgs a = base;
                a.epoch = ++epoch;
                CK(launch_eval_decode(a, dir, grid, s, nullptr, nullptr, 3, cus));
                CK(hipStreamSynchronize(s));
                std::vector<uint64_t> d(2 * (uint64_t)tiles);
                CK(hipMemcpy(d.data(), dir, d.size() * 8, hipMemcpyDeviceToHost));
                std::vector<uint64_t> pre(tiles);
                uint64_t acc = 0;
                for (uint32_t tt = 0; tt < tiles; ++tt) {
                    pre[tt] = acc;
                    acc += d[2 * tt + 1];
                }
                CK(hipMalloc(&d_prefix, tiles * 8ull));
                CK(hipMemcpy(d_prefix, pre.data(), tiles * 8ull, hipMemcpyHostToDevice));
            }
            vs.push_back({"prefixed (offsets known)", [&](EvalArgs& a, hipStream_t st) {
                              a.tile_prefix = d_prefix;
                              hipLaunchKernelGGL((eval_decode_lookback<1, FORM_CONJ, kLookbackStage, 3, 16, 0>),
                                                 dim3(a.num_tiles), dim3(512), 0, st, a, dir);
                          }, true});
            vs.push_back({"prefixed, ids staged by rank (DBG 128)", [&](EvalArgs& a, hipStream_t st) {
                              a.tile_prefix = d_prefix;
                              hipLaunchKernelGGL((eval_decode_lookback<1, FORM_CONJ, kLookbackStage, 3, 16, 128>),
                                                 dim3(a.num_tiles), dim3(512), 0, st, a, dir);
                          }, true});
            vs.push_back({"prefixed DBG staging loop without LDS stores", [&](EvalArgs& a, hipStream_t st) {
                              a.tile_prefix = d_prefix;
                              hipLaunchKernelGGL((eval_decode_lookback<1, FORM_CONJ, kLookbackStage, 3, 16, 64>),
                                                 dim3(a.num_tiles), dim3(512), 0, st, a, dir);
                          }, false});
            vs.push_back({"prefixed DBG no ids", [&](EvalArgs& a, hipStream_t st) {
                              a.tile_prefix = d_prefix;
                              hipLaunchKernelGGL((eval_decode_lookback<1, FORM_CONJ, kLookbackStage, 3, 16, 2>),
                                                 dim3(a.num_tiles), dim3(512), 0, st, a, dir);
                          }, false});
            vs.push_back({"prefixed DBG no LDS staging", [&](EvalArgs& a, hipStream_t st) {
                              a.tile_prefix = d_prefix;
                              hipLaunchKernelGGL((eval_decode_lookback<1, FORM_CONJ, kLookbackStage, 3, 16, 16>),
                                                 dim3(a.num_tiles), dim3(512), 0, st, a, dir);
                          }, false});
        }
        vs.push_back({"AUTO (library policy)", [&](EvalArgs& a, hipStream_t st) {
                          a.epoch = ++epoch;
                          CK(launch_eval_decode(a, dir, grid, st, nullptr, nullptr, 0, cus));
                      }, true});
        vs.push_back({"count kernel", [&](EvalArgs& a, hipStream_t st) {
                          a.num_tiles = (uint32_t)(pw / count_tile_words(a.prog.n_leaves));
                          CK(launch_eval_count(a, st));
                      }, false});
        vs.push_back({"floor: leaves read, grid=tiles", [&](EvalArgs& a, hipStream_t st) {
                          if (c.k == 4) hipLaunchKernelGGL((floor_kernel<4, 0>), dim3(tiles), dim3(512), 0, st, a, fl_out);
                          else hipLaunchKernelGGL((floor_kernel<1, 0>), dim3(tiles), dim3(512), 0, st, a, fl_out);
                      }, false});
        vs.push_back({"floor: read + ids 16B, grid=tiles", [&](EvalArgs& a, hipStream_t st) {
                          // Q6 density: 2,496 ids per tile (K4) / 1,310 (K1 1 %)
                          if (c.k == 4) hipLaunchKernelGGL((floor_kernel<4, 2496>), dim3(tiles), dim3(512), 0, st, a, fl_out);
                          else hipLaunchKernelGGL((floor_kernel<1, 1310>), dim3(tiles), dim3(512), 0, st, a, fl_out);
                      }, false});
        vs.push_back({"empty kernel, grid=tiles", [&](EvalArgs&, hipStream_t st) {
                          hipLaunchKernelGGL(empty_kernel, dim3(tiles), dim3(512), 0, st, nullptr);
                      }, false});
        // correctness: every checked variant's ids (directory order) equal the pair kernel's
        std::vector<int64_t> ref;
        uint64_t ref_n = 0;
        for (size_t i = 0; i < vs.size(); ++i) {
            if (!vs[i].check) continue;
            EvalArgs a = base;
            const uint32_t vt = tiles * vs[i].tmul;
            CK(hipMemsetAsync(dir, 0, 2 * (uint64_t)vt * 8, s));
            CK(hipMemsetAsync(cnt, 0xff, 8, s));
            vs[i].launch(a, s);
            CK(hipStreamSynchronize(s));
            uint64_t got = 0;
            CK(hipMemcpy(&got, cnt, 8, hipMemcpyDeviceToHost));
            std::vector<int64_t> h(std::min<uint64_t>(got, cap));
            CK(hipMemcpy(h.data(), ids, h.size() * 8, hipMemcpyDeviceToHost));
            std::vector<uint64_t> d(2 * (uint64_t)vt);
            CK(hipMemcpy(d.data(), dir, d.size() * 8, hipMemcpyDeviceToHost));
            std::vector<int64_t> o;
            o.reserve(h.size());
            bool ok_dir = true;
            for (uint32_t tt = 0; tt < vt; ++tt) {
                if (d[2 * tt] + d[2 * tt + 1] > h.size()) {
                    ok_dir = false;
                    break;
                }
                o.insert(o.end(), h.begin() + d[2 * tt], h.begin() + d[2 * tt] + d[2 * tt + 1]);
            }
            if (i == 0) {
                ref = o;
                ref_n = got;
                printf("== %s: %llu rows, %u tiles, K = %d, %llu qualifying (%.2f %%)\n", c.name, (unsigned long long)n,
                       tiles, c.k, (unsigned long long)got, 100.0 * got / n);
            } else {
                printf("   %s %s\n", (ok_dir && got == ref_n && o == ref) ? "ok" : "MISMATCH", vs[i].name.c_str());
            }
        }
        // steady state: warm, then `reps` launches back to back between two events
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        const double alg = 8.0 * W * c.k + 8.0 * ref_n;
        printf("   %-38s %9s %9s %9s %9s\n", "variant", "us/launch", "min-run", "alg GB/s", "frac8TB");
        for (auto& v : vs) {
            std::vector<float> runs;
            for (int r = 0; r < 5; ++r) {
                EvalArgs a = base;
                for (int i = 0; i < 3; ++i) {
                    EvalArgs b2 = a;
                    v.launch(b2, s);
                }
                CK(hipEventRecord(e0, s));
                for (int i = 0; i < reps; ++i) {
                    EvalArgs b2 = a;
                    v.launch(b2, s);
                }
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                runs.push_back(ms * 1e3f / reps);
            }
            std::sort(runs.begin(), runs.end());
            const double us = runs[runs.size() / 2];
            printf("   %-38s %9.2f %9.2f %9.0f %9.3f\n", v.name.c_str(), us, runs[0], alg / (us * 1e-6) / 1e9,
                   alg / (us * 1e-6) / 8e12);
        }
        CK(hipEventDestroy(e0));
        CK(hipEventDestroy(e1));
        for (auto* l : leaf) CK(hipFree(l));
        CK(hipFree(ids));
        CK(hipFree(ids_ref));
        CK(hipFree(fl_out));
        CK(hipFree(ids_ord));
        CK(hipFree(dst_off));
        CK(hipFree(cnt));
        CK(hipFree(dir));
        CK(hipFree(dir_ref));
        if (d_prefix) CK(hipFree(d_prefix));
    }
    return 0;
}
