// Load-balance microbenchmark (development tool, not shipped). The headline decode's
// workgroups end over a ~22 us window while every CU streams; this asks whether
// a dynamic tile hand-out can narrow it when the dequeue never delays a leaf wait. It times, at
// SF100 size with K = 4 leaves at Q6's density, the streaming floor kernel (leaves read, the
// tile's ids written as 16-byte runs, no evaluation) with
//   static  : workgroup g walks tiles g, g + G, ... (production walk)
//   ldsnext : the same static walk through an LDS slot and one barrier per tile (the dynamic
//             variant's structure without the atomics)
//   xcd     : tiles [0, G) static, the rest from eight per-XCD heads (512-byte lines); the last
//             wave's lane 0 dequeues one tile ahead, after that wave issued its leaf loads, so
//             only the wave that waits on the atomic anyway is held by it; an exhausted head
//             sends the workgroup to the next XCD's head
//   global  : the same with one head
// next to the production run-claimed decode, with per-workgroup end stamps.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-atomic-optimizer-strategy=None \
//         -I duckdb-cubit_amd/csrc scripts/balbench.hip -o scripts/balbench
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

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void fill_random(uint64_t* w, uint64_t pw, uint64_t n_rows, uint32_t thresh, uint64_t seed) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < pw; i += stride) {
        uint64_t word = 0;
        for (int b = 0; b < 64; ++b) {
            const uint64_t row = i * 64 + b;
            const uint32_t h = (uint32_t)(mix(seed * 0x9E3779B97F4A7C15ull + row) >> 32);
            if (row < n_rows && h < thresh) word |= 1ull << b;
        }
        w[i] = word;
    }
}

constexpr int kHeadStride = 64;  // u64 words between heads: one 512-byte line each

// leaf loads with cache-policy bits LAUX (gfx950: 1 = sc0, 2 = nt, 16 = sc1)
template <int K, int PAIRS, int THREADS, int LAUX>
__device__ __forceinline__ void load_tile_aux(const EvalArgs& a, uint64_t tile_word0, int t, u64x2 (&v)[K][PAIRS]) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint64_t tw = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(tile_word0 >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)tile_word0);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(a.prog.leaf[k] + tw), (short)0, PAIRS * THREADS * 16, 0x00020000);
#pragma unroll
        for (int p = 0; p < PAIRS; ++p) {
            const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(p * THREADS + t) * 16u, 0, LAUX);
            v[k][p] = __builtin_bit_cast(u64x2, x);
        }
    }
}

// MODE 0 static, 1 ldsnext, 2 xcd heads, 3 one global head; LAUX / SAUX: cache-policy bits of
// the leaf loads / the id stores (SAUX < 0: plain stores)
template <int K, int WR, int MODE, int LAUX = 2, int SAUX = -1, bool NOWR = false, bool NORD = false>
__global__ __launch_bounds__(512, 4) void floor_walk(EvalArgs a, int64_t* out, unsigned long long* heads,
                                                      unsigned long long* done, uint64_t* stamps) {
    constexpr int THREADS = 512, PAIRS = 2;
    constexpr uint64_t TILE_WORDS = THREADS * 2 * PAIRS;
    typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
    const int t = threadIdx.x, lane = t & 63;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const uint32_t G = gridDim.x, n = a.num_tiles;
    if (t == 0) stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    __shared__ uint32_t s_next[2];
    u64x2 v[K][PAIRS];
    uint32_t cx = MODE == 3 ? 0 : (blockIdx.x & 7), tries = 0;
    unsigned long long pend = 0;
    const uint32_t stride = MODE == 3 ? 1 : 8;
    auto dequeue = [&]() {
        if (lane == 0) pend = atomicAdd(&heads[cx * kHeadStride], 1ull);
    };
    uint32_t tile = blockIdx.x, count = 0, u = 0;
    if (NORD) {
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int p = 0; p < PAIRS; ++p) v[k][p] = u64x2{(uint64_t)t, (uint64_t)blockIdx.x};
    }
    if (tile < n && !NORD) load_tile_aux<K, PAIRS, THREADS, LAUX>(a, (uint64_t)tile * TILE_WORDS, t, v);
    if (MODE >= 2 && wave == 7) dequeue();
    while (tile < n) {
        uint64_t x = 0;
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int p = 0; p < PAIRS; ++p) x ^= v[k][p].x ^ v[k][p].y;
        uint32_t next = tile + G;
        if (MODE >= 1) {
            if (wave == 7) {
                if (MODE >= 2) {
                    for (;;) {
                        const uint64_t k = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(pend >> 32)) << 32) |
                                           __builtin_amdgcn_readfirstlane((uint32_t)pend);
                        const uint64_t cand = (uint64_t)G + stride * k + cx;
                        next = cand < n ? (uint32_t)cand : n;
                        if (next < n || MODE == 3 || ++tries >= 8) break;
                        cx = (cx + 1) & 7;
                        dequeue();  // this head is exhausted: the next XCD's, synchronously
                    }
                    if (next < n) dequeue();  // for the tile after next
                }
                if (lane == 0) s_next[u & 1] = next;
            }
            __syncthreads();
            next = s_next[u & 1];
        }
        if (next < n && !NORD) load_tile_aux<K, PAIRS, THREADS, LAUX>(a, (uint64_t)next * TILE_WORDS, t, v);
        i64x2* o = reinterpret_cast<i64x2*>(out + (uint64_t)tile * (WR + 6));
        if (NOWR) {
            if (x == 0x123456789ull) out[tile] = 1;  // keep the loads
        } else if (SAUX < 0) {
            for (int i = t; i < (WR + 1) / 2; i += THREADS) {
                i64x2 val;
                val.x = (int64_t)(x + 2 * i);
                val.y = (int64_t)(x + 2 * i + 1);
                o[i] = val;
            }
        } else {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)o, (short)0, (WR + 1) / 2 * 16, 0x00020000);
            for (int i = t; i < (WR + 1) / 2; i += THREADS) {
                i64x2 val;
                val.x = (int64_t)(x + 2 * i);
                val.y = (int64_t)(x + 2 * i + 1);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, val), rs, (uint32_t)i * 16u, 0, SAUX < 0 ? 0 : SAUX);
            }
        }
        ++count;
        tile = next;
        ++u;
    }
    if (t == 0) {
        atomicAdd(done, (unsigned long long)count);
        stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 600037902ull;
    const int rounds = argc > 2 ? atoi(argv[2]) : 25;
    const uint64_t W = (n + 63) / 64, pw = padded_words(n);
    const double dens[4] = {0.25, 0.40, 0.50, 0.46};
    uint64_t* leaf[4];
    for (int k = 0; k < 4; ++k) {
        CK(hipMalloc(&leaf[k], pw * 8));
        hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, leaf[k], pw, n, (uint32_t)(dens[k] * 4294967296.0),
                           (uint64_t)k + 1);
    }
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const unsigned cus = prop.multiProcessorCount;
    const uint32_t dtiles = (uint32_t)(pw / decode_tile_words());
    const unsigned grid = std::min<unsigned>(dtiles, 2 * cus);
    const uint64_t cap = n / 10 + 4096;
    constexpr int WR = 2496;  // Q6's 11.4 M ids over 4,578 tiles
    int64_t *ids, *ids2;
    uint64_t *cnt, *dir, *ticket, *stamps;
    unsigned long long *heads, *done;
    CK(hipMalloc(&ticket, kTicketWords * 8));
    CK(hipMemset(ticket, 0, kTicketWords * 8));
    CK(hipMalloc(&ids, cap * 8));
    CK(hipMalloc(&ids2, ((uint64_t)dtiles * (WR + 6) + 64) * 8));
    CK(hipMalloc(&cnt, 64));
    CK(hipMalloc(&dir, (pw / 512 + 16) * 16));
    CK(hipMalloc(&heads, 8 * kHeadStride * 8));
    CK(hipMalloc(&done, 64));
    CK(hipMalloc(&stamps, 2 * grid * 8));
    CK(hipDeviceSynchronize());

    EvalArgs base{};
    for (int k = 0; k < 4; ++k) base.prog.leaf[k] = leaf[k];
    base.prog.n_leaves = 4;
    base.prog.form = FORM_CONJ;
    for (int k = 1; k < 4; ++k) base.prog.nops |= 1u << (4 * k);
    base.n_rows = n;
    base.n_words = W;
    base.rowids = ids;
    base.capacity = cap;
    base.count = cnt;
    base.ticket = ticket;
    base.num_tiles = dtiles;

    struct V {
        std::string name;
        std::function<void(hipStream_t)> launch;
        bool floor;
    };
    std::vector<V> vs;
    vs.push_back({"prod runs K4 (static)", [&](hipStream_t s) {
                      EvalArgs a = base;
                      hipLaunchKernelGGL((eval_decode_runs<4, 2, 9984, 512, FORM_CONJ>), dim3(grid), dim3(512), 0, s, a, dir);
                  }, false});
    // materialise one leaf AND another into a result bitvector (count kernel + result words)
    uint64_t* res;
    CK(hipMalloc(&res, pw * 8));
#define MAT(NAME, SA)                                                                                           \
    vs.push_back({NAME, [&](hipStream_t s) {                                                                   \
                      EvalArgs a = base;                                                                      \
                      a.prog.n_leaves = 2;                                                                    \
                      a.prog.nops = 1u << 4;                                                                  \
                      a.result_words = res;                                                                   \
                      a.num_tiles = (uint32_t)(pw / (512 * 2 * 2));                                           \
                      hipLaunchKernelGGL((eval_count_kernel<2, 2, FORM_CONJ, SA>), dim3(std::min<unsigned>(a.num_tiles, 4 * cus)), \
                                         dim3(512), 0, s, a);                                                 \
                  }, false})
    MAT("materialise K2 plain", -1);
    MAT("materialise K2 sc1", 16);
    vs.push_back({"runs K4 late loads", [&](hipStream_t s) {
                      EvalArgs a = base;
                      hipLaunchKernelGGL((eval_decode_runs<4, 2, 9984, 512, FORM_CONJ, 16, false, true, 16, 16, 3>), dim3(grid),
                                         dim3(512), 0, s, a, dir);
                  }, false});
    vs.push_back({"runs K4 st18 (nt+sc1)", [&](hipStream_t s) {
                      EvalArgs a = base;
                      hipLaunchKernelGGL((eval_decode_runs<4, 2, 9984, 512, FORM_CONJ, 16, false, true, 18>), dim3(grid),
                                         dim3(512), 0, s, a, dir);
                  }, false});
    vs.push_back({"runs K4 sc1 align128", [&](hipStream_t s) {
                      EvalArgs a = base;
                      hipLaunchKernelGGL((eval_decode_runs<4, 2, 9984, 512, FORM_CONJ, 16, false, true, 16, 128>), dim3(grid),
                                         dim3(512), 0, s, a, dir);
                  }, false});
    vs.push_back({"runs K4 plain align128", [&](hipStream_t s) {
                      EvalArgs a = base;
                      hipLaunchKernelGGL((eval_decode_runs<4, 2, 9984, 512, FORM_CONJ, 16, false, true, -1, 128>), dim3(grid),
                                         dim3(512), 0, s, a, dir);
                  }, false});
    vs.push_back({"runs K4 plain stores", [&](hipStream_t s) {
                      EvalArgs a = base;
                      hipLaunchKernelGGL((eval_decode_runs<4, 2, 9984, 512, FORM_CONJ, 16, false, true, -1>), dim3(grid),
                                         dim3(512), 0, s, a, dir);
                  }, false});
    vs.push_back({"runs K4 buffer st0", [&](hipStream_t s) {
                      EvalArgs a = base;
                      hipLaunchKernelGGL((eval_decode_runs<4, 2, 9984, 512, FORM_CONJ, 16, false, true, 0>), dim3(grid),
                                         dim3(512), 0, s, a, dir);
                  }, false});
    vs.push_back({"pairs K4 (sc1)", [&](hipStream_t s) {
                      EvalArgs a = base;
                      hipLaunchKernelGGL((eval_decode_pairs<4, 2, 4096, 512, 0, FORM_CONJ>), dim3(grid), dim3(512), 0, s, a, dir);
                  }, false});
    vs.push_back({"pairs K4 plain stores", [&](hipStream_t s) {
                      EvalArgs a = base;
                      hipLaunchKernelGGL((eval_decode_pairs<4, 2, 4096, 512, 0, FORM_CONJ, 2, true, -1>), dim3(grid), dim3(512), 0,
                                         s, a, dir);
                  }, false});
    // the ordered output pass over the directory and ids the variants above left
    int64_t* ord;
    CK(hipMalloc(&ord, cap * 8));
#define OR(NAME, MODE)                                                                                          \
    vs.push_back({NAME, [&](hipStream_t s) {                                                                   \
                      const uint32_t tpw = std::max<uint32_t>(1, std::min<uint32_t>(8, dtiles / 1024));        \
                      hipLaunchKernelGGL(order_runs_kernel<MODE>, dim3((dtiles + tpw - 1) / tpw), dim3(256), 0, s, dir, \
                                         dtiles, tpw, ids, cap, ord);                                           \
                  }, false})
    OR("order pass plain", 0);
    OR("order pass nt+sc1", 1);
    OR("order pass nt", 2);
#define FW(NAME, MODE, ...)                                                                                        \
    vs.push_back({NAME, [&](hipStream_t s) {                                                                   \
                      CK(hipMemsetAsync(heads, 0, 8 * kHeadStride * 8, s));                                    \
                      hipLaunchKernelGGL((floor_walk<4, WR, MODE, ##__VA_ARGS__>), dim3(grid), dim3(512), 0, s, base, ids2, heads, \
                                         done, stamps);                                                        \
                  }, true})
    FW("floor static", 0);
    FW("floor ldsnext", 1);
    FW("floor xcd heads", 2);
    FW("floor global head", 3);
    FW("ldsnext ld0 st-", 1, 0, -1);
    FW("ldsnext ld2 st0", 1, 2, 0);
    FW("ldsnext ld2 st2", 1, 2, 2);
    FW("ldsnext ld2 st16", 1, 2, 16);
    FW("ldsnext ld2 st17", 1, 2, 17);
    FW("ldsnext ld16 st-", 1, 16, -1);
    FW("ldsnext ld18 st-", 1, 18, -1);
    FW("ldsnext ld3 st-", 1, 3, -1);
    FW("ldsnext ld0 st2", 1, 0, 2);
    FW("ldsnext ld2 st18", 1, 2, 18);
    FW("ldsnext ld18 st16", 1, 18, 16);
    FW("ldsnext ld3 st16", 1, 3, 16);
    FW("reads only ld2", 1, 2, -1, true);
    FW("writes only st-", 1, 2, -1, false, true);
    FW("writes only st16", 1, 2, 16, false, true);
    FW("reads only ld0", 1, 0, -1, true);

    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> times(vs.size());
    std::vector<std::vector<double>> spreads(vs.size()), medends(vs.size());
    std::vector<uint64_t> h(2 * grid);
    for (int r = 0; r < rounds + 2; ++r) {
        for (size_t i = 0; i < vs.size(); ++i) {
            CK(hipMemsetAsync(done, 0, 8, s));
            if (!vs[i].floor && vs[i].name.rfind("order", 0) != 0) CK(hipMemsetAsync(dir, 0, dtiles * 16, s));
            CK(hipEventRecord(e0, s));
            vs[i].launch(s);
            CK(hipEventRecord(e1, s));
            CK(hipStreamSynchronize(s));
            CK(hipGetLastError());
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r < 2) continue;
            times[i].push_back(ms);
            if (vs[i].floor) {
                unsigned long long d = 0;
                CK(hipMemcpy(&d, done, 8, hipMemcpyDeviceToHost));
                if (d != dtiles) {
                    printf("MISMATCH %s: %llu tiles walked of %u\n", vs[i].name.c_str(), d, dtiles);
                    return 1;
                }
                CK(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
                uint64_t s0 = ~0ull, e_min = ~0ull, e_max = 0;
                std::vector<double> ends;
                for (unsigned g = 0; g < grid; ++g) {
                    s0 = std::min(s0, h[2 * g]);
                    e_min = std::min(e_min, h[2 * g + 1]);
                    e_max = std::max(e_max, h[2 * g + 1]);
                }
                for (unsigned g = 0; g < grid; ++g) ends.push_back((h[2 * g + 1] - s0) / 100.0);
                std::sort(ends.begin(), ends.end());
                spreads[i].push_back((e_max - e_min) / 100.0);
                medends[i].push_back(ends[grid / 2]);
            }
        }
    }
    auto med = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v.empty() ? 0.0 : v[v.size() / 2];
    };
    printf("n %llu, %u tiles, grid %u, %d rounds; floor bytes = 4 leaves + %d ids per tile\n", (unsigned long long)n,
           dtiles, grid, rounds, WR);
    printf("%-24s %10s %10s %10s %12s %12s\n", "variant", "median_us", "min_us", "GB/s", "end_spread", "median_end");
    const double bytes = 8.0 * W * 4 + 8.0 * WR * dtiles;
    for (size_t i = 0; i < vs.size(); ++i) {
        std::vector<double> t(times[i].begin(), times[i].end());
        std::sort(t.begin(), t.end());
        const double m = med(t) * 1e3;
        printf("%-24s %10.1f %10.1f %10.0f %12.1f %12.1f\n", vs[i].name.c_str(), m, t[0] * 1e3, bytes / (m * 1e-6) / 1e9,
               med(spreads[i]), med(medends[i]));
    }
    return 0;
}
