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

// look-back variants with the kernel's diagnostic switches (DBG: 1 no wait, 2 no ids, 4 no sleep)
template <int K, int SAUX, int DBG>
void lookback_variant(EvalArgs& a, uint64_t* dir, hipStream_t st) {
    hipLaunchKernelGGL((eval_decode_lookback<K, FORM_CONJ, kLookbackStage, lookback_wpc(K), SAUX, DBG>), dim3(a.num_tiles),
                       dim3(512), 0, st, a, dir);
}

struct Variant {
    std::string name;
    std::function<void(EvalArgs&, hipStream_t)> launch;
    bool check;
};

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
        CK(hipMalloc(&cnt, 16));
        CK(hipMalloc(&dir, 2 * (uint64_t)tiles * 8 + 64));
        CK(hipMalloc(&dir_ref, 2 * (uint64_t)tiles * 8 + 64));
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
            add("SAUX plain", lookback_variant<1, -1, 0>, lookback_variant<4, -1, 0>, true);
            add("SAUX nt", lookback_variant<1, 2, 0>, lookback_variant<4, 2, 0>, true);
            add("SAUX 0", lookback_variant<1, 0, 0>, lookback_variant<4, 0, 0>, true);
            add("no sleep", lookback_variant<1, 16, 4>, lookback_variant<4, 16, 4>, true);
            add("DBG no wait", lookback_variant<1, 16, 1>, lookback_variant<4, 16, 1>, false);
            add("DBG no ids", lookback_variant<1, 16, 2>, lookback_variant<4, 16, 2>, false);
            add("DBG no wait, no ids", lookback_variant<1, 16, 3>, lookback_variant<4, 16, 3>, false);
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
            CK(hipMemsetAsync(dir, 0, 2 * (uint64_t)tiles * 8, s));
            CK(hipMemsetAsync(cnt, 0xff, 8, s));
            vs[i].launch(a, s);
            CK(hipStreamSynchronize(s));
            uint64_t got = 0;
            CK(hipMemcpy(&got, cnt, 8, hipMemcpyDeviceToHost));
            std::vector<int64_t> h(std::min<uint64_t>(got, cap));
            CK(hipMemcpy(h.data(), ids, h.size() * 8, hipMemcpyDeviceToHost));
            std::vector<uint64_t> d(2 * (uint64_t)tiles);
            CK(hipMemcpy(d.data(), dir, d.size() * 8, hipMemcpyDeviceToHost));
            std::vector<int64_t> o;
            o.reserve(h.size());
            bool ok_dir = true;
            for (uint32_t tt = 0; tt < tiles; ++tt) {
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
        CK(hipFree(cnt));
        CK(hipFree(dir));
        CK(hipFree(dir_ref));
    }
    return 0;
}
