// Kernel microbenchmark (development tool, not shipped): times the evaluate/decode kernels
// interleaved in one process on SF100-sized bitvectors (600,037,902 rows, K = 5 leaves,
// Q6-like densities, ~1.9 % selected) and checks every variant against the production
// decode (row ids rebuilt in row order through the tile directory).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-atomic-optimizer-strategy=None \
//         -I duckdb-cubit_amd/csrc scripts/kbench.hip -o scripts/kbench
// (the library's flags: the claims stay single-lane atomics, as in libcubitgpu.so)
// The variant sweep that chose the production geometry is summarised in DESIGN.md §3.
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

// Bandwidth floor for this read/write mix: the same persistent tile walk and leaf loads,
// then WR int64 written per tile as one contiguous coalesced run (no eval / LDS / atomics).
template <int K, int WR, int MODE = 0>
__global__ __launch_bounds__(512, 4) void stream_floor(EvalArgs a, int64_t* out) {
    constexpr int THREADS = 512, PAIRS = 2;
    constexpr uint64_t TILE_WORDS = THREADS * 2 * PAIRS;
    const int t = threadIdx.x;
    u64x2 v[K][PAIRS];
    __shared__ uint32_t s_st[4096];
    uint32_t tile = blockIdx.x;
    if (tile < a.num_tiles) load_tile<K, PAIRS, THREADS>(a, (uint64_t)tile * TILE_WORDS, t, v);
    while (tile < a.num_tiles) {
        if (MODE >= 3) __syncthreads();
        uint64_t x = 0;
#pragma unroll
        for (int k = 0; k < K; ++k)
#pragma unroll
            for (int p = 0; p < PAIRS; ++p) x ^= v[k][p].x ^ v[k][p].y;
        const uint32_t next = tile + gridDim.x;
        if (next < a.num_tiles) load_tile<K, PAIRS, THREADS>(a, (uint64_t)next * TILE_WORDS, t, v);
        if (WR > 0) {
            if (MODE == 0) {
                for (int i = t; i < WR; i += THREADS) out[(uint64_t)tile * WR + i] = (int64_t)(x + i);
            } else if (MODE == 1) {
                for (int i = t; i < WR; i += THREADS) __builtin_nontemporal_store((int64_t)(x + i), out + (uint64_t)tile * WR + i);
            } else if (MODE == 3) {
                // one block barrier per tile, 16 B stores from registers
                typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
                i64x2* o = reinterpret_cast<i64x2*>(out + (uint64_t)tile * (WR + 6));
                for (int i = t; i < (WR + 1) / 2; i += THREADS) {
                    i64x2 val;
                    val.x = (int64_t)(x + 2 * i);
                    val.y = (int64_t)(x + 2 * i + 1);
                    o[i] = val;
                }
            } else if (MODE == 4) {
                // LDS staging: every thread writes ~WR/THREADS u32, barrier, 16 B stores from LDS
                for (int i = t; i < WR; i += THREADS) s_st[(i * 5) % WR] = (uint32_t)(x + i);
                __syncthreads();
                typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
                i64x2* o = reinterpret_cast<i64x2*>(out + (uint64_t)tile * (WR + 6));
                for (int i = t; i < (WR + 1) / 2; i += THREADS) {
                    i64x2 val;
                    val.x = (int64_t)s_st[2 * i];
                    val.y = (int64_t)s_st[2 * i + 1];
                    o[i] = val;
                }
            } else {
                // 16 B per lane
                typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
                i64x2* o = reinterpret_cast<i64x2*>(out + (uint64_t)tile * (WR + 6));
                for (int i = t; i < (WR + 1) / 2; i += THREADS) {
                    i64x2 val;
                    val.x = (int64_t)(x + 2 * i);
                    val.y = (int64_t)(x + 2 * i + 1);
                    o[i] = val;
                }
            }
        } else if (x == 0x123456789ull) {
            out[tile] = 1;  // keep the loads
        }
        tile = next;
    }
}

struct Variant {
    std::string name;
    std::function<void(EvalArgs&, hipStream_t)> launch;
    int kind;  // 0 = tile runs + dir, 1 = ordered output, 2 = count only
};

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 600037902ull;
    const int rounds = argc > 2 ? atoi(argv[2]) : 15;
    const uint64_t W = (n + 63) / 64, pw = padded_words(n);
    const double dens[6] = {0.25, 0.40, 0.50, 0.45, 0.46, 0.01};
    uint64_t* leaf[6];
    for (int k = 0; k < 6; ++k) {
        CK(hipMalloc(&leaf[k], pw * 8));
        hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, leaf[k], pw, n, (uint32_t)(dens[k] * 4294967296.0),
                           (uint64_t)k + 1);
    }
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const unsigned cus = prop.multiProcessorCount;
    const uint64_t cap = n / 10 + 4096;  // diag no-claim writes up to n/50 + a tile
    int64_t *ids, *ids2;
    uint64_t* ovf;
    uint64_t *cnt, *dir, *dst_off, *ticket;
    CK(hipMalloc(&ticket, kTicketWords * 8));
    CK(hipMemset(ticket, 0, kTicketWords * 8));
    CK(hipMalloc(&ids, cap * 8));
    CK(hipMalloc(&ids2, (cap + pw * 2) * 8));
    CK(hipMalloc(&ovf, 64));
    CK(hipMalloc(&cnt, 64));
    CK(hipMalloc(&dir, (pw / 512 + 16) * 16));
    CK(hipMalloc(&dst_off, (pw / 512 + 16) * 8));
    CK(hipDeviceSynchronize());

    EvalArgs base{};
    for (int k = 0; k < 5; ++k) base.prog.leaf[k] = leaf[k];
    base.prog.n_leaves = 5;
    // (L0 ANDNOT L1) AND (L2 ANDNOT L3) AND L4
    const uint32_t nops[5] = {0, 1, 0, 2, 1};
    const uint32_t ops[4] = {OP_ANDNOT, OP_ANDNOT, OP_AND, OP_AND};
    for (int k = 0; k < 5; ++k) base.prog.nops |= nops[k] << (4 * k);
    for (int i = 0; i < 4; ++i) base.prog.ops |= ops[i] << (2 * i);
    base.n_rows = n;
    base.n_words = W;
    base.rowids = ids;
    base.capacity = cap;
    base.count = cnt;
    base.ticket = ticket;

    std::vector<Variant> vs;
    const uint32_t dtiles = (uint32_t)(pw / decode_tile_words());
    vs.push_back({"decode (prod, interpreted)", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      CK(launch_eval_decode(a, dir, std::min<unsigned>(dtiles, 2 * cus), s));
                  }, 0});
    vs.push_back({"tiles kernel (r01 prod)", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      hipLaunchKernelGGL((eval_decode_tiles<5, 2, 4096, 512>), dim3(std::min<unsigned>(dtiles, 2 * cus)),
                                         dim3(512), 0, s, a, dir);
                  }, 0});
    // the same predicate as a left-deep AND chain with complemented leaves → branch-free CONJ path
    vs.push_back({"decode conj (prod)", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      a.prog.negate = 0b01010;
                      a.prog.nops = 0;
                      for (int k = 1; k < 5; ++k) a.prog.nops |= 1u << (4 * k);
                      a.prog.ops = 0;
                      for (int i = 0; i < 4; ++i) a.prog.ops |= (uint32_t)OP_AND << (2 * i);
                      CK(launch_eval_decode(a, dir, std::min<unsigned>(dtiles, 2 * cus), s));
                  }, 0});
#define DT(NAME, P, S, T, WGPC)                                                                                \
    vs.push_back({NAME, [&](EvalArgs& a, hipStream_t s) {                                                     \
                      a.num_tiles = (uint32_t)(pw / ((uint64_t)T * 2 * P));                                   \
                      hipLaunchKernelGGL((eval_decode_tiles<5, P, S, T>), dim3(std::min<unsigned>(a.num_tiles, WGPC * cus)), \
                                         dim3(T), 0, s, a, dir);                                              \
                  }, 0})
#define DX(NAME, CL, DE)                                                                                       \
    vs.push_back({NAME, [&](EvalArgs& a, hipStream_t s) {                                                     \
                      a.num_tiles = dtiles;                                                                   \
                      hipLaunchKernelGGL((eval_decode_tiles<5, 2, 4096, 512, CL, DE>), dim3(std::min<unsigned>(dtiles, 2 * cus)), \
                                         dim3(512), 0, s, a, dir);                                            \
                  }, 3})
#define DP(NAME, P, S, T, WGPC)                                                                                \
    vs.push_back({NAME, [&](EvalArgs& a, hipStream_t s) {                                                     \
                      a.num_tiles = (uint32_t)(pw / ((uint64_t)T * 2 * P));                                   \
                      hipLaunchKernelGGL((eval_decode_pairs<5, P, S, T>), dim3(std::min<unsigned>(a.num_tiles, WGPC * cus)), \
                                         dim3(T), 0, s, a, dir);                                              \
                  }, 0})
    DP("pairs P2 T512 x2/CU", 2, 4096, 512, 2);
#define DPD(NAME, D)                                                                                           \
    vs.push_back({NAME, [&](EvalArgs& a, hipStream_t s) {                                                     \
                      a.num_tiles = dtiles;                                                                   \
                      hipLaunchKernelGGL((eval_decode_pairs<5, 2, 4096, 512, D>), dim3(std::min<unsigned>(dtiles, 2 * cus)), \
                                         dim3(512), 0, s, a, dir);                                            \
                  }, 3})
    vs.push_back({"pairs conj", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      a.prog.negate = 0b01010;
                      a.prog.nops = 0;
                      for (int k = 1; k < 5; ++k) a.prog.nops |= 1u << (4 * k);
                      a.prog.ops = 0;
                      hipLaunchKernelGGL((eval_decode_pairs<5, 2, 4096, 512, 0, FORM_CONJ>), dim3(std::min<unsigned>(dtiles, 2 * cus)),
                                         dim3(512), 0, s, a, dir);
                  }, 0});
    // run-claimed decode (one claim per LDS-stage-full run, one barrier per tile)
    vs.push_back({"runs conj", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      a.prog.negate = 0b01010;
                      a.prog.nops = 0;
                      for (int k = 1; k < 5; ++k) a.prog.nops |= 1u << (4 * k);
                      a.prog.ops = 0;
                      hipLaunchKernelGGL((eval_decode_runs<5, 2, 8192, 512, FORM_CONJ>), dim3(std::min<unsigned>(dtiles, 2 * cus)),
                                         dim3(512), 0, s, a, dir);
                  }, 0});
    vs.push_back({"runs conj MAXT8", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      a.prog.negate = 0b01010;
                      a.prog.nops = 0;
                      for (int k = 1; k < 5; ++k) a.prog.nops |= 1u << (4 * k);
                      a.prog.ops = 0;
                      hipLaunchKernelGGL((eval_decode_runs<5, 2, 8192, 512, FORM_CONJ, 8>), dim3(std::min<unsigned>(dtiles, 2 * cus)),
                                         dim3(512), 0, s, a, dir);
                  }, 0});
    DT("tiles P2 T512 x2/CU", 2, 4096, 512, 2);
    DT("tiles P2 T512 grid=tiles", 2, 4096, 512, 1000000);
    DT("tiles P1 T512 x2/CU", 1, 2048, 512, 2);
    DT("tiles P1 T256 x4/CU", 1, 1024, 256, 4);
    DT("tiles P2 T256 x4/CU", 2, 2048, 256, 4);
    DP("pairs P1 T512 x2/CU", 1, 2048, 512, 2);
    DP("pairs P1 T256 x4/CU", 1, 1024, 256, 4);
#define DPC(NAME, S, OCC, T)                                                                                   \
    vs.push_back({NAME, [&](EvalArgs& a, hipStream_t s) {                                                     \
                      a.num_tiles = (uint32_t)(pw / ((uint64_t)T * 4));                                       \
                      a.prog.negate = 0b01010;                                                                \
                      a.prog.nops = 0;                                                                        \
                      for (int k = 1; k < 5; ++k) a.prog.nops |= 1u << (4 * k);                              \
                      a.prog.ops = 0;                                                                         \
                      hipLaunchKernelGGL((eval_decode_pairs<5, 2, S, T, 0, FORM_CONJ, OCC>),                  \
                                         dim3(std::min<unsigned>(a.num_tiles, OCC * cus)), dim3(T), 0, s, a, dir); \
                  }, 0})
    // DPC("pairs conj S3072 x3/CU", 3072, 3, 512);  // 80-VGPR cap spills 107 VGPRs: not viable
    DPC("pairs conj S4096 x2/CU", 4096, 2, 512);
    // one pair of words per thread: 1,024-word tiles (finer balance for mid-size partitions)
    vs.push_back({"pairs conj P1 S2048", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = (uint32_t)(pw / 1024);
                      a.prog.negate = 0b01010;
                      a.prog.nops = 0;
                      for (int k = 1; k < 5; ++k) a.prog.nops |= 1u << (4 * k);
                      a.prog.ops = 0;
                      hipLaunchKernelGGL((eval_decode_pairs<5, 1, 2048, 512, 0, FORM_CONJ, 2>),
                                         dim3(std::min<unsigned>(a.num_tiles, 2 * cus)), dim3(512), 0, s, a, dir);
                  }, 0});
    DPC("pairs conj T256 S2048 x4/CU", 2048, 4, 256);
    // K = 4 (Q6 with the year bin): L0 ∧ ¬L1 ∧ L2 ∧ L4 as CONJ, at 2 and 3 workgroups per CU
#define DK4(NAME, S, OCC)                                                                                      \
    vs.push_back({NAME, [&](EvalArgs& a, hipStream_t s) {                                                     \
                      a.num_tiles = dtiles;                                                                   \
                      a.prog.leaf[3] = leaf[4];                                                               \
                      a.prog.n_leaves = 4;                                                                    \
                      a.prog.negate = 0b0010;                                                                 \
                      a.prog.nops = 0;                                                                        \
                      for (int k = 1; k < 4; ++k) a.prog.nops |= 1u << (4 * k);                              \
                      a.prog.ops = 0;                                                                         \
                      hipLaunchKernelGGL((eval_decode_pairs<4, 2, S, 512, 0, FORM_CONJ, OCC>),                \
                                         dim3(std::min<unsigned>(dtiles, OCC * cus)), dim3(512), 0, s, a, dir); \
                  }, 3})
    DK4("K4 conj x2/CU (prod)", 4096, 2);
    // K = 4 at Q6's density (L0 ∧ L1 ∧ L2 ∧ L4 ≈ 2.3 %). Measured: issuing B's loads after
    // the copy-out stores instead of right after A's evaluation changed nothing (72.9 vs
    // 73.1 µs), so the wait for B does not pay for the stores
    vs.push_back({"K4 q6-density conj (prod)", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      a.prog.leaf[3] = leaf[4];
                      a.prog.n_leaves = 4;
                      a.prog.negate = 0;
                      a.prog.nops = 0;
                      for (int k = 1; k < 4; ++k) a.prog.nops |= 1u << (4 * k);
                      a.prog.ops = 0;
                      hipLaunchKernelGGL((eval_decode_pairs<4, 2, 4096, 512, 0, FORM_CONJ>),
                                         dim3(std::min<unsigned>(dtiles, 2 * cus)), dim3(512), 0, s, a, dir);
                  }, 3});
    // (S3072 x3/CU: the 80-VGPR cap spills 192 B per thread, 199 µs — not viable)
    DK4("K4 conj S3072 x2/CU", 3072, 2);
    // larger grids: the hardware dispatcher hands out the work (WGs beyond the two resident
    // per CU start as others finish) — load balance without atomics, no cross-tile prefetch
#define K4G(NAME, DIV)                                                                                         \
    vs.push_back({NAME, [&](EvalArgs& a, hipStream_t s) {                                                     \
                      a.num_tiles = dtiles;                                                                   \
                      a.prog.leaf[3] = leaf[4];                                                               \
                      a.prog.n_leaves = 4;                                                                    \
                      a.prog.negate = 0;                                                                      \
                      a.prog.nops = 0;                                                                        \
                      for (int k = 1; k < 4; ++k) a.prog.nops |= 1u << (4 * k);                              \
                      a.prog.ops = 0;                                                                         \
                      hipLaunchKernelGGL((eval_decode_pairs<4, 2, 4096, 512, 0, FORM_CONJ>),                  \
                                         dim3((dtiles + DIV - 1) / DIV), dim3(512), 0, s, a, dir);            \
                  }, 3})
    vs.push_back({"K4 q6-density auto", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      a.prog.leaf[3] = leaf[4];
                      a.prog.n_leaves = 4;
                      a.prog.negate = 0;
                      a.prog.nops = 0;
                      for (int k = 1; k < 4; ++k) a.prog.nops |= 1u << (4 * k);
                      a.prog.ops = 0;
                      a.prog.form = FORM_CONJ;
                      CK(launch_eval_decode(a, dir, std::min<unsigned>(dtiles, 2 * cus), s));
                  }, 3});
    K4G("K4 q6-density pairs grid=tiles/2", 2);
    K4G("K4 q6-density pairs grid=tiles/4", 4);
    K4G("K4 q6-density pairs grid=tiles/6", 6);
    vs.push_back({"K4 q6-density runs cap9984", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      a.prog.leaf[3] = leaf[4];
                      a.prog.n_leaves = 4;
                      a.prog.negate = 0;
                      a.prog.nops = 0;
                      for (int k = 1; k < 4; ++k) a.prog.nops |= 1u << (4 * k);
                      a.prog.ops = 0;
                      hipLaunchKernelGGL((eval_decode_runs<4, 2, 9984, 512, FORM_CONJ>),
                                         dim3(std::min<unsigned>(dtiles, 2 * cus)), dim3(512), 0, s, a, dir);
                  }, 3});
    vs.push_back({"K4 q6-density runs", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      a.prog.leaf[3] = leaf[4];
                      a.prog.n_leaves = 4;
                      a.prog.negate = 0;
                      a.prog.nops = 0;
                      for (int k = 1; k < 4; ++k) a.prog.nops |= 1u << (4 * k);
                      a.prog.ops = 0;
                      hipLaunchKernelGGL((eval_decode_runs<4, 2, 8192, 512, FORM_CONJ>),
                                         dim3(std::min<unsigned>(dtiles, 2 * cus)), dim3(512), 0, s, a, dir);
                  }, 3});
    DPD("pairs diag no-claim", 1);
    DPD("pairs diag fake-decode", 2);
    DPD("pairs diag no-claim fake-decode", 3);
    vs.push_back({"floor: reads only", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      hipLaunchKernelGGL((stream_floor<5, 0>), dim3(std::min<unsigned>(dtiles, 2 * cus)), dim3(512), 0, s, a, ids2);
                  }, 3});
    vs.push_back({"floor: + ids nt store", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      hipLaunchKernelGGL((stream_floor<5, 2490, 1>), dim3(std::min<unsigned>(dtiles, 2 * cus)), dim3(512), 0, s, a, ids2);
                  }, 3});
    vs.push_back({"floor: + ids 16B/lane", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      hipLaunchKernelGGL((stream_floor<5, 2490, 2>), dim3(std::min<unsigned>(dtiles, 2 * cus)), dim3(512), 0, s, a, ids2);
                  }, 3});
    vs.push_back({"floor: 16B + 1 barrier", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      hipLaunchKernelGGL((stream_floor<5, 2490, 3>), dim3(std::min<unsigned>(dtiles, 2 * cus)), dim3(512), 0, s, a, ids2);
                  }, 3});
    vs.push_back({"floor: 16B + LDS stage", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      hipLaunchKernelGGL((stream_floor<5, 2490, 4>), dim3(std::min<unsigned>(dtiles, 2 * cus)), dim3(512), 0, s, a, ids2);
                  }, 3});
    vs.push_back({"floor: reads + 2490 ids/tile", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      hipLaunchKernelGGL((stream_floor<5, 2490>), dim3(std::min<unsigned>(dtiles, 2 * cus)), dim3(512), 0, s, a, ids2);
                  }, 3});
    DX("diag no-claim", false, true);
    DX("diag no-decode", true, false);
    DX("diag no-claim no-decode", false, false);

    // K = 1 at 1 % density (config 2's shape): production path vs a non-persistent grid
    auto k1 = [&](EvalArgs& a) {
        a.prog = EvalProgram{};
        a.prog.leaf[0] = leaf[5];
        a.prog.n_leaves = 1;
    };
    vs.push_back({"K1 1% prod (pairs)", [&](EvalArgs& a, hipStream_t s) {
                      k1(a);
                      a.num_tiles = dtiles;
                      CK(launch_eval_decode(a, dir, std::min<unsigned>(dtiles, 2 * cus), s));
                  }, 3});
    // K = 1 breakdown: no claim (fixed offsets), uniform fake decode, both; the streaming floor
    // of the same bytes (1 leaf read + 1,310 ids per tile written as 16 B runs)
#define K1D(NAME, D)                                                                                           \
    vs.push_back({NAME, [&](EvalArgs& a, hipStream_t s) {                                                     \
                      k1(a);                                                                                  \
                      a.num_tiles = dtiles;                                                                   \
                      hipLaunchKernelGGL((eval_decode_pairs<1, 2, 4096, 512, D, FORM_CONJ>),                  \
                                         dim3(std::min<unsigned>(dtiles, 2 * cus)), dim3(512), 0, s, a, dir); \
                  }, 3})
    K1D("K1 1% diag no-claim", 1);
    K1D("K1 1% diag fake-decode", 2);
    K1D("K1 1% diag no-claim fake", 3);
    vs.push_back({"K1 1% floor: 16B ids", [&](EvalArgs& a, hipStream_t s) {
                      k1(a);
                      a.num_tiles = dtiles;
                      hipLaunchKernelGGL((stream_floor<1, 1310, 2>), dim3(std::min<unsigned>(dtiles, 2 * cus)), dim3(512), 0, s, a, ids2);
                  }, 3});
    vs.push_back({"K1 1% floor: LDS stage", [&](EvalArgs& a, hipStream_t s) {
                      k1(a);
                      a.num_tiles = dtiles;
                      hipLaunchKernelGGL((stream_floor<1, 1310, 4>), dim3(std::min<unsigned>(dtiles, 2 * cus)), dim3(512), 0, s, a, ids2);
                  }, 3});
    vs.push_back({"K1 1% runs", [&](EvalArgs& a, hipStream_t s) {
                      k1(a);
                      a.num_tiles = dtiles;
                      hipLaunchKernelGGL((eval_decode_runs<1, 2, 8192, 512, FORM_CONJ>),
                                         dim3(std::min<unsigned>(dtiles, 2 * cus)), dim3(512), 0, s, a, dir);
                  }, 3});
    vs.push_back({"K1 1% runs grid=tiles/2", [&](EvalArgs& a, hipStream_t s) {
                      k1(a);
                      a.num_tiles = dtiles;
                      hipLaunchKernelGGL((eval_decode_runs<1, 2, 8192, 512, FORM_CONJ>),
                                         dim3(std::min<unsigned>((dtiles + 1) / 2, 2 * cus)), dim3(512), 0, s, a, dir);
                  }, 3});
    // K = 2 (1 % ∧ ¬25 %) and K = 3 (1 % ∧ ¬25 % ∧ ¬50 %), CONJ: pairs vs runs
#define KPR(NAME, KK, NEG, RUNS)                                                                               \
    vs.push_back({NAME, [&](EvalArgs& a, hipStream_t s) {                                                     \
                      a.prog = EvalProgram{};                                                                 \
                      a.prog.leaf[0] = leaf[5];                                                               \
                      a.prog.leaf[1] = leaf[0];                                                               \
                      a.prog.leaf[2] = leaf[2];                                                               \
                      a.prog.n_leaves = KK;                                                                   \
                      a.prog.negate = NEG;                                                                    \
                      a.num_tiles = dtiles;                                                                   \
                      if (RUNS)                                                                               \
                          hipLaunchKernelGGL((eval_decode_runs<KK, 2, 8192, 512, FORM_CONJ>),                 \
                                             dim3(std::min<unsigned>(dtiles, 2 * cus)), dim3(512), 0, s, a, dir); \
                      else                                                                                    \
                          hipLaunchKernelGGL((eval_decode_pairs<KK, 2, 4096, 512, 0, FORM_CONJ>),             \
                                             dim3(std::min<unsigned>(dtiles, 2 * cus)), dim3(512), 0, s, a, dir); \
                  }, 3})
    KPR("K2 0.75% pairs", 2, 0b10, false);
    KPR("K2 0.75% runs", 2, 0b10, true);
    KPR("K3 0.4% pairs", 3, 0b110, false);
    KPR("K3 0.4% runs", 3, 0b110, true);
    vs.push_back({"K3 0.4% auto", [&](EvalArgs& a, hipStream_t s) {
                      a.prog = EvalProgram{};
                      a.prog.leaf[0] = leaf[5];
                      a.prog.leaf[1] = leaf[0];
                      a.prog.leaf[2] = leaf[2];
                      a.prog.n_leaves = 3;
                      a.prog.negate = 0b110;
                      a.prog.form = FORM_CONJ;
                      a.num_tiles = dtiles;
                      CK(launch_eval_decode(a, dir, std::min<unsigned>(dtiles, 2 * cus), s));
                  }, 3});
    vs.push_back({"K1 1% pairs P1", [&](EvalArgs& a, hipStream_t s) {
                      k1(a);
                      a.num_tiles = (uint32_t)(pw / 1024);
                      hipLaunchKernelGGL((eval_decode_pairs<1, 1, 2048, 512, 0, FORM_CONJ, 2>),
                                         dim3(std::min<unsigned>(a.num_tiles, 2 * cus)), dim3(512), 0, s, a, dir);
                  }, 3});
    // fewer claims for small inputs: one pair per workgroup (the library's grid for ≤ 2 tiles
    // per workgroup), and 4,096-word tiles with half the workgroups and half the claims
    vs.push_back({"K1 1% P2 grid=tiles/2", [&](EvalArgs& a, hipStream_t s) {
                      k1(a);
                      a.num_tiles = dtiles;
                      hipLaunchKernelGGL((eval_decode_pairs<1, 2, 4096, 512, 0, FORM_CONJ, 2>),
                                         dim3(std::min<unsigned>((dtiles + 1) / 2, 2 * cus)), dim3(512), 0, s, a, dir);
                  }, 3});
    vs.push_back({"K1 1% tiles grid=tiles", [&](EvalArgs& a, hipStream_t s) {
                      k1(a);
                      a.num_tiles = dtiles;
                      hipLaunchKernelGGL((eval_decode_tiles<1, 2, 4096, 512>), dim3(dtiles), dim3(512), 0, s, a, dir);
                  }, 3});
    vs.push_back({"K1 1% tiles P1 grid=tiles", [&](EvalArgs& a, hipStream_t s) {
                      k1(a);
                      a.num_tiles = (uint32_t)(pw / 1024);
                      hipLaunchKernelGGL((eval_decode_tiles<1, 1, 2048, 512>), dim3(a.num_tiles), dim3(512), 0, s, a, dir);
                  }, 3});
    vs.push_back({"K1 1% count only", [&](EvalArgs& a, hipStream_t s) {
                      k1(a);
                      a.num_tiles = (uint32_t)(pw / count_tile_words(a.prog.n_leaves));
                      CK(launch_eval_count(a, s));
                  }, 3});
    vs.push_back({"decode + ordered pass", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = dtiles;
                      a.rowids = ids2;
                      CK(launch_eval_decode(a, dir, std::min<unsigned>(dtiles, 2 * cus), s));
                      CK(launch_order_runs(dir, dtiles, dst_off, ids2, cap, ids, s));
                  }, 1});
    vs.push_back({"count only", [&](EvalArgs& a, hipStream_t s) {
                      a.num_tiles = (uint32_t)(pw / count_tile_words(a.prog.n_leaves));
                      CK(launch_eval_count(a, s));
                  }, 2});

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::vector<float>> times(vs.size());
    uint64_t ref_count = 0;
    std::vector<int64_t> ref_ids;
    for (int r = -1; r < rounds; ++r) {
        for (size_t i = 0; i < vs.size(); ++i) {
            EvalArgs a = base;
            CK(hipMemsetAsync(cnt, 0, 8, 0));
            CK(hipEventRecord(e0, 0));
            vs[i].launch(a, 0);
            CK(hipGetLastError());
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 0) times[i].push_back(ms);
            if (r != -1) continue;
            uint64_t c = 0;
            CK(hipMemcpy(&c, cnt, 8, hipMemcpyDeviceToHost));
            if (vs[i].kind == 3) continue;
            if (vs[i].kind == 2) {
                printf("%s %s\n", c == ref_count ? "ok" : "MISMATCH", vs[i].name.c_str());
                continue;
            }
            std::vector<int64_t> h(c);
            if (vs[i].kind == 4) {
                // slotted: gather runs in tile order through the directory
                std::vector<uint64_t> d(2 * a.num_tiles);
                CK(hipMemcpy(d.data(), dir, d.size() * 8, hipMemcpyDeviceToHost));
                std::vector<int64_t> o;
                o.reserve(c);
                for (uint32_t tt = 0; tt < a.num_tiles; ++tt) {
                    std::vector<int64_t> run(d[2 * tt + 1]);
                    if (!run.empty())
                        CK(hipMemcpy(run.data(), ids2 + d[2 * tt], run.size() * 8, hipMemcpyDeviceToHost));
                    o.insert(o.end(), run.begin(), run.end());
                }
                h.swap(o);
            } else {
                CK(hipMemcpy(h.data(), ids, c * 8, hipMemcpyDeviceToHost));
            }
            if (vs[i].kind == 0) {
                std::vector<uint64_t> d(2 * a.num_tiles);
                CK(hipMemcpy(d.data(), dir, d.size() * 8, hipMemcpyDeviceToHost));
                std::vector<int64_t> o;
                o.reserve(c);
                for (uint32_t tt = 0; tt < a.num_tiles; ++tt)
                    o.insert(o.end(), h.begin() + d[2 * tt], h.begin() + d[2 * tt] + d[2 * tt + 1]);
                h.swap(o);
            }
            if (i == 0) {
                ref_count = c;
                ref_ids = h;
                printf("reference count %llu (%.3f %% of %llu rows)\n", (unsigned long long)c, 100.0 * c / n,
                       (unsigned long long)n);
            } else {
                printf("%s %s\n", h == ref_ids ? "ok" : "MISMATCH", vs[i].name.c_str());
            }
        }
    }
    // per-workgroup start / end stamps of K = 4 CONJ decodes (Q6-like 2.3 % density): how much
    // of the launch is dispatch ramp and how much is the tail after the first workgroup finishes
    auto stamps = [&](const char* label, std::function<void(EvalArgs&, uint64_t*)> launch) {
        const unsigned grid = std::min<unsigned>(dtiles, 2 * cus);
        uint64_t* d_times;
        CK(hipMalloc(&d_times, 2 * grid * 8));
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_diag_times), &d_times, sizeof(d_times)));
        std::vector<uint64_t> h(2 * grid);
        std::vector<double> ramp, tail, span;
        for (int r = 0; r < rounds + 1; ++r) {
            EvalArgs a = base;
            a.num_tiles = dtiles;
            a.prog.leaf[3] = leaf[4];
            a.prog.n_leaves = 4;
            a.prog.negate = 0;
            a.prog.nops = 0;
            for (int k = 1; k < 4; ++k) a.prog.nops |= 1u << (4 * k);
            a.prog.ops = 0;
            launch(a, d_times);
            CK(hipDeviceSynchronize());
            if (r == 0) continue;
            CK(hipMemcpy(h.data(), d_times, h.size() * 8, hipMemcpyDeviceToHost));
            uint64_t s0 = ~0ull, s1 = 0, e0 = ~0ull, e1 = 0;
            for (unsigned g = 0; g < grid; ++g) {
                s0 = std::min(s0, h[2 * g]);
                s1 = std::max(s1, h[2 * g]);
                e0 = std::min(e0, h[2 * g + 1]);
                e1 = std::max(e1, h[2 * g + 1]);
            }
            ramp.push_back((s1 - s0) / 100.0);  // 100 MHz ticks → µs
            tail.push_back((e1 - e0) / 100.0);
            span.push_back((e1 - s0) / 100.0);
            if (r == rounds) {
                std::vector<double> ends;
                double xsum[8] = {0}, xmax[8] = {0};
                int xn[8] = {0};
                for (unsigned g = 0; g < grid; ++g) {
                    const double e = (h[2 * g + 1] - s0) / 100.0;
                    ends.push_back(e);
                    xsum[g % 8] += e;
                    xmax[g % 8] = std::max(xmax[g % 8], e);
                    xn[g % 8]++;
                }
                std::sort(ends.begin(), ends.end());
                printf("  [%s] end times (us from first start): p0 %.1f p10 %.1f p25 %.1f p50 %.1f p75 %.1f p90 %.1f p100 %.1f\n",
                       label, ends[0], ends[grid / 10], ends[grid / 4], ends[grid / 2], ends[3 * grid / 4],
                       ends[9 * grid / 10], ends[grid - 1]);
                printf("  [%s] per XCD mean/max end:", label);
                for (int x = 0; x < 8; ++x) printf(" %.1f/%.1f", xsum[x] / std::max(xn[x], 1), xmax[x]);
                printf("\n");
            }
        }
        auto med = [](std::vector<double> v) {
            std::sort(v.begin(), v.end());
            return v[v.size() / 2];
        };
        printf("%s per-WG stamps: start spread %.1f us, end spread %.1f us, first start -> last end %.1f us\n", label,
               med(ramp), med(tail), med(span));
        CK(hipFree(d_times));
    };
    {
        const unsigned grid = std::min<unsigned>(dtiles, 2 * cus);
        stamps("K4 pairs", [&](EvalArgs& a, uint64_t*) {
            hipLaunchKernelGGL((eval_decode_pairs<4, 2, 4096, 512, 4, FORM_CONJ>), dim3(grid), dim3(512), 0, 0, a, dir);
        });
        stamps("K4 runs", [&](EvalArgs& a, uint64_t*) {
            hipLaunchKernelGGL((eval_decode_runs<4, 2, 8192, 512, FORM_CONJ, 16, true>), dim3(grid), dim3(512), 0, 0, a,
                               dir);
        });
    }
    const double alg = 8.0 * W * 5 + 8.0 * ref_count;
    printf("%-26s %10s %10s %10s\n", "variant", "median_us", "min_us", "alg_GB/s");
    for (size_t i = 0; i < vs.size(); ++i) {
        auto t = times[i];
        std::sort(t.begin(), t.end());
        const double med = t[t.size() / 2] * 1e3, mn = t[0] * 1e3;
        printf("%-26s %10.1f %10.1f %10.0f\n", vs[i].name.c_str(), med, mn, alg / (med * 1e-6) / 1e9);
    }
    return 0;
}
