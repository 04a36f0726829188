// Dense-tile microbenchmark (development tool, not shipped): the run-claimed decode at high
// selectivity, where tiles hold more qualifying rows than an LDS stage (the dense path), with
// the dense rows staged through LDS in rounds (DSTAGE, production) vs written straight from
// each lane (the round-2 path), beside the pair-claimed kernel and a streaming floor (the same
// leaf read and the same number of ids written as one contiguous 16-byte run per tile). Also
// the zonemap shape: a leaf dense in a contiguous band of tiles and empty elsewhere, decoded
// over every tile and over the band's live-tile list. Every variant's ids are checked
// (count, sum, xor of mixed ids) against the production kernel.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-atomic-optimizer-strategy=None \
//         -I duckdb-cubit_amd/csrc scripts/densebench.hip -o scripts/densebench
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

// density thresh / 2^32 inside tiles [band0, band1) (every tile when band1 == 0), 0 elsewhere
__global__ void fill_leaf(uint64_t* w, uint64_t pw, uint64_t n_rows, uint32_t thresh, uint64_t seed, uint64_t band0,
                          uint64_t band1) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < pw; i += stride) {
        const uint64_t tile = i / 2048;
        uint64_t word = 0;
        if (band1 == 0 || (tile >= band0 && tile < band1))
            for (int b = 0; b < 64; ++b) {
                const uint64_t row = i * 64 + b;
                const uint32_t h = (uint32_t)(mix64(seed * 0x9E3779B97F4A7C15ull + row) >> 32);
                if (row < n_rows && h < thresh) word |= 1ull << b;
            }
        w[i] = word;
    }
}

__global__ void checksum(const int64_t* ids, const uint64_t* cnt, uint64_t* out) {
    const uint64_t n = *cnt;
    uint64_t s = 0, x = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        s += (uint64_t)ids[i];
        x ^= mix64((uint64_t)ids[i]);
    }
    atomicAdd(reinterpret_cast<unsigned long long*>(out), (unsigned long long)s);
    atomicXor(reinterpret_cast<unsigned long long*>(out + 1), (unsigned long long)x);
}

// the floor: the same leaf walk, then `per_tile[tile]` int64 written as one contiguous run per
// tile (offsets precomputed) with 16-byte stores — no evaluation, scan, claim or decode
__global__ __launch_bounds__(512, 4) void floor_kernel(EvalArgs a, const uint64_t* __restrict__ dir,
                                                       int64_t* __restrict__ out) {
    constexpr int THREADS = 512, PAIRS = 2;
    constexpr uint64_t TILE_WORDS = THREADS * 2 * PAIRS;
    typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
    const int t = threadIdx.x;
    u64x2 v[1][PAIRS];
    uint32_t i = blockIdx.x;
    if (i < a.num_tiles) load_tile<1, PAIRS, THREADS>(a, (uint64_t)tile_at(a, i) * TILE_WORDS, t, v);
    while (i < a.num_tiles) {
        const uint32_t tile = tile_at(a, i);
        const uint64_t x = v[0][0].x ^ v[0][1].y;
        const uint32_t next = i + gridDim.x;
        if (next < a.num_tiles) load_tile<1, PAIRS, THREADS>(a, (uint64_t)tile_at(a, next) * TILE_WORDS, t, v);
        const uint64_t start = dir[2 * tile], len = dir[2 * tile + 1];
        i64x2* o = reinterpret_cast<i64x2*>(out + (start & ~1ull));
        for (uint64_t j = t; j < (len + 1) / 2; j += THREADS) {
            i64x2 val;
            val.x = (int64_t)(x + 2 * j);
            val.y = (int64_t)(x + 2 * j + 1);
            o[j] = val;
        }
        i = next;
    }
}

struct Variant {
    std::string name;
    std::function<void(EvalArgs&, hipStream_t)> launch;
    bool check;
};

int main(int argc, char** argv) {
    const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 600037902ull;
    const int rounds = argc > 2 ? atoi(argv[2]) : 10;
    const uint64_t W = (n + 63) / 64, pw = padded_words(n);
    const uint32_t tiles = (uint32_t)(pw / decode_tile_words());
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const unsigned G = 2 * prop.multiProcessorCount;
    uint64_t* leaf;
    CK(hipMalloc(&leaf, pw * 8));
    const uint64_t cap = n + 4096;
    int64_t* ids;
    uint64_t *cnt, *dir, *ticket, *sums, *live_u64;
    uint32_t* live;
    CK(hipMalloc(&ids, cap * 8));
    CK(hipMalloc(&cnt, 64));
    CK(hipMalloc(&dir, (uint64_t)tiles * 16 + 64));
    CK(hipMalloc(&ticket, kTicketWords * 8));
    CK(hipMemset(ticket, 0, kTicketWords * 8));
    CK(hipMalloc(&sums, 16));
    CK(hipMalloc(&live, (uint64_t)tiles * 4));
    (void)live_u64;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    struct Case {
        double dens;
        uint64_t band0, band1;
    };
    // uniform densities; then the zonemap shape (12 % inside 673 tiles, the Q6 year of a
    // ship-date-clustered lineitem)
    const std::vector<Case> cases = {{0.02, 0, 0}, {0.05, 0, 0}, {0.08, 0, 0}, {0.12, 0, 0}, {0.25, 0, 0},
                                     {0.5, 0, 0},  {0.9, 0, 0},  {0.12, 1900, 2573}};
    for (const Case& cs : cases) {
        hipLaunchKernelGGL(fill_leaf, dim3(4096), dim3(256), 0, 0, leaf, pw, n, (uint32_t)(cs.dens * 4294967296.0), 7,
                           cs.band0, cs.band1);
        CK(hipDeviceSynchronize());
        EvalArgs base{};
        base.prog.leaf[0] = leaf;
        base.prog.n_leaves = 1;
        base.prog.form = FORM_CONJ;
        base.n_rows = n;
        base.n_words = W;
        base.rowids = ids;
        base.capacity = cap;
        base.count = cnt;
        base.ticket = ticket;
        base.num_tiles = tiles;
        std::vector<uint32_t> hl;
        for (uint32_t z = (uint32_t)cs.band0; z < (uint32_t)std::min<uint64_t>(cs.band1, tiles); ++z) hl.push_back(z);
        if (!hl.empty()) CK(hipMemcpy(live, hl.data(), hl.size() * 4, hipMemcpyHostToDevice));
        const unsigned grid_all = std::min<unsigned>(tiles, G);
        std::vector<Variant> vs;
        vs.push_back({"runs staged-dense (prod)", [&](EvalArgs& a, hipStream_t s) {
                          hipLaunchKernelGGL((eval_decode_runs<1, 2, 9984, 512, FORM_CONJ>), dim3(grid_all), dim3(512), 0,
                                             s, a, dir);
                      }, true});
        vs.push_back({"runs direct-dense (r02)", [&](EvalArgs& a, hipStream_t s) {
                          hipLaunchKernelGGL((eval_decode_runs<1, 2, 9984, 512, FORM_CONJ, 16, false, false>),
                                             dim3(grid_all), dim3(512), 0, s, a, dir);
                      }, true});
        vs.push_back({"pairs staged-dense (prod)", [&](EvalArgs& a, hipStream_t s) {
                          hipLaunchKernelGGL((eval_decode_pairs<1, 2, 4096, 512, 0, FORM_CONJ>), dim3(grid_all), dim3(512),
                                             0, s, a, dir);
                      }, true});
        vs.push_back({"pairs direct-dense (r02)", [&](EvalArgs& a, hipStream_t s) {
                          hipLaunchKernelGGL((eval_decode_pairs<1, 2, 4096, 512, 0, FORM_CONJ, 2, false>), dim3(grid_all),
                                             dim3(512), 0, s, a, dir);
                      }, true});
        // small partition (cfg 2 size: 768 tiles): the policy's pair kernel, one pair per workgroup
        const unsigned small_tiles = std::min<unsigned>(tiles, 768);
        vs.push_back({"pairs staged, 1e8-row prefix", [&, small_tiles](EvalArgs& a, hipStream_t s) {
                          a.num_tiles = small_tiles;
                          a.n_rows = std::min<uint64_t>(n, 100000000ull);
                          a.n_words = (a.n_rows + 63) / 64;
                          hipLaunchKernelGGL((eval_decode_pairs<1, 2, 4096, 512, 0, FORM_CONJ>), dim3(small_tiles / 2),
                                             dim3(512), 0, s, a, dir);
                      }, false});
        vs.push_back({"runs staged, 1e8-row prefix", [&, small_tiles](EvalArgs& a, hipStream_t s) {
                          a.num_tiles = small_tiles;
                          a.n_rows = std::min<uint64_t>(n, 100000000ull);
                          a.n_words = (a.n_rows + 63) / 64;
                          hipLaunchKernelGGL((eval_decode_runs<1, 2, 9984, 512, FORM_CONJ>), dim3(small_tiles / 2),
                                             dim3(512), 0, s, a, dir);
                      }, false});
        if (!hl.empty()) {
            const unsigned gl = std::min<unsigned>((unsigned)hl.size(), G);
            vs.push_back({"runs staged-dense, live list", [&, gl](EvalArgs& a, hipStream_t s) {
                              a.live = live;
                              a.num_tiles = (uint32_t)hl.size();
                              hipLaunchKernelGGL((eval_decode_runs<1, 2, 9984, 512, FORM_CONJ>), dim3(gl), dim3(512), 0, s,
                                                 a, dir);
                          }, true});
            vs.push_back({"runs direct-dense, live list", [&, gl](EvalArgs& a, hipStream_t s) {
                              a.live = live;
                              a.num_tiles = (uint32_t)hl.size();
                              hipLaunchKernelGGL((eval_decode_runs<1, 2, 9984, 512, FORM_CONJ, 16, false, false>), dim3(gl),
                                                 dim3(512), 0, s, a, dir);
                          }, true});
        }
        // reference checksum + directory for the floor
        uint64_t ref[2] = {0, 0}, ref_cnt = 0;
        std::vector<float> best(vs.size() + 1, 1e30f), sum(vs.size() + 1, 0.f);
        for (int r = 0; r < rounds; ++r) {
            for (size_t v = 0; v < vs.size(); ++v) {
                EvalArgs a = base;
                CK(hipEventRecord(e0, 0));
                vs[v].launch(a, 0);
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best[v] = std::min(best[v], ms);
                sum[v] += ms;
                if (r == 0 && vs[v].check) {
                    CK(hipMemset(sums, 0, 16));
                    hipLaunchKernelGGL(checksum, dim3(1024), dim3(256), 0, 0, ids, cnt, sums);
                    uint64_t h[2], c;
                    CK(hipMemcpy(h, sums, 16, hipMemcpyDeviceToHost));
                    CK(hipMemcpy(&c, cnt, 8, hipMemcpyDeviceToHost));
                    if (v == 0) {
                        ref[0] = h[0];
                        ref[1] = h[1];
                        ref_cnt = c;
                    } else if (h[0] != ref[0] || h[1] != ref[1] || c != ref_cnt) {
                        printf("MISMATCH %s: count %llu vs %llu\n", vs[v].name.c_str(), (unsigned long long)c,
                               (unsigned long long)ref_cnt);
                    }
                }
                if (v == 0 && r == 0) {  // production directory → the floor's contiguous runs
                    std::vector<uint64_t> d((uint64_t)tiles * 2);
                    CK(hipMemcpy(d.data(), dir, d.size() * 8, hipMemcpyDeviceToHost));
                    uint64_t off = 0;
                    for (uint32_t tt = 0; tt < tiles; ++tt) {
                        d[2 * tt] = off;
                        off += d[2 * tt + 1];
                    }
                    CK(hipMemcpy(dir + 0, d.data(), d.size() * 8, hipMemcpyHostToDevice));
                }
            }
            // floor (reads the directory rewritten above: it is not rewritten by the floor)
            EvalArgs a = base;
            CK(hipEventRecord(e0, 0));
            hipLaunchKernelGGL(floor_kernel, dim3(grid_all), dim3(512), 0, 0, a, dir, ids);
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best.back() = std::min(best.back(), ms);
            sum.back() += ms;
        }
        printf("density %.2f%s: %llu ids (%.1f MB written), leaf %.1f MB\n", cs.dens,
               cs.band1 ? " in tiles [1900, 2573)" : "", (unsigned long long)ref_cnt, ref_cnt * 8 / 1e6, W * 8 / 1e6);
        for (size_t v = 0; v <= vs.size(); ++v) {
            const double bytes = W * 8.0 + ref_cnt * 8.0;
            const double avg = sum[v] / rounds;
            printf("  %-34s best %8.1f us  mean %8.1f us  %6.2f TB/s (alg. bytes / best)\n",
                   v < vs.size() ? vs[v].name.c_str() : "floor: leaf + contiguous writes", best[v] * 1e3, avg * 1e3,
                   bytes / (best[v] * 1e-3) / 1e12);
        }
    }
    return 0;
}
