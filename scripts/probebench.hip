// Probe microbenchmark (development tool, not shipped): where the time of the fused Q6
// aggregate (eval_sum_product: evaluate + gather l_extendedprice at the qualifying rows +
// l_discount decoded from its index) goes, at SF100 size with Q6's density, against
//   * the leaf stream alone (count kernel over the same K + M leaves),
//   * the random gather alone (the same rows' values summed from precomputed row ids, U loads
//     in flight per thread), and the number of distinct 64-byte sectors those gathers touch —
//     the line-granular floor of a probe at ~2 % density.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-atomic-optimizer-strategy=None \
//         -I duckdb-cubit_amd/csrc scripts/probebench.hip -o scripts/probebench
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

__global__ void fill_values(int64_t* v, uint64_t n, uint64_t seed, uint64_t mod) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        v[i] = (int64_t)(mix64(seed + i) % mod);
}

// sum of a[ids[i]] over i < n: U gathers in flight per thread (nontemporal, like the probes)
template <int U>
__global__ __launch_bounds__(256) void gather_sum(const int64_t* __restrict__ a, const int64_t* __restrict__ ids,
                                                  uint64_t n, unsigned long long* out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += U * stride) {
        int64_t r[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + u * stride;
            r[u] = j < n ? __builtin_nontemporal_load(ids + j) : -1;
        }
        int64_t v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = r[u] >= 0 ? __builtin_nontemporal_load(a + r[u]) : 0;
#pragma unroll
        for (int u = 0; u < U; ++u) acc += (uint64_t)v[u];
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)acc);
}

__global__ void iota_ids(int64_t* ids, uint64_t m, uint64_t stride) {
    const uint64_t st = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += st) ids[i] = (int64_t)(i * stride);
}

// contiguous read of a column, 16 B per lane (the streaming rate the gathers compare with)
__global__ __launch_bounds__(256) void stream_sum(const int64_t* __restrict__ a, uint64_t n, unsigned long long* out) {
    typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
    const i64x2* p = reinterpret_cast<const i64x2*>(a);
    const uint64_t m = n / 2, st = (uint64_t)gridDim.x * blockDim.x;
    uint64_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += 4 * st) {
        i64x2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = i + u * st < m ? __builtin_nontemporal_load(p + i + u * st) : i64x2{0, 0};
#pragma unroll
        for (int u = 0; u < 4; ++u) acc += (uint64_t)(v[u].x + v[u].y);
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)acc);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    CK(hipSetDevice(0));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const uint64_t n = 600037902, W = (n + 63) / 64, pw = padded_words(n);
    hipStream_t s;
    CK(hipStreamCreate(&s));
    // K = 4 filter leaves at Q6's density (≈ 1.9 % kept) + M = 2 decode leaves (b = 5 + [¬L6] + [¬L7])
    std::vector<uint64_t*> leaf(6);
    for (int k = 0; k < 6; ++k) {
        CK(hipMalloc(&leaf[k], pw * 8));
        hipLaunchKernelGGL(fill_leaf, dim3(4096), dim3(256), 0, s, leaf[k], pw, n,
                           (uint32_t)((k < 4 ? 0.372 : 0.5) * 4294967296.0), (uint64_t)(k + 11));
    }
    int64_t *a, *b;
    CK(hipMalloc(&a, n * 8));
    CK(hipMalloc(&b, n * 8));
    hipLaunchKernelGGL(fill_values, dim3(4096), dim3(256), 0, s, a, n, 77ull, 10494951ull);
    hipLaunchKernelGGL(fill_values, dim3(4096), dim3(256), 0, s, b, n, 99ull, 11ull);
    uint64_t *ticket, *cnt, *dir;
    CK(hipMalloc(&ticket, kTicketWords * 8));
    CK(hipMemset(ticket, 0, kTicketWords * 8));
    CK(hipMalloc(&cnt, 16));
    const uint32_t tiles = (uint32_t)((W + 2047) / 2048);
    CK(hipMalloc(&dir, 2ull * tiles * 8));
    const uint64_t cap = n / 16;
    int64_t *ids, *ordered, *partials, *out;
    CK(hipMalloc(&ids, cap * 8));
    CK(hipMalloc(&ordered, cap * 8));
    CK(hipMalloc(&partials, 2 * kSumBlocks * 8));
    CK(hipMalloc(&out, 16));
    unsigned long long* gsum;
    CK(hipMalloc(&gsum, 8));
    EvalArgs base{};
    for (int k = 0; k < 4; ++k) base.prog.leaf[k] = leaf[k];
    base.prog.n_leaves = 4;
    base.prog.form = FORM_CONJ;
    base.n_rows = n;
    base.n_words = W;
    base.rowids = ids;
    base.capacity = cap;
    base.count = cnt;
    base.num_tiles = tiles;
    base.ticket = ticket;
    const unsigned dgrid = 2 * cus;
    // the rows once, for the gather-only variants and the sector count
    CK(launch_eval_decode(base, dir, dgrid, s, nullptr, nullptr, 2, cus));
    CK(launch_order_runs(dir, tiles, nullptr, ids, cap, ordered, s));
    CK(hipStreamSynchronize(s));
    uint64_t q = 0;
    CK(hipMemcpy(&q, cnt, 8, hipMemcpyDeviceToHost));
    std::vector<int64_t> h(q);
    CK(hipMemcpy(h.data(), ordered, q * 8, hipMemcpyDeviceToHost));
    uint64_t sectors64 = 0, sectors32 = 0, lines128 = 0;
    for (uint64_t i = 0; i < q; ++i) {
        if (i == 0 || (h[i] >> 3) != (h[i - 1] >> 3)) ++sectors64;
        if (i == 0 || (h[i] >> 2) != (h[i - 1] >> 2)) ++sectors32;
        if (i == 0 || (h[i] >> 4) != (h[i - 1] >> 4)) ++lines128;
    }
    printf("rows %llu, qualifying %llu (%.2f %%); distinct sectors of the int64 column touched: 32 B %llu (%.0f MB), "
           "64 B %llu (%.0f MB), 128 B lines %llu (%.0f MB); logical probe bytes %.0f MB\n",
           (unsigned long long)n, (unsigned long long)q, 100.0 * q / n, (unsigned long long)sectors32,
           sectors32 * 32 / 1e6, (unsigned long long)sectors64, sectors64 * 64 / 1e6, (unsigned long long)lines128,
           lines128 * 128 / 1e6, q * 8 / 1e6);
    SumArgs sa{};
    sa.a = a;
    sa.partials = partials;
    sa.v0 = 5;
    sa.n_decode = 2;
    sa.dleaf[0] = leaf[4];
    sa.dleaf[1] = leaf[5];
    sa.delta[0] = 1;
    sa.delta[1] = 1;
    SumArgs sg = sa;
    sg.b = b;
    sg.n_decode = 0;
    const unsigned sgrid = sum_product_grid(cus);
    struct V {
        std::string name;
        std::function<void()> f;
        double bytes;  // algorithmic
    };
    const double leaf_b = 8.0 * W;
    std::vector<V> vs = {
        {"fused sum, b decoded (production)", [&] { CK(launch_eval_sum_product(base, sa, sgrid, out, s)); },
         6 * leaf_b + 8.0 * q},
        {"fused sum, b gathered", [&] { CK(launch_eval_sum_product(base, sg, sgrid, out, s)); }, 4 * leaf_b + 16.0 * q},
        {"leaf stream: count over 6 leaves", [&] {
             EvalArgs c = base;
             for (int k = 0; k < 6; ++k) c.prog.leaf[k] = leaf[k];
             c.prog.n_leaves = 6;
             c.num_tiles = (uint32_t)(pw / count_tile_words(6));
             CK(launch_eval_count(c, s));
         }, 6 * leaf_b},
        {"gather a only, ordered ids, U=1", [&] {
             hipLaunchKernelGGL(gather_sum<1>, dim3(2048), dim3(256), 0, s, a, ordered, q, gsum);
         }, 16.0 * q},
        {"gather a only, ordered ids, U=4", [&] {
             hipLaunchKernelGGL(gather_sum<4>, dim3(2048), dim3(256), 0, s, a, ordered, q, gsum);
         }, 16.0 * q},
        {"gather a only, ordered ids, U=8", [&] {
             hipLaunchKernelGGL(gather_sum<8>, dim3(2048), dim3(256), 0, s, a, ordered, q, gsum);
         }, 16.0 * q},
        {"unfused: decode + gather_sum_product", [&] {
             CK(launch_eval_decode(base, dir, dgrid, s, nullptr, nullptr, 0, cus));
             CK(launch_gather_sum_product(a, b, ids, cnt, cap, 0, partials, out, s));
         }, 4 * leaf_b + 8.0 * q + 24.0 * q},
    };
    // fetch-granularity calibration: one gather per 128-B line (every 16th int64) and one per
    // two lines (every 32nd), against the contiguous read of the whole column
    vs.push_back({"calib: stream the whole column a", [&] {
                      hipLaunchKernelGGL(stream_sum, dim3(4096), dim3(256), 0, s, a, n, gsum);
                  }, 8.0 * n});
    vs.push_back({"calib: gather every 16th row (1/line)", [&] {
                      hipLaunchKernelGGL(gather_sum<4>, dim3(2048), dim3(256), 0, s, a, ids, n / 16, gsum);
                  }, 8.0 * (n / 16)});
    vs.push_back({"calib: gather every 32nd row (1/2 lines)", [&] {
                      hipLaunchKernelGGL(gather_sum<4>, dim3(2048), dim3(256), 0, s, a, ordered, n / 32, gsum);
                  }, 8.0 * (n / 32)});
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("%-40s %10s %12s %10s %12s\n", "variant", "us", "alg GB/s", "frac", "w/ sectors");
    bool calib_ids = false;
    for (auto& v : vs) {
        if (!calib_ids && v.name.rfind("calib:", 0) == 0) {
            hipLaunchKernelGGL(iota_ids, dim3(4096), dim3(256), 0, s, ids, n / 16, 16ull);
            hipLaunchKernelGGL(iota_ids, dim3(4096), dim3(256), 0, s, ordered, n / 32, 32ull);
            calib_ids = true;
        }
        for (int i = 0; i < 3; ++i) v.f();
        std::vector<float> t;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0, s));
            for (int i = 0; i < reps; ++i) v.f();
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t.push_back(ms * 1e3f / reps);
        }
        std::sort(t.begin(), t.end());
        const double us = t[t.size() / 2];
        // bytes when every gathered value costs its 64-byte sector (the leaf / id streams at
        // their size): what the HBM moves at this density
        const double gathered = v.name.find("gather a only") != std::string::npos ? 1.0
                                : v.name.find("unfused") != std::string::npos  ? 2.0
                                : v.name.find("b gathered") != std::string::npos ? 2.0 : 1.0;
        const double sect = (v.name.find("count") != std::string::npos || v.name.rfind("calib:", 0) == 0)
                                ? v.bytes
                                : v.bytes - gathered * 8.0 * q + gathered * 64.0 * sectors64;
        printf("%-40s %10.1f %12.0f %10.3f %12.0f\n", v.name.c_str(), us, v.bytes / (us * 1e-6) / 1e9,
               v.bytes / (us * 1e-6) / 8e12, sect / (us * 1e-6) / 1e9);
    }
    return 0;
}
