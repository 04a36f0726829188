// Host-side read rate of page-locked memory the GPU just wrote (diagnostic for the table
// function's chunk fill): 8 threads widen 3-byte values (as the staged l_extendedprice) into a
// 2,048-value int64 chunk, reading (a) cubit_host_alloc memory filled by a device-to-host copy,
// (b) malloc'd memory filled by memcpy from it, (c) the page-locked memory again (now warm).
//   g++ -O3 -mavx2 -std=c++17 scripts/hostread.cpp -Iinclude -Lduckdb-cubit_amd/lib -lcubitgpu \
//       -Wl,-rpath,$PWD/duckdb-cubit_amd/lib -lpthread -o scripts/hostread
#include <immintrin.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "cubit_gpu.h"

static void widen24(const uint8_t* src, int64_t off, size_t n, int64_t* dst) {
    const __m128i shuf = _mm_setr_epi8(0, 1, 2, -1, 3, 4, 5, -1, 6, 7, 8, -1, 9, 10, 11, -1);
    const __m256i vo = _mm256_set1_epi64x(off);
    size_t k = 0;
    for (; k + 8 <= n; k += 8) {
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + 3 * k));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + 3 * k + 12));
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + k),
                            _mm256_add_epi64(vo, _mm256_cvtepu32_epi64(_mm_shuffle_epi8(a, shuf))));
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(dst + k + 4),
                            _mm256_add_epi64(vo, _mm256_cvtepu32_epi64(_mm_shuffle_epi8(b, shuf))));
    }
    for (; k < n; ++k) dst[k] = off + (int64_t)(src[3 * k] | src[3 * k + 1] << 8 | src[3 * k + 2] << 16);
}

static double run(const uint8_t* buf, size_t values, int threads, int64_t* sink) {
    std::vector<std::thread> th;
    std::vector<int64_t> sums(threads);
    const auto t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t] {
            alignas(64) int64_t chunk[2048];
            const size_t b = values * t / threads, e = values * (t + 1) / threads;
            int64_t s = 0;
            for (size_t i = b; i < e; i += 2048) {
                const size_t n = std::min<size_t>(2048, e - i);
                widen24(buf + 3 * i, 7, n, chunk);
                s += chunk[0] + chunk[n - 1];
            }
            sums[t] = s;
        });
    for (auto& x : th) x.join();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (int64_t s : sums) *sink += s;
    return ms;
}

int main(int argc, char** argv) {
    const size_t values = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 11421368;
    const int threads = argc > 2 ? std::atoi(argv[2]) : 8;
    const size_t bytes = values * 3 + 64;
    cubit_ctx* ctx = nullptr;
    if (cubit_ctx_create(0, &ctx) != CUBIT_OK) return 1;
    void *d = nullptr, *pinned = nullptr;
    if (cubit_dev_alloc(ctx, bytes, &d) || cubit_host_alloc(ctx, bytes, &pinned)) return 1;
    cubit_memset_d(ctx, d, 0x5a, bytes);
    uint8_t* plain = static_cast<uint8_t*>(std::aligned_alloc(64, (bytes + 63) / 64 * 64));
    int64_t sink = 0;
    for (int rep = 0; rep < 5; ++rep) {
        cubit_memcpy_d2h(ctx, pinned, d, bytes);  // the DMA engine writes it: the CPU caches hold none of it
        const double cold = run(static_cast<const uint8_t*>(pinned), values, threads, &sink);
        const double warm = run(static_cast<const uint8_t*>(pinned), values, threads, &sink);
        cubit_memcpy_d2h(ctx, pinned, d, bytes);
        std::memcpy(plain, pinned, bytes);
        const double mal = run(plain, values, threads, &sink);
        std::printf("hostread values %zu threads %d pinned_after_dma_ms %.3f pinned_warm_ms %.3f malloc_ms %.3f\n",
                    values, threads, cold, warm, mal);
    }
    std::printf("sink %lld\n", (long long)sink);
    cubit_host_free(ctx, pinned);
    cubit_dev_free(ctx, d);
    cubit_ctx_destroy(ctx);
    return 0;
}
