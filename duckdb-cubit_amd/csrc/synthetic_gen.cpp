// Seeded synthetic columns for the non-TPC-H configurations:
// v[i] = splitmix64(seed, row_begin + i) mod modulus, as INT32. Row-addressable so every
// partition of a multi-GPU table generates exactly its own rows.
#include <algorithm>
#include <cstdint>
#include <thread>
#include <vector>

namespace {

inline uint64_t splitmix64(uint64_t seed, uint64_t i) {
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

}  // namespace

extern "C" {

uint64_t cubit_splitmix64(uint64_t seed, uint64_t i) { return splitmix64(seed, i); }

// out[i] = splitmix64(seed, row_begin + i) % modulus, i in [0, n)
int cubit_synth_uniform_i32(uint64_t seed, uint64_t row_begin, uint64_t n, uint32_t modulus, int32_t* out,
                            int nthreads) {
    if (!out || modulus == 0) return 1;
    if (nthreads <= 0) nthreads = (int)std::max(1u, std::min(std::thread::hardware_concurrency(), 16u));
    if (n < (1u << 20)) nthreads = 1;
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) {
        const uint64_t b = n * t / nthreads, e = n * (t + 1) / nthreads;
        th.emplace_back([=] {
            for (uint64_t i = b; i < e; ++i) out[i] = (int32_t)(splitmix64(seed, row_begin + i) % modulus);
        });
    }
    for (auto& x : th) x.join();
    return 0;
}

}  // extern "C"
