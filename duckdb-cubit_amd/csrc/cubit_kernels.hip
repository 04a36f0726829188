// CDNA4 (gfx950) kernels of the bitmap-indexed scan filter.
//
//   K1+K2  eval_decode   — postfix AND/OR/ANDNOT over K bitvectors, fused with the
//                          bitvector → ascending int64 row-id compaction (single pass,
//                          decoupled look-back across tiles). Replaces the per-vector
//                          selection narrowing of RowGroup::TemplatedScan
//                          (src/storage/table/row_group.cpp:537-550 → ColumnSegment::
//                          FilterSelection, column_segment.cpp:378-522) and the row-id
//                          synthesis start+current_row+sel[i] (row_group.cpp:573-580).
//   K0     compare_bitvector — predicate → bitvector over a raw column, the comparison
//                          semantics of TemplatedFilterSelection (column_segment.cpp:261-349).
//   K3     gather / gather_sum_product — probe columns at row ids
//                          (ColumnData::FilterScan / FetchRow, column_data.cpp:305-309,452-461).
//   K4     visibility / update_mask — MVCC delta → bitvectors
//                          (ChunkVectorInfo::TemplatedGetSelVector chunk_info.cpp:123-161,
//                           UpdateInfo::UpdatesForTransaction update_info.hpp:44-55).
//
// Bandwidth-bound integer work: no MFMA. Loads are 16 B per lane (dwordx4), a wave moves
// 1 KiB per load instruction; row ids are staged in LDS and written as contiguous runs.
#include <hip/hip_runtime.h>

#include "cubit_internal.hpp"

namespace cubit {

namespace {

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

constexpr uint64_t kFlagShift = 62;
constexpr uint64_t kFlagAggregate = 1ull << kFlagShift;
constexpr uint64_t kFlagPrefix = 2ull << kFlagShift;
constexpr uint64_t kValueMask = (1ull << kFlagShift) - 1;
constexpr uint32_t kMaxSpins = 1u << 22;

__device__ __forceinline__ uint64_t load_status(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_status(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

__device__ __forceinline__ uint64_t apply_op(int8_t op, uint64_t a, uint64_t b) {
    return op == OP_AND ? (a & b) : (op == OP_OR ? (a | b) : (a & ~b));
}

// Evaluate the program on this thread's kWordsPerThread words. Leaves are loaded by the
// caller (compile-time indexed), the stack is 4 deep and shifted with constant indices so
// it stays in VGPRs.
template <int K>
__device__ __forceinline__ void eval_words(const EvalProgram& prog, const u64x2 (&v)[K][kPairs],
                                           uint64_t (&r)[kWordsPerThread]) {
    uint64_t s0[kWordsPerThread], s1[kWordsPerThread], s2[kWordsPerThread], s3[kWordsPerThread];
#pragma unroll
    for (int j = 0; j < kWordsPerThread; ++j) s0[j] = s1[j] = s2[j] = s3[j] = 0;
    int op_i = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t neg = ((prog.negate >> k) & 1u) ? ~0ull : 0ull;
#pragma unroll
        for (int j = 0; j < kWordsPerThread; ++j) {
            s3[j] = s2[j];
            s2[j] = s1[j];
            s1[j] = s0[j];
            const u64x2 p = v[k][j >> 1];
            s0[j] = ((j & 1) ? p.y : p.x) ^ neg;
        }
        const int nops = prog.nops[k];
        for (int t = 0; t < nops; ++t) {
            const int8_t op = prog.ops[op_i++];
#pragma unroll
            for (int j = 0; j < kWordsPerThread; ++j) {
                s0[j] = apply_op(op, s1[j], s0[j]);
                s1[j] = s2[j];
                s2[j] = s3[j];
            }
        }
    }
#pragma unroll
    for (int j = 0; j < kWordsPerThread; ++j) r[j] = s0[j];
}

// One workgroup = one tile of kTileWords words (65,536 rows). Word layout inside a tile:
// pair p of thread t holds words p*512 + 2t + {0,1}, so every dwordx4 wave-load is a
// contiguous 1 KiB. Tile ids come from an atomic counter in launch order, so a tile only
// ever waits on tiles that already started (forward progress for the look-back).
template <int K, EvalMode MODE>
__global__ __launch_bounds__(kThreads) void eval_decode_kernel(EvalArgs a) {
    __shared__ uint64_t s_wave_tot[kThreads / 64];
    __shared__ uint64_t s_excl;
    __shared__ uint32_t s_tile;
    __shared__ int64_t s_stage[MODE == EvalMode::kDecode ? kStageCap : 1];

    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = t >> 6;

    if (t == 0) s_tile = atomicAdd(a.tile_counter, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    const uint64_t tile_word0 = (uint64_t)tile * kTileWords;

    // ---- load K leaves (padded: always in bounds)
    u64x2 v[K][kPairs];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const u64x2* base = reinterpret_cast<const u64x2*>(a.prog.leaf[k] + tile_word0);
#pragma unroll
        for (int p = 0; p < kPairs; ++p) v[k][p] = __builtin_nontemporal_load(base + p * kThreads + t);
    }

    // ---- evaluate + tail mask
    uint64_t r[kWordsPerThread];
    eval_words<K>(a.prog, v, r);
#pragma unroll
    for (int j = 0; j < kWordsPerThread; ++j) {
        const uint64_t gw = tile_word0 + (uint64_t)(j >> 1) * (2 * kThreads) + 2 * t + (j & 1);
        if (gw >= a.n_words) {
            r[j] = 0;
        } else if (gw == a.n_words - 1 && (a.n_rows & 63)) {
            r[j] &= (1ull << (a.n_rows & 63)) - 1;
        }
    }
    if (a.result_words) {
#pragma unroll
        for (int p = 0; p < kPairs; ++p) {
            u64x2 o;
            o.x = r[2 * p];
            o.y = r[2 * p + 1];
            reinterpret_cast<u64x2*>(a.result_words + tile_word0)[p * kThreads + t] = o;
        }
    }

    // ---- per-thread counts in tile order: pair 0 of every thread, then pair 1
    const uint64_t c0 = (uint64_t)(__popcll(r[0]) + __popcll(r[1]));
    const uint64_t c1 = (uint64_t)(__popcll(r[2]) + __popcll(r[3]));
    const uint64_t packed = c0 | (c1 << 32);
    const uint64_t incl = wave_incl_scan(packed, lane);
    if (lane == 63) s_wave_tot[wave] = incl;
    __syncthreads();
    uint64_t wave_prefix = 0, block_tot = 0;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) {
        const uint64_t x = s_wave_tot[w];
        if (w < wave) wave_prefix += x;
        block_tot += x;
    }
    const uint64_t excl_packed = wave_prefix + incl - packed;
    const uint64_t tot0 = block_tot & 0xffffffffull, tot1 = block_tot >> 32;
    const uint64_t tile_count = tot0 + tot1;

    if (MODE == EvalMode::kCount) {
        if (t == 0 && tile_count) atomicAdd(reinterpret_cast<unsigned long long*>(a.count), tile_count);
        return;
    }

    // ---- decoupled look-back (wave 0). Status words are 8-byte {flag, value} granules
    // written by one agent-scope store: the data is the flag (MI355X guide R2).
    if (wave == 0) {
        uint64_t excl = 0;
        if (tile == 0) {
            if (lane == 0) store_status(&a.tile_status[0], kFlagPrefix | tile_count);
        } else {
            if (lane == 0) store_status(&a.tile_status[tile], kFlagAggregate | tile_count);
            int64_t base = (int64_t)tile - 1;
            uint32_t spins = 0;
            for (;;) {
                const int64_t idx = base - lane;
                const uint64_t s = idx >= 0 ? load_status(&a.tile_status[idx]) : kFlagPrefix;
                const uint64_t flag = s >> kFlagShift;
                const uint64_t pmask = __ballot(flag == 2);
                const uint64_t imask = __ballot(flag == 0);
                const uint64_t win = pmask ? ((pmask & (~pmask + 1)) << 1) - 1 : ~0ull;
                if (imask & win) {
                    if (++spins > kMaxSpins) {
                        if (lane == 0) atomicOr(a.error_flag, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += wave_sum(((win >> lane) & 1ull) ? (s & kValueMask) : 0ull);
                if (pmask) break;
                base -= 64;
            }
            if (lane == 0) store_status(&a.tile_status[tile], kFlagPrefix | (excl + tile_count));
        }
        if (lane == 0) s_excl = excl;
    }
    __syncthreads();
    const uint64_t tile_off = s_excl;
    if (t == 0 && tile == a.num_tiles - 1) *a.count = tile_off + tile_count;
    if (tile_count == 0 || a.rowids == nullptr) return;

    // ---- decode: thread-local ascending runs, staged in LDS when the tile fits
    const bool stage = tile_count <= (uint64_t)kStageCap;
    const int64_t row0 = a.row_base + (int64_t)(tile_word0 * 64);
#pragma unroll
    for (int p = 0; p < kPairs; ++p) {
        uint64_t off = p == 0 ? (excl_packed & 0xffffffffull) : tot0 + (excl_packed >> 32);
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            uint64_t w = r[2 * p + e];
            const int64_t wrow = row0 + (int64_t)((p * 2 * kThreads + 2 * t + e) * 64);
            while (w) {
                const int b = __builtin_ctzll(w);
                const int64_t rid = wrow + b;
                if (stage) {
                    s_stage[off] = rid;
                } else {
                    const uint64_t g = tile_off + off;
                    if (g < a.capacity) a.rowids[g] = rid;
                }
                ++off;
                w &= w - 1;
            }
        }
    }
    if (stage) {
        __syncthreads();
        for (uint64_t i = t; i < tile_count; i += kThreads) {
            const uint64_t g = tile_off + i;
            if (g < a.capacity) a.rowids[g] = s_stage[i];
        }
    }
}

template <int K>
hipError_t launch_eval_k(const EvalArgs& a, EvalMode mode, hipStream_t stream) {
    const dim3 grid(a.num_tiles), block(kThreads);
    if (mode == EvalMode::kDecode)
        hipLaunchKernelGGL((eval_decode_kernel<K, EvalMode::kDecode>), grid, block, 0, stream, a);
    else
        hipLaunchKernelGGL((eval_decode_kernel<K, EvalMode::kCount>), grid, block, 0, stream, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------ K0: compare → bitvector

template <int CMP>
__device__ __forceinline__ bool cmp_op(int64_t v, int64_t c) {
    if (CMP == 0) return v == c;
    if (CMP == 1) return v != c;
    if (CMP == 2) return v < c;
    if (CMP == 3) return v <= c;
    if (CMP == 4) return v > c;
    return v >= c;
}

// Each wave produces 64 consecutive words: for word j every lane tests one row and the
// ballot is the word; lane j keeps it, then the wave stores 512 contiguous bytes.
template <typename T, int CMP>
__global__ __launch_bounds__(256) void compare_bitvector_kernel(const T* __restrict__ col,
                                                                const uint64_t* __restrict__ validity,
                                                                uint64_t n_rows, uint64_t n_words_padded,
                                                                int64_t c, uint64_t* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const uint64_t wave_id = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t n_waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t w0 = wave_id * 64; w0 < n_words_padded; w0 += n_waves * 64) {
        uint64_t mine = 0;
        for (int j = 0; j < 64; ++j) {
            const uint64_t row = (w0 + j) * 64 + lane;
            bool p = false;
            if (row < n_rows) {
                const bool valid = validity ? ((validity[w0 + j] >> lane) & 1ull) : true;
                p = valid && cmp_op<CMP>((int64_t)col[row], c);
            }
            const uint64_t b = __ballot(p);
            if (lane == j) mine = b;
        }
        out[w0 + lane] = mine;
    }
}

template <typename T>
hipError_t launch_compare_t(const T* col, const uint64_t* validity, uint64_t n_rows, int cmp, int64_t c,
                            uint64_t* out, hipStream_t stream) {
    const uint64_t nw = padded_words(n_rows);
    const uint64_t waves = nw / 64;
    const uint64_t blocks = std::min<uint64_t>((waves + 3) / 4, 8192);
    const dim3 grid((unsigned)std::max<uint64_t>(blocks, 1)), block(256);
    switch (cmp) {
    case 0: hipLaunchKernelGGL((compare_bitvector_kernel<T, 0>), grid, block, 0, stream, col, validity, n_rows, nw, c, out); break;
    case 1: hipLaunchKernelGGL((compare_bitvector_kernel<T, 1>), grid, block, 0, stream, col, validity, n_rows, nw, c, out); break;
    case 2: hipLaunchKernelGGL((compare_bitvector_kernel<T, 2>), grid, block, 0, stream, col, validity, n_rows, nw, c, out); break;
    case 3: hipLaunchKernelGGL((compare_bitvector_kernel<T, 3>), grid, block, 0, stream, col, validity, n_rows, nw, c, out); break;
    case 4: hipLaunchKernelGGL((compare_bitvector_kernel<T, 4>), grid, block, 0, stream, col, validity, n_rows, nw, c, out); break;
    case 5: hipLaunchKernelGGL((compare_bitvector_kernel<T, 5>), grid, block, 0, stream, col, validity, n_rows, nw, c, out); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------ K3: probe

template <typename T>
__global__ __launch_bounds__(256) void gather_kernel(const T* __restrict__ col, const int64_t* __restrict__ rowids,
                                                     const uint64_t* __restrict__ d_count, uint64_t max_n,
                                                     int64_t row_base, int64_t* __restrict__ out) {
    const uint64_t n = min(*d_count, max_n);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = (int64_t)col[rowids[i] - row_base];
}

__global__ __launch_bounds__(256) void gather_sum_product_kernel(const int64_t* __restrict__ x,
                                                                 const int64_t* __restrict__ y,
                                                                 const int64_t* __restrict__ rowids,
                                                                 const uint64_t* __restrict__ d_count, uint64_t max_n,
                                                                 int64_t row_base, int64_t* __restrict__ partials) {
    __shared__ __int128 s_part[4];
    const uint64_t n = min(*d_count, max_n);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    __int128 acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const int64_t r = rowids[i] - row_base;
        acc += (__int128)x[r] * (__int128)y[r];
    }
    // wave reduce on the two halves
    uint64_t lo = (uint64_t)acc;
    int64_t hi = (int64_t)(acc >> 64);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t olo = __shfl_xor(lo, d, 64);
        const int64_t ohi = __shfl_xor(hi, d, 64);
        const uint64_t nlo = lo + olo;
        hi = hi + ohi + (nlo < lo ? 1 : 0);
        lo = nlo;
    }
    if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = ((__int128)hi << 64) | lo;
    __syncthreads();
    if (threadIdx.x == 0) {
        __int128 s = s_part[0] + s_part[1] + s_part[2] + s_part[3];
        partials[2 * blockIdx.x] = (int64_t)(uint64_t)s;
        partials[2 * blockIdx.x + 1] = (int64_t)(s >> 64);
    }
}

__global__ __launch_bounds__(64) void sum_partials_kernel(const int64_t* __restrict__ partials, int nblocks,
                                                          int64_t* __restrict__ out) {
    if (threadIdx.x != 0) return;
    __int128 s = 0;
    for (int b = 0; b < nblocks; ++b)
        s += ((__int128)partials[2 * b + 1] << 64) | (unsigned __int128)(uint64_t)partials[2 * b];
    out[0] = (int64_t)(uint64_t)s;
    out[1] = (int64_t)(s >> 64);
}

// ------------------------------------------------------------------ K4: MVCC

__global__ __launch_bounds__(256) void fill_valid_kernel(uint64_t* __restrict__ words, uint64_t n_rows,
                                                         uint64_t n_words_padded) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t full = n_rows / 64;
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < n_words_padded; w += stride) {
        uint64_t v = 0;
        if (w < full) v = ~0ull;
        else if (w == full && (n_rows & 63)) v = (1ull << (n_rows & 63)) - 1;
        words[w] = v;
    }
}

// A delete is in effect for the reader when UseInsertedVersion(start, tid, delete_id)
// (chunk_info.cpp:11-19): clear that row.
__global__ __launch_bounds__(256) void visibility_kernel(const int64_t* __restrict__ rows,
                                                         const uint64_t* __restrict__ ids, uint64_t n,
                                                         uint64_t start_time, uint64_t tid,
                                                         uint64_t* __restrict__ words) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t id = ids[i];
        if (id < start_time || id == tid) {
            const uint64_t r = (uint64_t)rows[i];
            atomicAnd(reinterpret_cast<unsigned long long*>(&words[r >> 6]), ~(1ull << (r & 63)));
        }
    }
}

__global__ __launch_bounds__(256) void update_mask_kernel(const int64_t* __restrict__ rows,
                                                          const uint64_t* __restrict__ versions, uint64_t n,
                                                          uint64_t start_time, uint64_t tid,
                                                          uint64_t* __restrict__ mask) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint64_t v = versions[i];
        if (v < start_time || v == tid) {
            const uint64_t r = (uint64_t)rows[i];
            atomicOr(reinterpret_cast<unsigned long long*>(&mask[r >> 6]), 1ull << (r & 63));
        }
    }
}

unsigned grid_for(uint64_t n, unsigned cap = 4096) {
    const uint64_t b = (n + 255) / 256;
    return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(b, cap));
}

}  // namespace

hipError_t launch_eval(const EvalArgs& a, EvalMode mode, hipStream_t stream) {
    switch (a.prog.n_leaves) {
    case 1: return launch_eval_k<1>(a, mode, stream);
    case 2: return launch_eval_k<2>(a, mode, stream);
    case 3: return launch_eval_k<3>(a, mode, stream);
    case 4: return launch_eval_k<4>(a, mode, stream);
    case 5: return launch_eval_k<5>(a, mode, stream);
    case 6: return launch_eval_k<6>(a, mode, stream);
    case 7: return launch_eval_k<7>(a, mode, stream);
    case 8: return launch_eval_k<8>(a, mode, stream);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_compare_bitvector(const void* col, int type, const uint64_t* validity, uint64_t n_rows, int cmp,
                                    int64_t constant, uint64_t* out_words, hipStream_t stream) {
    if (type == 0)
        return launch_compare_t<int32_t>(static_cast<const int32_t*>(col), validity, n_rows, cmp, constant, out_words,
                                         stream);
    return launch_compare_t<int64_t>(static_cast<const int64_t*>(col), validity, n_rows, cmp, constant, out_words,
                                     stream);
}

hipError_t launch_gather(const void* col, int type, const int64_t* rowids, const uint64_t* d_count, uint64_t max_n,
                         int64_t row_base, int64_t* out, hipStream_t stream) {
    const dim3 grid(grid_for(max_n, 8192)), block(256);
    if (type == 0)
        hipLaunchKernelGGL(gather_kernel<int32_t>, grid, block, 0, stream, static_cast<const int32_t*>(col), rowids,
                           d_count, max_n, row_base, out);
    else
        hipLaunchKernelGGL(gather_kernel<int64_t>, grid, block, 0, stream, static_cast<const int64_t*>(col), rowids,
                           d_count, max_n, row_base, out);
    return hipGetLastError();
}

hipError_t launch_gather_sum_product(const int64_t* x, const int64_t* y, const int64_t* rowids,
                                     const uint64_t* d_count, uint64_t max_n, int64_t row_base, int64_t* partials,
                                     int64_t* out, hipStream_t stream) {
    hipLaunchKernelGGL(gather_sum_product_kernel, dim3(kSumBlocks), dim3(256), 0, stream, x, y, rowids, d_count, max_n,
                       row_base, partials);
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(64), 0, stream, partials, kSumBlocks, out);
    return hipGetLastError();
}

hipError_t launch_fill_valid(uint64_t* words, uint64_t n_rows, hipStream_t stream) {
    const uint64_t nw = padded_words(n_rows);
    hipLaunchKernelGGL(fill_valid_kernel, dim3(grid_for(nw)), dim3(256), 0, stream, words, n_rows, nw);
    return hipGetLastError();
}

hipError_t launch_visibility(const int64_t* del_rows, const uint64_t* del_ids, uint64_t n_del, uint64_t n_rows,
                             uint64_t start_time, uint64_t transaction_id, uint64_t* words, hipStream_t stream) {
    hipError_t e = launch_fill_valid(words, n_rows, stream);
    if (e != hipSuccess || n_del == 0) return e;
    hipLaunchKernelGGL(visibility_kernel, dim3(grid_for(n_del)), dim3(256), 0, stream, del_rows, del_ids, n_del,
                       start_time, transaction_id, words);
    return hipGetLastError();
}

hipError_t launch_update_mask(const int64_t* upd_rows, const uint64_t* upd_versions, uint64_t n_upd,
                              uint64_t start_time, uint64_t transaction_id, uint64_t* mask, hipStream_t stream) {
    if (n_upd == 0) return hipSuccess;
    hipLaunchKernelGGL(update_mask_kernel, dim3(grid_for(n_upd)), dim3(256), 0, stream, upd_rows, upd_versions, n_upd,
                       start_time, transaction_id, mask);
    return hipGetLastError();
}

}  // namespace cubit
