// CDNA4 (gfx950) kernels of the bitmap-indexed scan filter.
//
//   K1+K2  eval_decode_pairs — AND/OR/ANDNOT over K bitvectors fused with the
//                          bitvector → int64 row-id compaction. Replaces the per-vector
//                          selection narrowing of RowGroup::TemplatedScan
//                          (src/storage/table/row_group.cpp:537-550 → ColumnSegment::
//                          FilterSelection, column_segment.cpp:378-522) and the row-id
//                          synthesis start+current_row+sel[i] (row_group.cpp:573-580).
//          eval_count_kernel — the same evaluation for count(*) / bitvector materialisation.
//          order_* — optional pass that lays the per-tile runs out in row order.
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
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "../../include/cubit_gpu.h"
#include "cubit_internal.hpp"

namespace cubit {

namespace {

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x, int lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

// Inclusive wave64 prefix sum of a uint32 with DPP (GFX9 row shifts, then row_bcast:15 / :31
// across the four 16-lane rows): six v_add with a DPP operand, no LDS traffic (the 64-bit
// __shfl_up scan above is twelve ds_bpermute). Lanes whose DPP source is outside the row, and
// rows outside row_mask, add `old` = 0.
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
    return x;
}

// Sum over the wave of values below 2^41 (look-back counts): two DPP scans of 24-bit low and high
// parts, the totals read from lane 63 — no ds_bpermute round trips. Every lane must be active.
__device__ __forceinline__ uint64_t wave_sum_flags(uint64_t x) {
    const uint32_t lo = wave_incl_scan32((uint32_t)x & 0xffffffu);
    const uint32_t hi = wave_incl_scan32((uint32_t)(x >> 24));
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, 63) << 24) +
           (uint32_t)__builtin_amdgcn_readlane((int)lo, 63);
}

__device__ __forceinline__ uint64_t wave_sum(uint64_t x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

// Claim-ticket layout (kTicketWords words, context-owned, zero between launches): word 0 =
// running claim counter; word kTicketStride·(1+g) = arrivals of workgroup group g
// (blockIdx % 8, one group per XCD under round-robin dispatch); word kTicketStride·9 =
// arrived groups. Counters sit 512 B apart: atomics on one line serialise (≈88/µs,
// MI355X_MICROARCH.md "dequeue"), and a flat arrival counter put a 512-atomic tail on
// every launch.
//
// finish_ticket is called by thread 0 of every workgroup after its last claim has RETURNED
// (every claim is a returning atomic whose value the caller consumed, so it is performed
// before the arrival is issued). `mine` = the rows this workgroup contributed. An arrival
// carries them: counter += (1 << kArriveShift) | mine, so the arrival count sits in the top
// 16 bits and the running row sum in the low 48. The last workgroup of a group adds the
// group's sum to the top counter; the last group holds the grand total in the value its
// returning atomic gave back, publishes it to *count and re-arms the ticket for the next
// launch on the stream (stream order guarantees that launch sees the zeroes). Two dependent
// atomics from the last arrival to the count, and no kernel has to claim on the running
// counter (word 0) just to be counted: count(*) and the fused sum only arrive.
// No __threadfence(): an agent-scope release on gfx950 writes back L2 (measured +18 µs on
// the decode); only the atomics need ordering, and they are coherent on their own.
constexpr int kArriveShift = 48;
__device__ __forceinline__ void finish_ticket(uint64_t* ticket, uint64_t* count, uint64_t mine) {
    constexpr unsigned long long kArrive = 1ull << kArriveShift, kValue = kArrive - 1;
    const uint32_t G = gridDim.x;
    const uint32_t groups = G < kTicketGroups ? G : kTicketGroups;
    const uint32_t g = blockIdx.x % groups;
    const uint32_t members = G / groups + (g < G % groups ? 1u : 0u);
    unsigned long long* gc = reinterpret_cast<unsigned long long*>(ticket + kTicketStride * (1 + g));
    const unsigned long long og = atomicAdd(gc, kArrive | (unsigned long long)mine);
    if ((og >> kArriveShift) != (unsigned long long)(members - 1)) return;
    const unsigned long long group_sum = (og & kValue) + mine;
    unsigned long long* top = reinterpret_cast<unsigned long long*>(ticket + kTicketStride * (1 + kTicketGroups));
    const unsigned long long ot = atomicAdd(top, kArrive | group_sum);
    if ((ot >> kArriveShift) != (unsigned long long)(groups - 1)) return;
    *count = (ot & kValue) + group_sum;
    atomicExch(reinterpret_cast<unsigned long long*>(ticket), 0ull);
    for (uint32_t i = 0; i < groups; ++i)
        atomicExch(reinterpret_cast<unsigned long long*>(ticket + kTicketStride * (1 + i)), 0ull);
    atomicExch(top, 0ull);
}

__device__ __forceinline__ uint64_t apply_op(uint32_t op, uint64_t a, uint64_t b) {
    return op == OP_AND ? (a & b) : (op == OP_OR ? (a | b) : (a & ~b));
}

// Evaluate the program on NW words per thread. Leaves are loaded by the caller
// (compile-time indexed); the stack is 4 deep and shifted with constant indices so it stays
// in VGPRs.
// FORM (template): FORM_POSTFIX interprets the postfix program; FORM_CONJ = AND of the
// (possibly complemented) leaves; FORM_DNF = OR over groups of AND-ed literals; FORM_CNF =
// AND over groups of OR-ed literals. The last three are branch-free on the data.
template <int K, int NW, int FORM = FORM_POSTFIX>
__device__ __forceinline__ void eval_words(const EvalProgram& prog, const u64x2 (&v)[K][NW / 2],
                                           uint64_t (&r)[NW]) {
    if (FORM == FORM_CONJ) {
        // leaf 0 initialises r; each complemented leaf is a uniform branch, so a word costs
        // one AND (or AND-NOT, v_bfi_b32) per 32 bits instead of an XOR and an AND
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if ((prog.negate >> k) & 1u) {
#pragma unroll
                for (int j = 0; j < NW; ++j) {
                    const uint64_t x = (j & 1) ? v[k][j >> 1].y : v[k][j >> 1].x;
                    r[j] = k == 0 ? ~x : (r[j] & ~x);
                }
            } else {
#pragma unroll
                for (int j = 0; j < NW; ++j) {
                    const uint64_t x = (j & 1) ? v[k][j >> 1].y : v[k][j >> 1].x;
                    r[j] = k == 0 ? x : (r[j] & x);
                }
            }
        }
        return;
    }
    if (FORM == FORM_DNF || FORM == FORM_CNF) {
        constexpr bool DNF = FORM == FORM_DNF;
        uint64_t cur[NW];
#pragma unroll
        for (int j = 0; j < NW; ++j) r[j] = DNF ? 0ull : ~0ull;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t neg = ((prog.negate >> k) & 1u) ? ~0ull : 0ull;
            const bool opens = k == 0 || ((prog.gstart >> k) & 1u);
#pragma unroll
            for (int j = 0; j < NW; ++j) {
                const u64x2 p = v[k][j >> 1];
                const uint64_t x = ((j & 1) ? p.y : p.x) ^ neg;
                if (k == 0) {
                    cur[j] = x;
                } else if (opens) {
                    r[j] = DNF ? (r[j] | cur[j]) : (r[j] & cur[j]);
                    cur[j] = x;
                } else {
                    cur[j] = DNF ? (cur[j] & x) : (cur[j] | x);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < NW; ++j) r[j] = DNF ? (r[j] | cur[j]) : (r[j] & cur[j]);
        return;
    }
    uint64_t s0[NW], s1[NW], s2[NW], s3[NW];
#pragma unroll
    for (int j = 0; j < NW; ++j) s0[j] = s1[j] = s2[j] = s3[j] = 0;
    int op_i = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const uint64_t neg = ((prog.negate >> k) & 1u) ? ~0ull : 0ull;
#pragma unroll
        for (int j = 0; j < NW; ++j) {
            s3[j] = s2[j];
            s2[j] = s1[j];
            s1[j] = s0[j];
            const u64x2 p = v[k][j >> 1];
            s0[j] = ((j & 1) ? p.y : p.x) ^ neg;
        }
        const int nops = (int)((prog.nops >> (4 * k)) & 15u);
        for (int t = 0; t < nops; ++t) {
            const uint32_t op = (prog.ops >> (2 * op_i++)) & 3u;
#pragma unroll
            for (int j = 0; j < NW; ++j) {
                s0[j] = apply_op(op, s1[j], s0[j]);
                s1[j] = s2[j];
                s2[j] = s3[j];
            }
        }
    }
#pragma unroll
    for (int j = 0; j < NW; ++j) r[j] = s0[j];
}

// Word j of a thread in a tile: pair p = j/2 holds words p·2·THREADS + 2t + {0,1}, so every
// dwordx4 wave-load reads a contiguous 1 KiB.
template <int THREADS>
__device__ __forceinline__ uint64_t word_index(uint64_t tile_word0, int j, int t) {
    return tile_word0 + (uint64_t)(j >> 1) * (2 * THREADS) + 2 * t + (j & 1);
}

template <int NW, int THREADS>
__device__ __forceinline__ void tail_mask(const EvalArgs& a, uint64_t tile_word0, int t, uint64_t (&r)[NW]) {
    // uniform: only the tile that holds the last word (or lies past it) has bits to clear
    if (tile_word0 + (uint64_t)THREADS * NW < a.n_words) return;
#pragma unroll
    for (int j = 0; j < NW; ++j) {
        const uint64_t gw = word_index<THREADS>(tile_word0, j, t);
        if (gw >= a.n_words) r[j] = 0;
        else if (gw == a.n_words - 1 && (a.n_rows & 63)) r[j] &= (1ull << (a.n_rows & 63)) - 1;
    }
}

// A tile's result words (materialised subtrees, narrowing masks). SAUX >= 0: buffer stores with
// those cache-policy bits through a descriptor over the tile (tile_word0 is uniform), as the
// decode's copy-out (emit_ids); SAUX < 0: plain stores.
template <int PAIRS, int THREADS, int SAUX = -1>
__device__ __forceinline__ void store_words(uint64_t* out, uint64_t tile_word0, int t, const uint64_t (&r)[2 * PAIRS]) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    if (SAUX >= 0) {
        const uint64_t tw = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(tile_word0 >> 32)) << 32) |
                            (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)tile_word0);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(out + tw), (short)0, PAIRS * THREADS * 16, 0x00020000);
#pragma unroll
        for (int p = 0; p < PAIRS; ++p) {
            u64x2 o;
            o.x = r[2 * p];
            o.y = r[2 * p + 1];
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rs, (int)((uint32_t)(p * THREADS + t) * 16u),
                                                   0, SAUX < 0 ? 0 : SAUX);
        }
        return;
    }
#pragma unroll
    for (int p = 0; p < PAIRS; ++p) {
        u64x2 o;
        o.x = r[2 * p];
        o.y = r[2 * p + 1];
        reinterpret_cast<u64x2*>(out + tile_word0)[p * THREADS + t] = o;
    }
}

// tile_word0 is uniform: each leaf's tile base goes into a buffer descriptor built from
// SGPRs (readfirstlane), and every load is `buffer_load_dwordx4 v, v_off32, s[rsrc] offen nt`
// with one 32-bit per-thread offset shared by all leaves — no 64-bit VGPR address per leaf
// and pair (MI355X guide T8). The descriptor covers exactly the tile's bytes.
template <int K, int PAIRS, int THREADS>
__device__ __forceinline__ void load_tile(const EvalArgs& a, uint64_t tile_word0, int t, u64x2 (&v)[K][PAIRS]) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint64_t tw = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(tile_word0 >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)tile_word0);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(a.prog.leaf[k] + tw), (short)0, PAIRS * THREADS * 16, 0x00020000);
#pragma unroll
        for (int p = 0; p < PAIRS; ++p) {
            const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(p * THREADS + t) * 16u, 0, 2);
            v[k][p] = __builtin_bit_cast(u64x2, x);
        }
    }
}

// rowids[base + i] = row0 + st[i] for i < n, ids at or past `capacity` dropped (base and n are
// workgroup-uniform; n ≤ 2^28 so the byte range fits a buffer descriptor). 16-byte stores from
// the first ALIGN-byte boundary on, the ids before it one per thread. SAUX >= 0: buffer stores through
// a descriptor built from SGPRs with cache-policy bits SAUX — sc1 (16, write-through) measured
// 64.4 µs against 70.1 µs for plain global stores in the decode's read/write floor at SF100 Q6
// (scripts/balbench.hip, profiles/r02e_balbench_cache_policy.txt); SAUX < 0: plain stores.
template <int THREADS, int SAUX, int ALIGN = 16>
__device__ __forceinline__ void emit_ids(int64_t* rowids, uint64_t capacity, const uint32_t* st, uint32_t n,
                                         uint64_t base, int64_t row0, int t) {
    typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint64_t room = capacity > base ? capacity - base : 0;
    const uint32_t lim = (uint32_t)(room < (uint64_t)n ? room : (uint64_t)n);
    if (lim == 0) return;
    int64_t* out = rowids + base;
    static_assert(ALIGN == 16 || ALIGN == 128, "16-byte stores, optionally from a 128-byte line boundary on");
    const uint32_t head = min(lim, (uint32_t)(((ALIGN - (reinterpret_cast<uintptr_t>(out) & (ALIGN - 1))) & (ALIGN - 1)) >> 3));
    if (SAUX < 0) {
        if (t < (int)head) out[t] = row0 + (int64_t)st[t];
        for (uint32_t i = head + 2 * t; i < lim; i += 2 * THREADS) {
            if (i + 1 < lim) {
                i64x2 val;
                val.x = row0 + (int64_t)st[i];
                val.y = row0 + (int64_t)st[i + 1];
                *reinterpret_cast<i64x2*>(out + i) = val;
            } else {
                out[i] = row0 + (int64_t)st[i];
            }
        }
        return;
    }
    const uint64_t ob = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)out >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)out);
    const uint32_t nb = (uint32_t)__builtin_amdgcn_readfirstlane(lim) * 8u;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)ob, (short)0, (int)nb, 0x00020000);
    if (t < (int)head)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, row0 + (int64_t)st[t]), rs, (int)(t * 8), 0,
                                              SAUX < 0 ? 0 : SAUX);
    for (uint32_t i = head + 2 * t; i < lim; i += 2 * THREADS) {
        if (i + 1 < lim) {
            i64x2 val;
            val.x = row0 + (int64_t)st[i];
            val.y = row0 + (int64_t)st[i + 1];
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, val), rs, (int)(i * 8u), 0, SAUX < 0 ? 0 : SAUX);
        } else {
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, row0 + (int64_t)st[i]), rs, (int)(i * 8u), 0,
                                                  SAUX < 0 ? 0 : SAUX);
        }
    }
}

// The i-th tile of a launch: entry i of the planner's live-tile list (zonemap skip) or i itself.
// i is uniform, so the list entry is a scalar load; callers fetch it one tile ahead.
__device__ __forceinline__ uint32_t tile_at(const EvalArgs& a, uint32_t i) { return a.live ? a.live[i] : i; }

// ------------------------------------------------------------------ K1: count / materialise

// count(*) of the program and/or its result bitvector. Persistent: workgroup g takes tiles
// g, g+G, …, two tiles in flight (register double buffer: the loads of tile i+2 are issued
// as soon as tile i is evaluated), keeps its count in registers and claims once at the end
// (one returning atomic per workgroup).
template <int K, int PAIRS, int FORM = FORM_POSTFIX, int SAUX = -1>
__global__ __launch_bounds__(512, 4) void eval_count_kernel(EvalArgs a) {
    constexpr int THREADS = 512, NW = 2 * PAIRS;
    constexpr uint64_t TILE_WORDS = (uint64_t)THREADS * NW;
    const int t = threadIdx.x;
    const uint32_t G = gridDim.x;
    uint64_t c = 0;
    u64x2 v0[K][PAIRS], v1[K][PAIRS];
    // i indexes the launch's tiles (tile_at: every tile, or the live-tile list)
    uint32_t i = blockIdx.x;
    const uint32_t n = a.num_tiles;
    if (i < n) load_tile<K, PAIRS, THREADS>(a, (uint64_t)tile_at(a, i) * TILE_WORDS, t, v0);
    if (i + G < n) load_tile<K, PAIRS, THREADS>(a, (uint64_t)tile_at(a, i + G) * TILE_WORDS, t, v1);
    auto step = [&](u64x2 (&v)[K][PAIRS], uint32_t ii) {
        const uint32_t ahead = ii + 2 * G;
        const uint32_t ahead_tile = ahead < n ? tile_at(a, ahead) : 0;  // list entry fetched before the eval
        const uint64_t tile_word0 = (uint64_t)tile_at(a, ii) * TILE_WORDS;
        uint64_t r[NW];
        eval_words<K, NW, FORM>(a.prog, v, r);
        if (ahead < n) load_tile<K, PAIRS, THREADS>(a, (uint64_t)ahead_tile * TILE_WORDS, t, v);
        tail_mask<NW, THREADS>(a, tile_word0, t, r);
        if (a.result_words) store_words<PAIRS, THREADS, SAUX>(a.result_words, tile_word0, t, r);
#pragma unroll
        for (int j = 0; j < NW; ++j) c += __popcll(r[j]);
    };
    while (i < n) {
        step(v0, i);
        i += G;
        if (i >= n) break;
        step(v1, i);
        i += G;
    }
    __shared__ uint64_t s_part[THREADS / 64];
    c = wave_sum(c);
    if ((t & 63) == 0) s_part[t >> 6] = c;
    __syncthreads();
    if (t == 0) {
        uint64_t s = 0;
#pragma unroll
        for (int w = 0; w < THREADS / 64; ++w) s += s_part[w];
        // one arrival carries the count: no returning claim per workgroup (512 of them on one
        // word queued ≈5.8 µs at the end of every count launch, ≈88 per µs)
        finish_ticket(a.ticket, a.count, s);
    }
}

// ------------------------------------------------------------------ K1+K2: evaluate + decode

// Per-tile-claim evaluate + decode (round-1 production kernel, now kept as the reference
// variant in scripts/kbench.hip; the library launches eval_decode_pairs below).
// Persistent, software-pipelined evaluate + decode. Workgroup g takes tiles g, g+G, g+2G, …
// (static striding: per-tile work is uniform up to the decode). Per tile:
//   evaluate the tile whose leaves landed → per-pair bit counts → block scan →
//   ONE returning atomicAdd on the running count claims the tile's output range →
//   issue the NEXT tile's loads (they fly during the rest of this iteration) →
//   decode the set bits into LDS as 32-bit tile-local offsets (each thread's run is
//   ascending and runs are in word order) → copy the run out coalesced as int64 row ids.
// Output: per-tile ascending runs, runs in claim order — the shape of DuckDB's parallel scan,
// whose morsels reach the sink in nondeterministic order with a batch index
// (table_scan.cpp:179-189). dir[2·tile] / dir[2·tile+1] = the run's start / length, so
// reading runs in tile order yields the ascending sequence (order_runs does that on device).
// There is no inter-workgroup wait: a claim is one atomic, so no prefix chain serialises the
// tiles (a decoupled look-back over ~10^4 tiles measured 1.7× slower).
// Per-pair counts are packed as FB-bit fields so one 64-bit scan covers several pairs
// (a pair-chunk holds at most THREADS·128 set bits).
// CLAIM / DECODE = false are diagnostic builds (scripts/kbench.hip). __launch_bounds__: two workgroups per CU (2·THREADS/256 waves per SIMD) caps
// VGPRs at 128.
template <int K, int PAIRS, int STAGE, int THREADS, bool CLAIM = true, bool DECODE = true, int FORM = FORM_POSTFIX>
__global__ __launch_bounds__(THREADS, 2 * THREADS / 256) void eval_decode_tiles(EvalArgs a, uint64_t* __restrict__ dir) {
    constexpr int NW = 2 * PAIRS;
    constexpr int FB = (THREADS * 128 < 65536) ? 16 : 32;
    constexpr int FPW = 64 / FB;
    constexpr uint64_t FMASK = (FB == 16) ? 0xffffull : 0xffffffffull;
    constexpr int NPK = (PAIRS + FPW - 1) / FPW;
    constexpr uint64_t TILE_WORDS = (uint64_t)THREADS * NW;
    constexpr int NWAVES = THREADS / 64;
    static_assert(TILE_WORDS * 64 < (1ull << 32), "tile-local offsets are 32-bit");
    __shared__ uint64_t s_wave_tot[NWAVES][NPK];
    __shared__ uint64_t s_off;
    __shared__ uint32_t s_stage[STAGE];

    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = t >> 6;
    uint32_t tile = blockIdx.x;
    uint64_t mine = 0;  // thread 0: rows claimed by this workgroup
    u64x2 v[K][PAIRS];
    if (tile < a.num_tiles) load_tile<K, PAIRS, THREADS>(a, (uint64_t)tile * TILE_WORDS, t, v);
    while (tile < a.num_tiles) {
        const uint64_t tile_word0 = (uint64_t)tile * TILE_WORDS;
        uint64_t r[NW];
        eval_words<K, NW, FORM>(a.prog, v, r);
        tail_mask<NW, THREADS>(a, tile_word0, t, r);
        if (a.result_words) store_words<PAIRS, THREADS>(a.result_words, tile_word0, t, r);
        uint64_t packed[NPK], incl[NPK];
#pragma unroll
        for (int q = 0; q < NPK; ++q) packed[q] = 0;
#pragma unroll
        for (int p = 0; p < PAIRS; ++p)
            packed[p / FPW] |= (uint64_t)(__popcll(r[2 * p]) + __popcll(r[2 * p + 1])) << (FB * (p % FPW));
#pragma unroll
        for (int q = 0; q < NPK; ++q) {
            incl[q] = wave_incl_scan(packed[q], lane);
            if (lane == 63) s_wave_tot[wave][q] = incl[q];
        }
        __syncthreads();  // A: wave totals visible
        uint64_t block_tot[NPK], wave_pre[NPK];
#pragma unroll
        for (int q = 0; q < NPK; ++q) {
            uint64_t wp = 0, bt = 0;
#pragma unroll
            for (int w = 0; w < NWAVES; ++w) {
                const uint64_t x = s_wave_tot[w][q];
                if (w < wave) wp += x;
                bt += x;
            }
            block_tot[q] = bt;
            wave_pre[q] = wp;
        }
        uint64_t pair_base[PAIRS];
        uint64_t tile_count = 0;
#pragma unroll
        for (int p = 0; p < PAIRS; ++p) {
            pair_base[p] = tile_count;
            tile_count += (block_tot[p / FPW] >> (FB * (p % FPW))) & FMASK;
        }
        uint64_t claimed = 0;
        if (t == 0 && tile_count) {  // not wave-aggregated: built with -amdgpu-atomic-optimizer-strategy=None
            claimed = CLAIM ? atomicAdd(reinterpret_cast<unsigned long long*>(a.ticket), (unsigned long long)tile_count)
                            : (uint64_t)tile * (TILE_WORDS * 64 / 50);  // diag: ~2 % density, disjoint runs
            mine += tile_count;
        }
        const uint32_t next = tile + gridDim.x;
        if (next < a.num_tiles) load_tile<K, PAIRS, THREADS>(a, (uint64_t)next * TILE_WORDS, t, v);  // prefetch
        const bool stage = tile_count <= (uint64_t)STAGE;
        const bool write = DECODE && tile_count && a.rowids;
        if (!stage || !write) {
            if (t == 0) {
                s_off = claimed;
                if (dir) {
                    dir[2 * tile] = tile_count ? claimed : 0;
                    dir[2 * tile + 1] = tile_count;
                }
            }
            __syncthreads();
        }
        const uint64_t direct_off = s_off;
        const int64_t row0 = a.row_base + (int64_t)(tile_word0 * 64);
        if (write) {
#pragma unroll
            for (int p = 0; p < PAIRS; ++p) {
                uint64_t off = pair_base[p] +
                               (((wave_pre[p / FPW] + incl[p / FPW] - packed[p / FPW]) >> (FB * (p % FPW))) & FMASK);
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    uint64_t w = r[2 * p + e];
                    const uint32_t wrow = (uint32_t)((p * 2 * THREADS + 2 * t + e) * 64);
                    while (w) {
                        const uint32_t b = (uint32_t)__builtin_ctzll(w);
                        if (stage) {
                            s_stage[off] = wrow + b;
                        } else {
                            const uint64_t g = direct_off + off;
                            if (g < a.capacity) a.rowids[g] = row0 + (int64_t)(wrow + b);
                        }
                        ++off;
                        w &= w - 1;
                    }
                }
            }
        }
        if (stage && write) {
            if (t == 0) {
                s_off = claimed;
                if (dir) {
                    dir[2 * tile] = claimed;
                    dir[2 * tile + 1] = tile_count;
                }
            }
            __syncthreads();  // B: staged run and its offset visible
            const uint64_t off0 = s_off;
            // 16-byte stores (a wave writes 1 KiB per instruction); one leading 8-byte element
            // when the run starts off a 16-byte boundary
            typedef int64_t i64x2 __attribute__((ext_vector_type(2)));
            int64_t* out = a.rowids + off0;
            const uint32_t head = (uint32_t)((reinterpret_cast<uintptr_t>(out) >> 3) & 1);
            const uint64_t room = a.capacity > off0 ? a.capacity - off0 : 0;
            const uint32_t n = (uint32_t)tile_count;
            if (t == 0 && head && room) out[0] = row0 + (int64_t)s_stage[0];
            for (uint32_t i = head + 2 * t; i < n; i += 2 * THREADS) {
                if (i + 1 < n && i + 1 < room) {
                    i64x2 val;
                    val.x = row0 + (int64_t)s_stage[i];
                    val.y = row0 + (int64_t)s_stage[i + 1];
                    *reinterpret_cast<i64x2*>(out + i) = val;
                } else if (i < room) {
                    out[i] = row0 + (int64_t)s_stage[i];
                }
            }
        }
        __syncthreads();  // C: stage / s_off / s_wave_tot free for the next tile
        tile = next;
    }
    if (t == 0) finish_ticket(a.ticket, a.count, mine);
}

__device__ uint64_t* g_diag_times;  // DIAG & 4 builds only (scripts/kbench.hip)

// Pair-claimed evaluate + decode: one returning atomic per PAIR of tiles, issued one unit
// before its result is needed, so the claim latency is covered by the next tile's work.
// Per pair (tiles A = u, B = u + G of this workgroup's walk):
//   unit A: wait A's leaves → eval → block scan → copy out the PREVIOUS pair (its claim
//           returned meanwhile) → prefetch B → decode A into the pair's stage
//   unit B: wait B's leaves → eval → block scan → claim cnt(A)+cnt(B) → prefetch the next A →
//           decode B into the stage right after A's run
// Stage entries are 32-bit row offsets from tile A's first row (tile B sits G·TILE_ROWS
// further), so the pair's output is ONE contiguous run of cnt(A)+cnt(B) ids, copied out with
// 16-byte stores (measured: 16 B/lane stores cut this read/write mix's floor from 81 to 77 µs).
// Copy-out stores are issued before the prefetch they precede, so the wait for the prefetched
// leaves (vmcnt counts stores too) does not add a store round trip. A tile with more than
// STAGE hits claims on its own and writes straight to the output (dense path).
template <int K, int PAIRS, int STAGE, int THREADS, int DIAG = 0, int FORM = FORM_POSTFIX, int WG_PER_CU = 2,
          bool DSTAGE = true, int SAUX = 16>
__global__ __launch_bounds__(THREADS, WG_PER_CU * THREADS / 256) void eval_decode_pairs(EvalArgs a,
                                                                                       uint64_t* __restrict__ dir) {
    // DIAG (scripts/kbench.hip only): bit 0 = no claim (fixed pair offsets), bit 1 = uniform
    // fake decode (same LDS traffic, no per-bit loop), bit 2 = record each workgroup's start
    // and end (s_memrealtime, 100 MHz) into g_diag_times[2·blockIdx + {0, 1}]
    constexpr int NW = 2 * PAIRS;
    constexpr uint64_t TILE_WORDS = (uint64_t)THREADS * NW;
    constexpr uint64_t TILE_ROWS = TILE_WORDS * 64;
    constexpr int NWAVES = THREADS / 64;
    constexpr bool EARLY = K <= 4;
    static_assert(TILE_WORDS * 64 < (1ull << 32), "tile-local offsets are 32-bit");
    static_assert(PAIRS <= 2, "pair counts are scanned as 16-bit fields of one uint32");
    __shared__ uint32_t s_wave_tot[2][NWAVES];
    __shared__ uint64_t s_off;        // claimed base of the pair being copied out
    __shared__ uint64_t s_dense_off;  // claimed base of a dense tile
    __shared__ uint32_t s_stage[2][2 * STAGE];
    __shared__ uint32_t s_tile_a[2], s_tile_b[2], s_cnt_a[2], s_cnt_b[2], s_dense[2];

    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = t >> 6;
    const uint32_t G = gridDim.x;
    // B's rows as offsets from A's first row must fit 32 bits
    if ((uint64_t)G * TILE_ROWS + TILE_ROWS >= (1ull << 32)) __builtin_trap();
    const bool write_ids = a.rowids != nullptr;
    if ((DIAG & 4) && t == 0) g_diag_times[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    uint64_t pend_claim = 0;  // thread 0: the previous pair's claimed base
    uint64_t mine = 0;        // thread 0: rows claimed by this workgroup (carried by its arrival)

    u64x2 v[K][PAIRS];
    uint32_t tile = blockIdx.x;
    if (tile < a.num_tiles) load_tile<K, PAIRS, THREADS>(a, (uint64_t)tile * TILE_WORDS, t, v);

    // evaluate the tile in v → r, block scan → per-pair offsets within the tile, tile count
    // publish the previous pair's claim (thread 0, before a barrier): base + directory entries
    auto publish = [&](int sp) {
        s_off = pend_claim;
        if (dir) {
            // staged tiles (dense ones wrote their own entry); empty tiles get {0, 0}
            const uint32_t ca = s_cnt_a[sp], cb = s_cnt_b[sp];
            if (!(s_dense[sp] & 1)) {
                dir[2 * s_tile_a[sp]] = ca ? pend_claim : 0;
                dir[2 * s_tile_a[sp] + 1] = ca;
            }
            if (!(s_dense[sp] & 2) && s_tile_b[sp] < a.num_tiles) {
                dir[2 * s_tile_b[sp]] = cb ? pend_claim + ca : 0;
                dir[2 * s_tile_b[sp] + 1] = cb;
            }
        }
    };

    // evaluate the tile in v → r; with EARLY, issue the loads of tile `prefetch` into v right
    // away (v is dead once evaluated: the longest prefetch distance one register set allows;
    // K ≤ 4 only — at K ≥ 5 the leaves in flight beside the scan state spill, measured
    // 92 vs 88 µs, so the loads wait until after the copy-out / claim);
    // block scan → per-pair offsets within the tile, tile count
    auto eval_scan = [&](uint32_t tl, int par, uint64_t (&r)[NW], uint32_t (&pair_off)[PAIRS],
                         int publish_sp, uint32_t prefetch) -> uint64_t {
        const uint64_t tile_word0 = (uint64_t)tl * TILE_WORDS;
        eval_words<K, NW, FORM>(a.prog, v, r);
        if (EARLY && prefetch < a.num_tiles) load_tile<K, PAIRS, THREADS>(a, (uint64_t)prefetch * TILE_WORDS, t, v);
        tail_mask<NW, THREADS>(a, tile_word0, t, r);
        if (a.result_words) store_words<PAIRS, THREADS>(a.result_words, tile_word0, t, r);
        // pair counts as 16-bit fields of one uint32 (a wave's total per pair ≤ 8,192), DPP scan
        uint32_t packed = 0;
#pragma unroll
        for (int p = 0; p < PAIRS; ++p)
            packed |= (uint32_t)(__popcll(r[2 * p]) + __popcll(r[2 * p + 1])) << (16 * p);
        const uint32_t incl = wave_incl_scan32(packed);
        if (lane == 63) s_wave_tot[par][wave] = incl;
        if (publish_sp >= 0 && t == 0) publish(publish_sp);
        __syncthreads();
        uint32_t wave_pre[2] = {0, 0}, block_tot[2] = {0, 0};
#pragma unroll
        for (int w = 0; w < NWAVES; ++w) {
            const uint32_t x = s_wave_tot[par][w];
            const uint32_t lo = x & 0xffffu, hi = x >> 16;
            if (w < wave) {
                wave_pre[0] += lo;
                wave_pre[1] += hi;
            }
            block_tot[0] += lo;
            block_tot[1] += hi;
        }
        const uint32_t excl = incl - packed;
        // in-tile offsets and counts fit 32 bits (≤ TILE_WORDS·64 < 2^32, static_assert below)
        uint32_t tile_count = 0;
#pragma unroll
        for (int p = 0; p < PAIRS; ++p) {
            pair_off[p] = tile_count + wave_pre[p] + ((excl >> (16 * p)) & 0xffffu);
            tile_count += block_tot[p];
        }
        return tile_count;
    };

    // rowids[base + i] = row0 + st[i] for i < n: 16-byte stores (the first id alone when the
    // output is not 16-byte aligned there), bounded by the capacity
    auto emit = [&](const uint32_t* st, uint32_t n, uint64_t base, int64_t row0) {
        emit_ids<THREADS, SAUX>(a.rowids, a.capacity, st, n, base, row0, t);
    };

    // decode r into stage sp at stage_base with row offsets + delta; a dense tile claims on its
    // own and leaves through the other stage (copied out already) in rounds of 2·STAGE ids.
    // Returns the staged count (0 for a dense tile).
    auto decode = [&](uint32_t tl, int sp, uint32_t stage_base, uint32_t delta, const uint64_t (&r)[NW],
                      const uint32_t (&pair_off)[PAIRS], uint64_t tile_count) -> uint32_t {
        if (tile_count <= (uint64_t)STAGE) {
            if (DIAG & 2) {
                for (uint32_t i = t; i < (uint32_t)tile_count; i += THREADS) s_stage[sp][stage_base + i] = delta + i * 53;
            } else if (write_ids) {
#pragma unroll
                for (int p = 0; p < PAIRS; ++p) {
                    uint32_t off = stage_base + (uint32_t)pair_off[p];
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        uint64_t w = r[2 * p + e];
                        const uint32_t wrow = delta + (uint32_t)((p * 2 * THREADS + 2 * t + e) * 64);
                        while (w) {
                            s_stage[sp][off++] = wrow + (uint32_t)__builtin_ctzll(w);
                            w &= w - 1;
                        }
                    }
                }
            }
            return (uint32_t)tile_count;
        }
        // dense tile: its own claim, direct writes
        const int64_t row0 = a.row_base + (int64_t)((uint64_t)tl * TILE_ROWS);
        if (t == 0) {
            const uint64_t c = atomicAdd(reinterpret_cast<unsigned long long*>(a.ticket), (unsigned long long)tile_count);
            mine += tile_count;
            s_dense_off = c;
            if (dir) {
                dir[2 * tl] = c;
                dir[2 * tl + 1] = tile_count;
            }
        }
        __syncthreads();  // also: every thread is done with the copy-out of stage sp ^ 1
        const uint64_t base = s_dense_off;
        if (write_ids && DSTAGE) {
            // stage sp ^ 1 was copied out before this pair's first barrier and is next written
            // by the next pair, behind its own barrier
            uint32_t* st = s_stage[sp ^ 1];
            constexpr uint32_t CAP = 2 * STAGE;
            for (uint32_t r0 = 0; r0 < (uint32_t)tile_count; r0 += CAP) {
                const uint32_t r1 = min((uint32_t)tile_count, r0 + CAP);
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
                                st[k - r0] = wrow + (uint32_t)__builtin_ctzll(w);
                                w &= w - 1;
                            }
                        }
                        off += c;
                    }
                }
                __syncthreads();
                emit(st, r1 - r0, base + r0, row0);
                __syncthreads();
            }
        } else if (write_ids) {
#pragma unroll
            for (int p = 0; p < PAIRS; ++p) {
                uint64_t off = base + pair_off[p];
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    uint64_t w = r[2 * p + e];
                    const uint32_t wrow = (uint32_t)((p * 2 * THREADS + 2 * t + e) * 64);
                    while (w) {
                        if (off < a.capacity) a.rowids[off] = row0 + (int64_t)(wrow + (uint32_t)__builtin_ctzll(w));
                        ++off;
                        w &= w - 1;
                    }
                }
            }
        }
        __syncthreads();  // s_dense_off (and the scratch stage) free again
        return 0;
    };

    // copy out stage sp (one contiguous run of cnt_a + cnt_b ids) at the claimed base, which
    // thread 0 published before the barrier that precedes this call. No barrier of its own:
    // stage sp is next written two units later and s_off next published one pair later,
    // both behind barriers every thread passes after this copy.
    auto copy_out = [&](int sp) {
        const uint64_t base = s_off;
        const uint32_t n = s_cnt_a[sp] + s_cnt_b[sp];
        if (write_ids && n)
            emit_ids<THREADS, SAUX>(a.rowids, a.capacity, s_stage[sp], n, base,
                                    a.row_base + (int64_t)((uint64_t)s_tile_a[sp] * TILE_ROWS), t);
    };

    bool pending = false;  // a claimed pair waits for copy-out (uniform)
    uint32_t pair = 0;
    while (tile < a.num_tiles) {
        const int sp = (int)(pair & 1);
        // ---- unit A
        uint64_t r[NW];
        uint32_t off[PAIRS];
        const uint32_t tile_b = tile + G;
        const uint64_t cnt_a_all = eval_scan(tile, 0, r, off, pending ? (sp ^ 1) : -1, tile_b);
        if (pending) copy_out(sp ^ 1);
        if (!EARLY && tile_b < a.num_tiles) load_tile<K, PAIRS, THREADS>(a, (uint64_t)tile_b * TILE_WORDS, t, v);
        const uint32_t ca = decode(tile, sp, 0, 0, r, off, cnt_a_all);
        // ---- unit B
        uint32_t cb = 0;
        uint32_t next = tile_b;
        bool dense_b = false;
        if (tile_b < a.num_tiles) {
            next = tile_b + G;
            const uint64_t cnt_b_all = eval_scan(tile_b, 1, r, off, -1, next);
            dense_b = cnt_b_all > (uint64_t)STAGE;
            const uint32_t staged_b = cnt_b_all <= (uint64_t)STAGE ? (uint32_t)cnt_b_all : 0;
            if (t == 0 && (ca + staged_b)) {
                pend_claim = (DIAG & 1) ? (uint64_t)tile * 5400
                                        : atomicAdd(reinterpret_cast<unsigned long long*>(a.ticket), (unsigned long long)(ca + staged_b));
                mine += ca + staged_b;
            }
            if (!EARLY && next < a.num_tiles) load_tile<K, PAIRS, THREADS>(a, (uint64_t)next * TILE_WORDS, t, v);
            cb = decode(tile_b, sp, ca, G * (uint32_t)TILE_ROWS, r, off, cnt_b_all);
        } else if (t == 0 && ca) {
            pend_claim = atomicAdd(reinterpret_cast<unsigned long long*>(a.ticket), (unsigned long long)ca);
            mine += ca;
        }
        if (t == 0) {
            s_tile_a[sp] = tile;
            s_tile_b[sp] = tile_b;
            s_cnt_a[sp] = ca;
            s_cnt_b[sp] = cb;
            s_dense[sp] = (cnt_a_all > (uint64_t)STAGE ? 1u : 0u) | (dense_b ? 2u : 0u);
        }
        __syncthreads();  // this pair's stage and counts complete
        pending = true;
        tile = next;
        ++pair;
    }
    if (pending) {
        const int sp = (int)((pair - 1) & 1);
        if (t == 0) publish(sp);
        __syncthreads();
        copy_out(sp);
    }
    if (t == 0) finish_ticket(a.ticket, a.count, mine);
    if ((DIAG & 4) && t == 0) g_diag_times[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
}

// Run-claimed evaluate + decode: the workgroup keeps decoding tiles into one LDS stage (a
// *run*) until the next tile would not fit (or the run holds MAXT tiles), then claims the whole
// run with ONE returning atomic and switches to the other stage; the claim returns while the
// next tile is evaluated, and the closed run is copied out (16-byte stores) after that tile's
// scan barrier. The claim count follows the output volume (≈ q / RUN_CAP + workgroups) instead
// of the tile count (pairs: one per two tiles), and a tile costs one block barrier instead of
// one and a half. A stage entry is the row's offset from the run's first tile row (a run spans
// fewer than 2^32 / TILE_ROWS tiles so that fits 32 bits), so the copy-out adds one base per run.
// With a live-tile list (zonemap skip) the workgroup walks list entries g, g+G, … instead of
// tiles; runs, offsets and the directory are per tile as before, skipped tiles keep the {0, 0}
// entries the host cleared. Tiles with more than RUN_CAP hits claim on
// their own and write straight to the output (dense path). The directory gets {start, len} per
// tile ({0, 0} for empty tiles) as with pairs.
// Workgroup g takes tiles g, g+G, … (static striding). A dynamic hand-out of the last third of
// the tiles from per-XCD heads (scripts/kbench.hip) evened the workgroups' end
// times (spread 25 → 14 µs) but slowed every workgroup more than that gained: its dequeue is a
// returning atomic that the next wait on the leaf loads (vmcnt counts in order) also waits for.
template <int K, int PAIRS, int RUN_CAP, int THREADS, int FORM = FORM_POSTFIX, int MAXT = 16, bool STAMP = false,
          bool DSTAGE = true, int SAUX = 16, int ALIGN = 16, int EARLY_AT = 4>
__global__ __launch_bounds__(THREADS, 2 * THREADS / 256) void eval_decode_runs(EvalArgs a, uint64_t* __restrict__ dir) {
    // STAMP (scripts/kbench.hip only): each workgroup's start / end (s_memrealtime) into g_diag_times
    if (STAMP && threadIdx.x == 0) g_diag_times[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    constexpr int NW = 2 * PAIRS;
    constexpr uint64_t TILE_WORDS = (uint64_t)THREADS * NW;
    constexpr uint64_t TILE_ROWS = TILE_WORDS * 64;
    static_assert(MAXT <= 64, "directory entries per run");
    constexpr int NWAVES = THREADS / 64;
    constexpr bool EARLY = K <= EARLY_AT;  // next tile's loads before the copy-out (K <= 4) or after it
    // per-wave totals of the pair counts, two 16-bit fields (a wave's total per pair is at most
    // 64 lanes × 128 bits = 8,192)
    static_assert(PAIRS <= 2, "pair counts are scanned as 16-bit fields of one uint32");
    __shared__ uint32_t s_wave_tot[2][NWAVES];
    __shared__ uint64_t s_off;        // claimed base of the run being copied out
    __shared__ uint64_t s_dense_off;  // claimed base of a dense tile
    __shared__ uint32_t s_stage[2][RUN_CAP];
    __shared__ uint32_t s_rt[2][MAXT], s_ro[2][MAXT], s_rc[2][MAXT];  // run tiles: tile, offset, count
    __shared__ uint32_t s_rn[2], s_rfill[2], s_rfirst[2];

    const int t = threadIdx.x;
    const int lane = t & 63;
    const int wave = t >> 6;
    const uint32_t G = gridDim.x;
    // a stage entry (tile - run's first tile)·TILE_ROWS + row must fit 32 bits
    constexpr uint32_t kMaxSpan = (uint32_t)((1ull << 32) / TILE_ROWS);
    const bool write_ids = a.rowids != nullptr;
    uint64_t pend_claim = 0;  // thread 0: the closed run's claimed base
    uint64_t mine = 0;        // thread 0: rows claimed by this workgroup

    u64x2 v[K][PAIRS];
    // i indexes the launch's tiles (every tile, or the live-tile list of the zonemap skip);
    // tile / next_tile are the current and the next tile, the list entry after them is fetched
    // one unit ahead
    const uint32_t n_idx = a.num_tiles;
    uint32_t i = blockIdx.x;
    uint32_t tile = i < n_idx ? tile_at(a, i) : 0;
    uint32_t next_tile = i + G < n_idx ? tile_at(a, i + G) : 0;
    if (i < n_idx) load_tile<K, PAIRS, THREADS>(a, (uint64_t)tile * TILE_WORDS, t, v);

    // rowids[base + i] = row0 + st[i] for i < n: 16-byte stores (the first id alone when the
    // output is not 16-byte aligned there), bounded by the capacity
    auto emit = [&](const uint32_t* st, uint32_t n, uint64_t base, int64_t row0) {
        emit_ids<THREADS, SAUX, ALIGN>(a.rowids, a.capacity, st, n, base, row0, t);
    };
    // copy out closed run rs at s_off (published before the preceding barrier) and write its
    // directory entries
    auto copy_out = [&](int rs) {
        const uint64_t base = s_off;
        const uint32_t n = s_rfill[rs];
        const uint32_t nt = s_rn[rs];
        if (dir && t < (int)nt) {
            dir[2 * s_rt[rs][t]] = s_rc[rs][t] ? base + s_ro[rs][t] : 0;
            dir[2 * s_rt[rs][t] + 1] = s_rc[rs][t];
        }
        if (write_ids && n) emit(s_stage[rs], n, base, a.row_base + (int64_t)((uint64_t)s_rfirst[rs] * TILE_ROWS));
    };

    int rs = 0;              // the open run's stage
    uint32_t fill = 0, rn = 0, rfirst = 0;  // open run: entries, tiles, first tile (uniform)
    bool pending = false;    // a closed run (stage rs ^ 1) waits for its claim and copy-out
    uint32_t u = 0;
    while (i < n_idx) {
        const int par = (int)(u & 1);
        const uint64_t tile_word0 = (uint64_t)tile * TILE_WORDS;
        const bool has_next = i + G < n_idx;
        const uint32_t after = i + 2 * G < n_idx ? tile_at(a, i + 2 * G) : 0;
        uint64_t r[NW];
        eval_words<K, NW, FORM>(a.prog, v, r);
        if (EARLY && has_next) load_tile<K, PAIRS, THREADS>(a, (uint64_t)next_tile * TILE_WORDS, t, v);
        tail_mask<NW, THREADS>(a, tile_word0, t, r);
        if (a.result_words) store_words<PAIRS, THREADS>(a.result_words, tile_word0, t, r);
        uint32_t packed = 0;
#pragma unroll
        for (int p = 0; p < PAIRS; ++p)
            packed |= (uint32_t)(__popcll(r[2 * p]) + __popcll(r[2 * p + 1])) << (16 * p);
        const uint32_t incl = wave_incl_scan32(packed);
        if (lane == 63) s_wave_tot[par][wave] = incl;
        if (pending && t == 0) s_off = pend_claim;  // the closed run's claim returned meanwhile
        __syncthreads();
        uint32_t wave_pre[2] = {0, 0}, block_tot[2] = {0, 0};
#pragma unroll
        for (int w = 0; w < NWAVES; ++w) {
            const uint32_t x = s_wave_tot[par][w];
            const uint32_t lo = x & 0xffffu, hi = x >> 16;
            if (w < wave) {
                wave_pre[0] += lo;
                wave_pre[1] += hi;
            }
            block_tot[0] += lo;
            block_tot[1] += hi;
        }
        const uint32_t excl = incl - packed;  // per field: no borrow (incl ≥ packed field-wise)
        uint32_t pair_off[PAIRS];
        uint32_t tile_count = 0;
#pragma unroll
        for (int p = 0; p < PAIRS; ++p) {
            pair_off[p] = tile_count + wave_pre[p] + ((excl >> (16 * p)) & 0xffffu);
            tile_count += block_tot[p];
        }
        const bool dense = tile_count > (uint32_t)RUN_CAP;
        // close the open run when this tile does not fit (claimed after the previous run's
        // copy-out: issuing the claim before it measured 3 µs slower at K = 5)
        const bool close = !dense && rn > 0 &&
                           (fill + tile_count > (uint32_t)RUN_CAP || rn == (uint32_t)MAXT || tile - rfirst >= kMaxSpan);
        const bool copied = pending;
        if (pending) {
            copy_out(rs ^ 1);
            pending = false;
        }
        if (!EARLY && has_next) load_tile<K, PAIRS, THREADS>(a, (uint64_t)next_tile * TILE_WORDS, t, v);
        const int64_t row0 = a.row_base + (int64_t)tile_word0 * 64;
        if (dense) {
            // dense tile: its own claim, direct writes
            if (t == 0) {
                const uint64_t c = atomicAdd(reinterpret_cast<unsigned long long*>(a.ticket), (unsigned long long)tile_count);
                mine += tile_count;
                s_dense_off = c;
                if (dir) {
                    dir[2 * tile] = c;
                    dir[2 * tile + 1] = tile_count;
                }
            }
            __syncthreads();  // also: every thread is done with the copy-out of stage rs ^ 1
            const uint64_t base = s_dense_off;
            if (write_ids && DSTAGE) {
                // in rounds of RUN_CAP ids through the free stage (rs ^ 1; the open run keeps
                // stage rs): each thread decodes its bits whose tile-local index falls in the
                // round, then the round leaves as 16-byte stores
                uint32_t* st = s_stage[rs ^ 1];
                for (uint32_t r0 = 0; r0 < tile_count; r0 += (uint32_t)RUN_CAP) {
                    const uint32_t r1 = min(tile_count, r0 + (uint32_t)RUN_CAP);
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
                                    st[k - r0] = wrow + (uint32_t)__builtin_ctzll(w);
                                    w &= w - 1;
                                }
                            }
                            off += c;
                        }
                    }
                    __syncthreads();
                    emit(st, r1 - r0, base + r0, row0);
                    __syncthreads();
                }
            } else if (write_ids) {
#pragma unroll
                for (int p = 0; p < PAIRS; ++p) {
                    uint64_t off = base + pair_off[p];
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        uint64_t w = r[2 * p + e];
                        const uint32_t wrow = (uint32_t)((p * 2 * THREADS + 2 * t + e) * 64);
                        while (w) {
                            if (off < a.capacity) a.rowids[off] = row0 + (int64_t)(wrow + (uint32_t)__builtin_ctzll(w));
                            ++off;
                            w &= w - 1;
                        }
                    }
                }
            }
            __syncthreads();  // s_dense_off (and the scratch stage) free again
        } else {
            if (close) {
                // one claim for the whole run (returns during the next tile)
                if (t == 0) {
                    s_rn[rs] = rn;
                    s_rfill[rs] = fill;
                    s_rfirst[rs] = rfirst;
                    pend_claim = 0;
                    if (fill) {
                        pend_claim = atomicAdd(reinterpret_cast<unsigned long long*>(a.ticket), (unsigned long long)fill);
                        mine += fill;
                    }
                }
                pending = true;
                rs ^= 1;
                fill = 0;
                rn = 0;
                // the stage we switch to was copied out in this unit: every thread must be done
                if (copied) __syncthreads();
            }
            if (rn == 0) rfirst = tile;
            if (tile_count && write_ids) {
                const uint32_t delta = (tile - rfirst) * (uint32_t)TILE_ROWS;
#pragma unroll
                for (int p = 0; p < PAIRS; ++p) {
                    uint32_t off = fill + pair_off[p];
#pragma unroll
                    for (int e = 0; e < 2; ++e) {
                        uint64_t w = r[2 * p + e];
                        const uint32_t wrow = delta + (uint32_t)((p * 2 * THREADS + 2 * t + e) * 64);
                        while (w) {
                            s_stage[rs][off++] = wrow + (uint32_t)__builtin_ctzll(w);
                            w &= w - 1;
                        }
                    }
                }
            }
            if (t == 0) {
                s_rt[rs][rn] = tile;
                s_ro[rs][rn] = fill;
                s_rc[rs][rn] = tile_count;
            }
            fill += tile_count;
            ++rn;
        }
        i += G;
        tile = next_tile;
        next_tile = after;
        ++u;
    }
    // drain: the closed run (if any), then the open one
    if (pending) {
        if (t == 0) s_off = pend_claim;
        __syncthreads();
        copy_out(rs ^ 1);
    }
    if (rn > 0) {
        if (t == 0) {
            s_rn[rs] = rn;
            s_rfill[rs] = fill;
            s_rfirst[rs] = rfirst;
            uint64_t c = 0;
            if (fill) {
                c = atomicAdd(reinterpret_cast<unsigned long long*>(a.ticket), (unsigned long long)fill);
                mine += fill;
            }
            pend_claim = c;
        }
        __syncthreads();  // s_off may still be read by the copy-out above
        if (t == 0) s_off = pend_claim;
        __syncthreads();
        copy_out(rs);
    }
    if (t == 0) finish_ticket(a.ticket, a.count, mine);
    if (STAMP && t == 0) g_diag_times[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
}

// ------------------------------------------------------------------ K1+K2 for small partitions

// One tile per workgroup, output offsets by look-back instead of a claim. For partitions whose
// tiles fit the co-resident grid (WPC workgroups per CU: SF100 split over 8 GPUs = 572 tiles,
// SURVEY config 2 = 768), where the claim kernels are latency-bound: every workgroup of those
// takes its one claim at about the same moment, and one word serves ≈ 88 returning atomics per µs
// (MI355X_MICROARCH.md "dequeue"), so the last claim of 572 returns ≈ 6.5 µs after the first.
// Here each workgroup
//   loads and evaluates its tile → block scan → publishes the tile's count in its own flag word
//   (agent-scope store; the word carries the launch's epoch in its high bits, so flags are never
//   reset) → decodes its rows into LDS (the flags of its predecessors land meanwhile) → sums the
//   counts of every earlier workgroup, each thread polling one or two flags (agent-scope loads,
//   MI355X_MICROARCH.md hand-off table row 1; the whole window in one round trip once they are
//   published) → copies its run out at that offset and writes its directory entry. The last
//   workgroup writes the count: no arrival ticket either. A workgroup waits only on lower block
//   indices, which are dispatched before it, so the walk completes whatever the residency.
// A tile with more rows than the stage leaves through it in rounds after the offset is known.
// A poll that exceeds the spin limit (EvalArgs::spin_limit, kLookbackSpins by default) does not
// fail the scan: the thread stops waiting and flags the workgroup, which then walks the earlier
// flags once more without waiting and counts every tile still unpublished from its bitvectors
// itself (lookback_recount — the same program over the same words, so the same count). No
// workgroup ever waits on another without bound, every workgroup writes its run, and the last
// one's count is the true count whatever the dispatch order: the kernel has no failure exit for
// the host to miss.
// Runs land in tile order, so the output is one ascending array: ordered scans take this kernel
// at any size up to kLookbackMaxTiles (SF100, 4,578 tiles: 68.5 µs against 95 µs for the
// run-claimed decode plus the ordering pass; scripts/smallbench.hip).
constexpr int kFlagCntBits = 20;  // a tile holds ≤ 131,072 rows
constexpr uint32_t kLookbackSpins = 1u << 22;

// The expiry path of the look-back (workgroup-uniform call): the rows of tiles 0 … b-1 of the
// launch, each taken from its published flag when it is there now, else counted by the whole
// workgroup from the tile's bitvectors (load_tile / eval_words / tail_mask, as the tile's own
// workgroup does). s_list holds THREADS entries, s_n and s_sum are scratch.
template <int K, int FORM, int THREADS, int PAIRS>
__device__ uint64_t lookback_recount(const EvalArgs& a, uint32_t b, int t, uint32_t* s_list, uint32_t* s_n,
                                     uint64_t* s_sum) {
    constexpr int NWAVES = THREADS / 64;
    constexpr uint64_t TILE_WORDS = (uint64_t)THREADS * 2 * PAIRS;
    constexpr uint64_t kCntMask = (1ull << kFlagCntBits) - 1;
    uint64_t acc = 0;
    for (uint32_t j0 = 0; j0 < b; j0 += THREADS) {
        const uint32_t j = j0 + (uint32_t)t;
        __syncthreads();  // the previous round's list is consumed
        if (t == 0) *s_n = 0;
        __syncthreads();
        if (j < b) {
            const uint64_t f = __hip_atomic_load(a.flags + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((f >> kFlagCntBits) == a.epoch) acc += f & kCntMask;
            else s_list[atomicAdd(s_n, 1u)] = j;
        }
        __syncthreads();
        const uint32_t n_miss = *s_n;
#pragma unroll 1
        for (uint32_t i = 0; i < n_miss; ++i) {
            // one word pair per thread at a time (half the registers of the tile's own pass:
            // this runs while that pass's words are still live)
#pragma unroll 1
            for (int h = 0; h < PAIRS; ++h) {
                const uint64_t w0 = (uint64_t)tile_at(a, s_list[i]) * TILE_WORDS + (uint64_t)h * 2 * THREADS;
                u64x2 v[K][1];
                load_tile<K, 1, THREADS>(a, w0, t, v);
                uint64_t r[2];
                eval_words<K, 2, FORM>(a.prog, v, r);
                tail_mask<2, THREADS>(a, w0, t, r);
                acc += (uint64_t)(__popcll(r[0]) + __popcll(r[1]));
            }
        }
    }
    acc = wave_sum_flags(acc);
    __syncthreads();
    if ((t & 63) == 0) s_sum[t >> 6] = acc;
    __syncthreads();
    uint64_t total = 0;
#pragma unroll
    for (int w = 0; w < NWAVES; ++w) total += s_sum[w];
    return total;
}
// DBG (diagnostic builds, scripts/smallbench.hip; 0 in the library): 1 no spin, 2 no ids, 4 no
// sleep, 8 no flag loads, 16 no LDS decode, 64 the staging loop without its LDS stores, 128 the
// staging by rank (stage_by_rank) instead of the per-lane loop.
// Measured and not kept (scripts/smallbench.hip; profiles/r03e_*, r03g_*, r03h_*): eight copies of
// every flag, each reader on its own; a two-level walk (groups of 64 tiles + group totals); flag
// loads issued before the LDS decode; a decoupled look-back (aggregate, then inclusive-prefix flags,
// walks that stop at the nearest prefix) — slower at every size measured, 573 to 4,578 tiles (at
// 4,578 the sum over every earlier flag costs 68.5 µs, the decoupled walk 91 µs).
// Diagnostic (DBG 128): a wave's set bits of one word pair handed out by rank instead of by
// word — lane l's two words are words 2l, 2l+1 of the wave's slice, `inc` its inclusive count
// in the slice, `wtot` the slice's total and `base` its first stage slot; `row0` is the slice's
// first row in the tile. Each lane takes ids k = lane, lane + 64, … : the owning lane by a binary
// search over the lanes' inclusive counts (LDS), the word by its popcount, the bit by a popcount
// walk over halves (no pdep on CDNA4). Trips per wave: ⌈wtot / 64⌉ instead of the largest
// per-lane popcount of each word. Uses s_words' wave region for the words and s_inc's.
template <int THREADS>
__device__ __forceinline__ void stage_by_rank(uint64_t w0, uint64_t w1, uint32_t inc, uint32_t wtot, uint32_t base,
                                              uint32_t row0, uint64_t* s_words, uint32_t* s_inc, uint32_t* s_stage,
                                              int lane, int wave) {
    uint64_t* sw = s_words + (uint32_t)wave * 128u;
    uint32_t* si = s_inc + (uint32_t)wave * 64u;
    sw[2 * lane] = w0;
    sw[2 * lane + 1] = w1;
    si[lane] = inc;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    for (uint32_t k = (uint32_t)lane; k < wtot; k += 64u) {
        // owner: the number of lanes whose inclusive count is <= k
        uint32_t l = 0;
#pragma unroll
        for (uint32_t step = 32; step; step >>= 1)
            if (si[l + step - 1] <= k) l += step;
        const uint32_t ex = l ? si[l - 1] : 0u;
        uint32_t rk = k - ex;
        const uint64_t a0 = sw[2 * l], a1 = sw[2 * l + 1];
        const uint32_t c0 = (uint32_t)__popcll(a0);
        const bool second = rk >= c0;
        uint64_t w = second ? a1 : a0;
        rk -= second ? c0 : 0u;
        uint32_t x = (uint32_t)w, pos = 0;
        uint32_t c = (uint32_t)__popc(x);
        if (rk >= c) {
            rk -= c;
            x = (uint32_t)(w >> 32);
            pos = 32;
        }
#pragma unroll
        for (uint32_t h = 16; h; h >>= 1) {
            c = (uint32_t)__popc(x & ((1u << h) - 1u));
            if (rk >= c) {
                rk -= c;
                x >>= h;
                pos += h;
            }
        }
        s_stage[base + k] = row0 + (2u * l + (second ? 1u : 0u)) * 64u + pos;
    }
    __builtin_amdgcn_wave_barrier();
}

template <int K, int FORM, int STAGE, int WPC, int SAUX = 16, int DBG = 0, int THREADS = 512>
__global__ __launch_bounds__(THREADS, WPC * THREADS / 256) void eval_decode_lookback(EvalArgs a,
                                                                                    uint64_t* __restrict__ dir) {
    constexpr int PAIRS = 2, NW = 2 * PAIRS, NWAVES = THREADS / 64;
    constexpr uint64_t TILE_WORDS = (uint64_t)THREADS * NW;
    constexpr uint64_t kCntMask = (1ull << kFlagCntBits) - 1;
    __shared__ uint32_t s_wave_tot[NWAVES];
    __shared__ uint64_t s_pre[NWAVES];
    __shared__ uint32_t s_expired;
    __shared__ uint32_t s_list_n;
    __shared__ uint32_t s_list_scratch[THREADS];
    __shared__ uint32_t s_stage[STAGE];
    // a dense tile's result words, kept here across the look-back walk (16 KiB: three workgroups
    // per CU still fit the 160 KiB) instead of being read and evaluated a second time
    __shared__ uint64_t s_words[(uint32_t)THREADS * 2 * PAIRS];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t b = blockIdx.x;
    const uint32_t tile = tile_at(a, b);
    const uint64_t tile_word0 = (uint64_t)tile * TILE_WORDS;
    const bool write_ids = a.rowids != nullptr;
    const uint32_t spin_limit = a.spin_limit ? a.spin_limit : kLookbackSpins;
    // with per-tile counts known up front (a single index leaf: EvalArgs::tile_prefix) the
    // offset is one load, issued here so that it lands while the tile is read and decoded, and
    // no workgroup publishes or waits
    const bool prefixed = a.tile_prefix != nullptr;
    const uint64_t known_base = prefixed ? a.tile_prefix[tile] : 0;
    if (t == 0) s_expired = 0;
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
    if (t == 0 && !prefixed)
        __hip_atomic_store(a.flags + b, (a.epoch << kFlagCntBits) | (uint64_t)tile_count, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    const bool staged = tile_count <= (uint32_t)STAGE;
    if (!staged && write_ids && !(DBG & 2)) {
#pragma unroll
        for (int j = 0; j < NW; ++j) s_words[(uint32_t)j * THREADS + t] = r[j];
    }
    if ((DBG & 128) && staged && write_ids && tile_count) {
        // every lane takes ids lane, lane + 64, … of its wave's slice of each pair
#pragma unroll
        for (int p = 0; p < PAIRS; ++p) {
            const uint32_t inc = (incl >> (16 * p)) & 0xffffu;
            const uint32_t wtot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            stage_by_rank<THREADS>(r[2 * p], r[2 * p + 1], inc, wtot, pair_off[p] - (inc - (uint32_t)(__popcll(r[2 * p]) + __popcll(r[2 * p + 1]))),
                                   (uint32_t)(p * 2 * THREADS + 2 * wave * 64) * 64u, s_words, s_list_scratch, s_stage,
                                   lane, wave);
        }
    } else if (!(DBG & 16) && staged && write_ids && tile_count) {
#pragma unroll
        for (int p = 0; p < PAIRS; ++p) {
            uint32_t off = pair_off[p];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                uint64_t w = r[2 * p + e];
                const uint32_t wrow = (uint32_t)((p * 2 * THREADS + 2 * t + e) * 64);
                if (DBG & 64) {  // diagnostic: the loop without its LDS stores (positions summed)
                    uint32_t acc = 0;
                    while (w) {
                        acc += wrow + (uint32_t)__builtin_ctzll(w) + off++;
                        w &= w - 1;
                    }
                    if (acc == 0xffffffffu) s_stage[0] = acc;
                    continue;
                }
                while (w) {
                    s_stage[off++] = wrow + (uint32_t)__builtin_ctzll(w);
                    w &= w - 1;
                }
            }
        }
    }
    // look-back over every earlier workgroup's flag
    uint64_t pre = 0;
    for (uint32_t j = t; !prefixed && j < b && !(DBG & 8); j += THREADS) {
        uint64_t f = __hip_atomic_load(a.flags + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t spins = 0;
        bool gave_up = false;
        while (!(DBG & 1) && (f >> kFlagCntBits) != a.epoch) {
            // stop waiting once this thread's limit is reached or another thread of the workgroup
            // gave up: the workgroup recounts every flag below anyway, so no further flag is
            // worth a wait (without this each remaining unpublished flag cost another full limit)
            if (++spins >= spin_limit || *static_cast<volatile uint32_t*>(&s_expired)) {
                s_expired = 1;
                gave_up = true;
                break;
            }
            if (!(DBG & 4)) __builtin_amdgcn_s_sleep(2);
            f = __hip_atomic_load(a.flags + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (gave_up) break;  // `pre` is replaced by the recount
        pre += f & kCntMask;
    }
    pre = wave_sum_flags(pre);
    if (lane == 0) s_pre[wave] = pre;
    __syncthreads();  // also: the stage is complete
    uint64_t base = 0;
#pragma unroll
    for (int w = 0; w < NWAVES; ++w) base += s_pre[w];
    if (prefixed) {
        base = known_base;
    } else if (s_expired) {
        // some earlier tile was not published within the limit: every flag once more, the
        // missing tiles counted here (s_pre and s_wave_tot are free again; s_stage is not)
        base = lookback_recount<K, FORM, THREADS, PAIRS>(a, b, t, s_list_scratch, &s_list_n, s_pre);
    }
    const int64_t row0 = a.row_base + (int64_t)(tile_word0 * 64);
    if (t == 0) {
        if (dir) {
            dir[2 * tile] = tile_count ? base : 0;
            dir[2 * tile + 1] = tile_count;
        }
        if (b == gridDim.x - 1) *a.count = base + tile_count;
    }
    if (!write_ids || !tile_count || (DBG & 2)) return;
    if (staged) {
        emit_ids<THREADS, SAUX>(a.rowids, a.capacity, s_stage, tile_count, base, row0, t);
        return;
    }
    // dense tile: rounds of STAGE ids through the stage, its result words back from s_words (no
    // word is held in registers across the look-back walk and its expiry recount; reading and
    // evaluating the tile a second time instead cost 39.2 vs 30.7 µs for 673 dense tiles)
#pragma unroll
    for (int j = 0; j < NW; ++j) r[j] = s_words[(uint32_t)j * THREADS + t];
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

// A decoded value in the segments' own T when T is narrower than the column's values
// (BpGroup::tnorm, uniform per group): mod 2^bits, then sign- or zero-extended — T's
// wrap-around arithmetic (a UINT32 DELTA_FOR run that wraps, an INT16 CONSTANT_DELTA that
// steps by -3) carried out in the wider U
template <typename U>
__device__ __forceinline__ U bp_norm(U v, uint32_t tn) {
    if (!tn) return v;
    typedef typename std::conditional<sizeof(U) == 8, int64_t, int32_t>::type S;
    const uint32_t sh = (uint32_t)(sizeof(U) * 8) - (tn & 0x7fu);
    return (tn & 0x80u) ? (U)((S)(v << sh) >> sh) : (U)((U)(v << sh) >> sh);
}

// ------------------------------------------------------------------ K1+K3: fused filter + probe-sum

__device__ __forceinline__ void add128(uint64_t& lo, int64_t& hi, __int128 x) {
    const uint64_t xl = (uint64_t)x;
    const int64_t xh = (int64_t)(x >> 64);
    const uint64_t nl = lo + xl;
    hi += xh + (nl < lo ? 1 : 0);
    lo = nl;
}

// SELECT sum(a * b) WHERE <program>: evaluate a tile, decode its set bits into LDS (row
// offset, and — when b is decoded from its index — which of the M decode leaves miss the row,
// as M bits above the 17-bit tile-local offset, so b = v0 + Σ delta[m] over those bits is
// rebuilt in full int64 at the gather), then gather a (and b) for the
// staged rows with several loads in flight per thread, accumulating in 128 bits
// (DECIMAL(38,4) storage, Q6's sum(l_extendedprice * l_discount)). No row ids are written.
// Persistent like eval_decode_pairs; per-workgroup partials are summed by sum_partials_kernel;
// the qualifying-row count goes through the claim ticket.
template <int K, int M, int FORM>
__global__ __launch_bounds__(512, 4) void eval_sum_product(EvalArgs a, SumArgs s) {
    constexpr int THREADS = 512, PAIRS = 2, NW = 4, STAGE = 4096;
    constexpr int FB = 32;  // THREADS * 128 ≥ 65536
    constexpr uint64_t FMASK = 0xffffffffull;
    constexpr int FPW = 2;
    constexpr uint64_t TILE_WORDS = (uint64_t)THREADS * NW;
    constexpr int NWAVES = THREADS / 64;
    __shared__ uint64_t s_wave_tot[NWAVES];
    // s_row: tile-local row offset (bits 0..16) | decode-leaf miss bits (bits kMissShift..)
    constexpr int kMissShift = 24;
    static_assert(TILE_WORDS * 64 <= (1u << kMissShift) && M <= 32 - kMissShift, "s_row packing");
    __shared__ uint32_t s_row[STAGE];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint64_t acc_lo = 0;
    int64_t acc_hi = 0;
    uint64_t total = 0;

    // b decoded from its range index: v0 plus the deltas of the leaves that miss the row (full
    // int64 — b may be any BIGINT / DECIMAL(18,x) storage value)
    auto decoded_b = [&](uint32_t miss) -> int64_t {
        uint64_t v = (uint64_t)s.v0;  // modular: v0 + Σ deltas lands on a stored value
#pragma unroll
        for (int m = 0; m < M; ++m)
            if ((miss >> m) & 1u) v += (uint64_t)s.delta[m];
        return (int64_t)v;
    };
    // a from its BITPACKING segments: the group records of the current tile (the groups from the
    // one holding the tile's first row on; 2,048 rows each inside a segment, so a tile of 131,072
    // rows spans 64 of them, a few more where segments end mid-vector) are staged in LDS at the
    // start of the tile, so a gathered value costs one load of its packed words, like the plain
    // column's one load of its value
    constexpr int NREC = 96;
    __shared__ int32_t s_gst[NREC];   // group's first row - the tile's first row
    __shared__ uint32_t s_gcnt[NREC];
    __shared__ uint64_t s_gbase[NREC], s_gaux[NREC], s_goff[NREC];
    __shared__ uint8_t s_gmode[NREC], s_gw[NREC], s_gtn[NREC];
    uint32_t tile_g0 = 0, tile_ng = 0;  // staged records: groups tile_g0 … tile_g0 + tile_ng - 1
    uint64_t tile_row0 = 0;
    auto stage_groups = [&](uint64_t row0) {
        tile_row0 = row0;
        const uint64_t n_vec = (a.n_rows + 2047) / 2048;
        const uint64_t v0 = row0 >> 11;
        tile_g0 = s.a_vgroup[v0 < n_vec ? v0 : n_vec - 1];
        tile_ng = (uint32_t)min<uint64_t>((uint64_t)NREC, s.a_n_groups - tile_g0);
        if (t < (int)tile_ng) {
            const BpGroup& gr = s.a_groups[tile_g0 + t];
            s_gst[t] = (int32_t)((int64_t)gr.row_start - (int64_t)row0);
            s_gcnt[t] = gr.count;
            s_gbase[t] = gr.base;
            s_gaux[t] = gr.aux;
            s_goff[t] = gr.words_off;
            s_gmode[t] = gr.mode;
            s_gtn[t] = gr.tnorm;
            s_gw[t] = (uint8_t)gr.width;
        }
    };
    // a[r], from the plain column or from its BITPACKING group (group record → packed bits)
    auto load_a = [&](uint64_t r) -> int64_t {
        if (!s.a_bytes) return __builtin_nontemporal_load(s.a + r);
        const int64_t rl = (int64_t)r - (int64_t)tile_row0;
        int32_t g = (int32_t)((rl - (int64_t)s_gst[0]) >> 11);  // exact inside one segment
        if (g >= (int32_t)tile_ng) g = (int32_t)tile_ng - 1;
        while (g > 0 && rl < (int64_t)s_gst[g]) --g;
        while (g + 1 < (int32_t)tile_ng && rl >= (int64_t)s_gst[g] + (int64_t)s_gcnt[g]) ++g;
        if (rl < (int64_t)s_gst[g] || rl >= (int64_t)s_gst[g] + (int64_t)s_gcnt[g])
            return __builtin_nontemporal_load(s.a_plain + r);  // past the staged groups
        const uint64_t i = (uint64_t)(rl - (int64_t)s_gst[g]);
        const uint32_t mode = s_gmode[g], tn = s_gtn[g];
        const uint64_t base = s_gbase[g];
        if (mode == 2) return (int64_t)bp_norm<uint64_t>(base, tn);
        if (mode == 3) return (int64_t)bp_norm<uint64_t>(base + s_gaux[g] * i, tn);
        if (mode != 5) return __builtin_nontemporal_load(s.a_plain + r);  // DELTA_FOR: needs its prefix
        const uint32_t w = s_gw[g];
        if (w == 0) return (int64_t)bp_norm<uint64_t>(base, tn);
        const uint32_t* words = reinterpret_cast<const uint32_t*>(s.a_bytes + s_goff[g]);
        const uint64_t bit = i * w;
        const uint32_t wi = (uint32_t)(bit >> 5), off = (uint32_t)(bit & 31);
        uint64_t x = ((uint64_t)__builtin_nontemporal_load(words + wi) |
                      (off + w > 32 ? (uint64_t)__builtin_nontemporal_load(words + wi + 1) << 32 : 0ull)) >> off;
        if (off + w > 64) x |= (uint64_t)__builtin_nontemporal_load(words + wi + 2) << (64 - off);
        if (w < 64) x &= (1ull << w) - 1;
        return (int64_t)bp_norm<uint64_t>(x + base, tn);
    };
    auto accumulate = [&](int64_t row, int64_t bval_decoded) {
        const uint64_t r = (uint64_t)(row - a.row_base);
        if (s.a_valid && !((s.a_valid[r >> 6] >> (r & 63)) & 1ull)) return;
        int64_t bv = bval_decoded;
        if (M == 0) {
            if (s.b_valid && !((s.b_valid[r >> 6] >> (r & 63)) & 1ull)) return;
            bv = s.b[r];
        }
        add128(acc_lo, acc_hi, (__int128)load_a(r) * (__int128)bv);
    };

    u64x2 v[K][PAIRS];
    u64x2 dv[M > 0 ? M : 1][PAIRS];
    // i indexes the launch's tiles (every tile, or the zonemap skip's live-tile list)
    const uint32_t n_idx = a.num_tiles;
    uint32_t i = blockIdx.x;
    uint32_t tile = i < n_idx ? tile_at(a, i) : 0;
    auto load_decode = [&](uint64_t tile_word0) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
            const u64x2* base = reinterpret_cast<const u64x2*>(s.dleaf[m] + tile_word0);
#pragma unroll
            for (int p = 0; p < PAIRS; ++p) dv[m][p] = __builtin_nontemporal_load(base + p * THREADS + t);
        }
    };
    if (i < n_idx) {
        load_tile<K, PAIRS, THREADS>(a, (uint64_t)tile * TILE_WORDS, t, v);
        load_decode((uint64_t)tile * TILE_WORDS);
    }
    while (i < n_idx) {
        const uint64_t tile_word0 = (uint64_t)tile * TILE_WORDS;
        const bool has_next = i + gridDim.x < n_idx;
        const uint32_t next = has_next ? tile_at(a, i + gridDim.x) : 0;
        // (read at the gathers, behind the "stage complete" barrier; the previous tile's gathers
        // finished behind the barrier that ends its iteration)
        if (s.a_bytes) stage_groups(tile_word0 * 64);
        uint64_t r[NW];
        eval_words<K, NW, FORM>(a.prog, v, r);
        tail_mask<NW, THREADS>(a, tile_word0, t, r);
        if (has_next) load_tile<K, PAIRS, THREADS>(a, (uint64_t)next * TILE_WORDS, t, v);
        uint64_t packed = 0;
#pragma unroll
        for (int p = 0; p < PAIRS; ++p)
            packed |= (uint64_t)(__popcll(r[2 * p]) + __popcll(r[2 * p + 1])) << (FB * (p % FPW));
        const uint64_t incl = wave_incl_scan(packed, lane);
        if (lane == 63) s_wave_tot[wave] = incl;
        __syncthreads();
        uint64_t wp = 0, bt = 0;
#pragma unroll
        for (int w = 0; w < NWAVES; ++w) {
            const uint64_t x = s_wave_tot[w];
            if (w < wave) wp += x;
            bt += x;
        }
        uint64_t pair_off[PAIRS];
        uint64_t tile_count = 0;
#pragma unroll
        for (int p = 0; p < PAIRS; ++p) {
            pair_off[p] = tile_count + (((wp + incl - packed) >> (FB * (p % FPW))) & FMASK);
            tile_count += (bt >> (FB * (p % FPW))) & FMASK;
        }
        total += tile_count;
        const int64_t row0 = a.row_base + (int64_t)(tile_word0 * 64);
        const bool staged = tile_count <= (uint64_t)STAGE;
#pragma unroll
        for (int p = 0; p < PAIRS; ++p) {
            uint32_t off = (uint32_t)pair_off[p];
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                uint64_t w = r[2 * p + e];
                const uint32_t wrow = (uint32_t)((p * 2 * THREADS + 2 * t + e) * 64);
                while (w) {
                    const uint32_t b = (uint32_t)__builtin_ctzll(w);
                    uint32_t miss = 0;  // bit m: the row is not in decode leaf m (b >= v_{m+1})
#pragma unroll
                    for (int m = 0; m < M; ++m) {
                        const u64x2 d = dv[m][p];
                        const uint64_t dw = e ? d.y : d.x;
                        miss |= (uint32_t)(((dw >> b) & 1ull) ^ 1ull) << m;
                    }
                    if (staged) {
                        s_row[off] = (wrow + b) | (miss << kMissShift);
                    } else {
                        accumulate(row0 + (int64_t)(wrow + b), decoded_b(miss));  // dense tile: direct
                    }
                    ++off;
                    w &= w - 1;
                }
            }
        }
        if (M > 0 && has_next) load_decode((uint64_t)next * TILE_WORDS);
        __syncthreads();  // stage complete
        if (staged) {
            // 4 gathers in flight per thread per round
            for (uint32_t i = t; i < (uint32_t)tile_count; i += 4 * THREADS) {
                int64_t av[4], bvv[4];
                bool ok[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const uint32_t k = i + u * THREADS;
                    ok[u] = k < (uint32_t)tile_count;
                    const uint32_t sr = ok[u] ? s_row[k] : 0u;
                    const uint64_t rr = (uint64_t)(row0 - a.row_base) + (sr & ((1u << kMissShift) - 1));
                    // line-granular gathers, no reuse: nontemporal like the leaf loads
                    av[u] = ok[u] ? load_a(rr) : 0;
                    bvv[u] = M > 0 ? (ok[u] ? decoded_b(sr >> kMissShift) : 0) : (ok[u] ? __builtin_nontemporal_load(s.b + rr) : 0);
                    if (ok[u] && s.a_valid && !((s.a_valid[rr >> 6] >> (rr & 63)) & 1ull)) ok[u] = false;
                    if (M == 0 && ok[u] && s.b_valid && !((s.b_valid[rr >> 6] >> (rr & 63)) & 1ull)) ok[u] = false;
                }
#pragma unroll
                for (int u = 0; u < 4; ++u)
                    if (ok[u]) add128(acc_lo, acc_hi, (__int128)av[u] * (__int128)bvv[u]);
            }
        }
        __syncthreads();  // stage / wave totals free
        i += gridDim.x;
        tile = next;
    }
    // block reduce of the 128-bit partial sums
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t olo = __shfl_xor(acc_lo, d, 64);
        const int64_t ohi = __shfl_xor(acc_hi, d, 64);
        const uint64_t nlo = acc_lo + olo;
        acc_hi = acc_hi + ohi + (nlo < acc_lo ? 1 : 0);
        acc_lo = nlo;
    }
    __shared__ uint64_t s_lo[NWAVES];
    __shared__ int64_t s_hi[NWAVES];
    if (lane == 0) {
        s_lo[wave] = acc_lo;
        s_hi[wave] = acc_hi;
    }
    __syncthreads();
    if (t == 0) {
        uint64_t lo = 0;
        int64_t hi = 0;
        for (int w = 0; w < NWAVES; ++w) add128(lo, hi, ((__int128)s_hi[w] << 64) | (unsigned __int128)s_lo[w]);
        s.partials[2 * blockIdx.x] = (int64_t)lo;
        s.partials[2 * blockIdx.x + 1] = hi;
        finish_ticket(a.ticket, a.count, total);
    }
}

__global__ __launch_bounds__(256) void sum_product_arrays_kernel(const int64_t* __restrict__ x,
                                                                 const int64_t* __restrict__ y,
                                                                 const uint64_t* __restrict__ d_count, uint64_t max_n,
                                                                 int64_t* __restrict__ partials) {
    __shared__ __int128 s_part[4];
    const uint64_t n = min(*d_count, max_n);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint64_t lo = 0;
    int64_t hi = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        add128(lo, hi, (__int128)x[i] * (__int128)y[i]);
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
        const __int128 tot = s_part[0] + s_part[1] + s_part[2] + s_part[3];
        partials[2 * blockIdx.x] = (int64_t)(uint64_t)tot;
        partials[2 * blockIdx.x + 1] = (int64_t)(tot >> 64);
    }
}

// ------------------------------------------------------------------ row-order pass

// One launch: workgroup w moves the runs of tiles [tpw·w, tpw·w + tpw) to their row-order
// position (tpw = tiles per workgroup, 1..8: at least ~1,024 workgroups when there are tiles
// for them).
// The position is the sum of the run lengths of every earlier tile, which the workgroup
// reads from the directory itself (16 B per tile, L2-resident: ≤ 37 KB at SF100, read with
// every thread's loads in flight), so no separate scan launch and no single-workgroup scan
// precede the copy. The copy keeps four 8-byte loads in flight per thread.
// MODE (scripts/balbench.hip compares them): 0 plain loads and stores, 1 nontemporal loads and
// sc1 (write-through) buffer stores, 2 nontemporal loads and plain stores.
template <int MODE = 0>
__global__ __launch_bounds__(256) void order_runs_kernel(const uint64_t* __restrict__ dir, uint32_t n_tiles,
                                                         uint32_t tpw, const int64_t* __restrict__ src,
                                                         uint64_t capacity, int64_t* __restrict__ dst) {
    constexpr int THREADS = 256;
    __shared__ uint64_t s_part[THREADS / 64];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const uint32_t t0 = blockIdx.x * tpw;
    uint64_t acc = 0;
#pragma unroll 4
    for (uint32_t i = t; i < t0; i += THREADS) acc += dir[2 * i + 1];
    acc = wave_sum(acc);
    if (lane == 0) s_part[wave] = acc;
    __syncthreads();
    uint64_t d = 0;
#pragma unroll
    for (int w = 0; w < THREADS / 64; ++w) d += s_part[w];
    const uint32_t t1 = t0 + tpw < n_tiles ? t0 + tpw : n_tiles;
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    for (uint32_t tile = t0; tile < t1; ++tile) {
        const uint64_t so = dir[2 * tile], n = dir[2 * tile + 1];
        // MODE 1: this tile's destination run through a descriptor from SGPRs (≤ 131,072 ids)
        const uint64_t lim = d < capacity ? min(n, capacity - d) : 0;
        const uintptr_t dp = reinterpret_cast<uintptr_t>(dst + d);
        const uint64_t db = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(dp >> 32)) << 32) |
                            (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)dp);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)db, (short)0, (int)((uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)lim) * 8u), 0x00020000);
        for (uint64_t i = t; i < n; i += 4 * THREADS) {
            int64_t v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint64_t j = i + (uint64_t)u * THREADS;
                v[u] = (j < n && so + j < capacity) ? (MODE ? __builtin_nontemporal_load(src + so + j) : src[so + j]) : 0;
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint64_t j = i + (uint64_t)u * THREADS;
                if (j < n && so + j < capacity && d + j < capacity) {
                    if (MODE == 1)
                        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v[u]), rs, (int)(j * 8u), 0, 16);
                    else
                        dst[d + j] = v[u];
                }
            }
        }
        d += n;
    }
}

// ------------------------------------------------------------------ K0: compare → bitvector

// K0: predicate → bitvector over a raw column, for M keys in one read of the column (M = 1:
// a constant with no index key at query time; M = kMultiKeys: index build — range L(k),
// equality E(k) or bins [k, k2)). A wave handles 64 consecutive words; 16 rows per lane are
// loaded ahead, then every key's predicate is one ballot per word, kept by lane j for word j,
// and each key's 64 words leave as one 512-byte store. Bytes per pass: n·w_c read + M·n/8
// written, instead of M·(n·w_c + n/8). Comparison semantics are TemplatedFilterSelection's
// (column_segment.cpp:261-349): NULL rows never qualify.
// CMP 0..5 = EQ NE LT LE GT GE (CUBIT_CMP_*); 6 = c <= v < c2 (bin of a CUBIT_INDEX_BINS index)
template <int CMP, typename CT>
__device__ __forceinline__ bool cmp_v(CT v, CT c, CT c2) {
    if (CMP == 0) return v == c;
    if (CMP == 1) return v != c;
    if (CMP == 2) return v < c;
    if (CMP == 3) return v <= c;
    if (CMP == 4) return v > c;
    if (CMP == 5) return v >= c;
    return v >= c && v < c2;
}

template <typename T, typename CT, int CMP, int M, int FK = 0>
__global__ __launch_bounds__(256) void compare_bitvectors_kernel(const T* __restrict__ col,
                                                                 const uint64_t* __restrict__ validity,
                                                                 uint64_t n_rows, uint64_t n_words_padded,
                                                                 MultiKeyArgs a) {
    // CT: compare type (int32 when the column and every key fit 32 bits: one VALU compare)
    static_assert(M >= 1 && M <= kMultiKeys, "keys per pass");
    constexpr int JB = 16;
    const int lane = threadIdx.x & 63;
    const uint64_t wave_id = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint64_t n_waves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t w0 = wave_id * 64; w0 < n_words_padded; w0 += n_waves * 64) {
        uint32_t lo[M], hi[M];  // lane j keeps word j of every key
#pragma unroll
        for (int k = 0; k < M; ++k) lo[k] = hi[k] = 0;
        for (int jb = 0; jb < 64; jb += JB) {
            CT v[JB];
            bool ok[JB];
#pragma unroll
            for (int j = 0; j < JB; ++j) {
                const uint64_t row = (w0 + jb + j) * 64 + lane;
                ok[j] = row < n_rows;
                v[j] = ok[j] ? (CT)key_of<FK>(__builtin_nontemporal_load(col + row)) : (CT)0;  // streamed once: nt
                if (validity) ok[j] = ok[j] && ((validity[w0 + jb + j] >> lane) & 1ull);
            }
#pragma unroll
            for (int j = 0; j < JB; ++j) {
                // every key's ballot for word jb + j (uniform, SGPRs), then lane jb + j alone
                // moves them into its registers under the exec mask: per (word, key) one
                // compare and two moves
                // (keys past a.m repeat the last key: the host pads them, their words are not stored)
                const uint64_t okm = __ballot(ok[j]);
                uint64_t b[M];
#pragma unroll
                for (int k = 0; k < M; ++k) {
                    const CT c = (CT)a.c[k], c2 = (CT)a.c2[k];
                    b[k] = __ballot(cmp_v<CMP, CT>(v[j], c, c2)) & okm;
                }
                if (lane == jb + j) {
#pragma unroll
                    for (int k = 0; k < M; ++k) {
                        lo[k] = (uint32_t)b[k];
                        hi[k] = (uint32_t)(b[k] >> 32);
                    }
                }
            }
        }
#pragma unroll
        for (int k = 0; k < M; ++k)
            if (k < (int)a.m) a.out[k][w0 + lane] = ((uint64_t)hi[k] << 32) | lo[k];
    }
}

template <typename T, typename CT, int M, int FK = 0>
hipError_t launch_compare_multi_t(const T* col, const uint64_t* validity, uint64_t n_rows, int cmp,
                                  const MultiKeyArgs& a, hipStream_t stream) {
    const uint64_t nw = padded_words(n_rows);
    const uint64_t waves = nw / 64;
    const uint64_t blocks = std::min<uint64_t>((waves + 3) / 4, 8192);
    const dim3 grid((unsigned)std::max<uint64_t>(blocks, 1)), block(256);
#define CUBIT_CMP_CASE(C)                                                                                       \
    case C:                                                                                                     \
        hipLaunchKernelGGL((compare_bitvectors_kernel<T, CT, C, M, FK>), grid, block, 0, stream, col, validity, n_rows, nw, a); \
        break;
    if constexpr (M == 1) {  // a query-time constant: every comparison
        switch (cmp) {
            CUBIT_CMP_CASE(0)
            CUBIT_CMP_CASE(1)
            CUBIT_CMP_CASE(2)
            CUBIT_CMP_CASE(3)
            CUBIT_CMP_CASE(4)
            CUBIT_CMP_CASE(5)
            CUBIT_CMP_CASE(6)
        default: return hipErrorInvalidValue;
        }
    } else {  // index build: L(k) = v < k, E(k) = v == k, bins k <= v < k2
        switch (cmp) {
            CUBIT_CMP_CASE(0)
            CUBIT_CMP_CASE(2)
            CUBIT_CMP_CASE(6)
        default: return hipErrorInvalidValue;
        }
    }
#undef CUBIT_CMP_CASE
    return hipGetLastError();
}

// Candidate check (binned range index): a query-time constant c that is not an index key
// falls in one bin [k_lo, k_hi) of the range index. Its rows are cand = L(k_hi) \ L(k_lo)
// (L(k) = valid rows with v < k; no k_lo → ∅, no k_hi → every valid row), and only they
// need the raw value:
//   v <  c  =  L(k_lo) ∪ {r ∈ cand : v[r] < c}
//   v == c  =           {r ∈ cand : v[r] == c}
// Per word: two bitvector words read, the column read at the candidate rows only, one word
// written — instead of K0's read of the whole column. Each thread owns two consecutive
// words (16-byte loads and stores), so a wave's bitvector traffic is 1 KiB per instruction;
// the candidate values are gathered per set bit (line-granular reads of the column where a
// line holds a candidate). Comparison semantics are TemplatedFilterSelection's
// (column_segment.cpp:261-349); NULL rows are never candidates.
template <typename T, typename CT, int CMP, int FK = 0>
__global__ __launch_bounds__(256) void candidate_check_kernel(const T* __restrict__ col,
                                                              const uint64_t* __restrict__ validity,
                                                              const uint64_t* __restrict__ lo_bv,
                                                              const uint64_t* __restrict__ hi_bv, uint64_t n_rows,
                                                              uint64_t n_words_padded, CT c,
                                                              uint64_t* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t n_words = (n_rows + 63) / 64;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; 2 * p < n_words_padded; p += stride) {
        const uint64_t w0 = 2 * p;
        u64x2 lo = {0ull, 0ull}, hi;
        if (lo_bv) lo = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(lo_bv) + p);
        if (hi_bv) {
            hi = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(hi_bv) + p);
        } else {
            // every valid row of the partition: full words, the tail word's rows, nothing past it
            hi.x = w0 < n_words ? ~0ull : 0ull;
            hi.y = w0 + 1 < n_words ? ~0ull : 0ull;
            if (w0 + 1 == n_words && (n_rows & 63)) hi.x = (1ull << (n_rows & 63)) - 1;
            if (w0 + 2 == n_words && (n_rows & 63)) hi.y = (1ull << (n_rows & 63)) - 1;
            if (validity) {
                const u64x2 vw = reinterpret_cast<const u64x2*>(validity)[p];
                hi.x &= vw.x;
                hi.y &= vw.y;
            }
        }
        u64x2 res;
        res.x = CMP == 2 ? lo.x : 0ull;
        res.y = CMP == 2 ? lo.y : 0ull;
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            uint64_t cand = e ? (hi.y & ~lo.y) : (hi.x & ~lo.x);
            uint64_t hit = 0;
            const T* base = col + (w0 + e) * 64;
            while (cand) {
                const int b = __builtin_ctzll(cand);
                const CT v = (CT)key_of<FK>(base[b]);
                if (CMP == 2 ? v < c : v == c) hit |= 1ull << b;
                cand &= cand - 1;
            }
            if (e) res.y |= hit;
            else res.x |= hit;
        }
        reinterpret_cast<u64x2*>(out)[p] = res;
    }
}

// Selection narrowing: RowGroup::TemplatedScan evaluates each filter column after the first
// only at the rows the earlier ones kept (ColumnData::Select over the shared SelectionVector,
// row_group.cpp:537-550). For a constant comparison on a column without a usable index inside a
// conjunction: out = mask ∩ valid ∩ {r : lo <= v[r] <= hi, complemented when neg}, the column
// read only at the mask's rows (line-granular gathers, as the candidate check). Each thread owns
// two consecutive words (16-byte loads and stores).
template <typename T, int FK = 0>
__global__ __launch_bounds__(256) void masked_compare_kernel(const T* __restrict__ col,
                                                             const uint64_t* __restrict__ validity,
                                                             const uint64_t* __restrict__ mask, uint64_t n_words_padded,
                                                             T lo, T hi, int neg, uint64_t* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; 2 * p < n_words_padded; p += stride) {
        const uint64_t w0 = 2 * p;
        u64x2 m = reinterpret_cast<const u64x2*>(mask)[p];
        if (validity) {
            const u64x2 vw = reinterpret_cast<const u64x2*>(validity)[p];
            m.x &= vw.x;
            m.y &= vw.y;
        }
        u64x2 res = {0ull, 0ull};
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            uint64_t cand = e ? m.y : m.x;
            uint64_t hit = 0;
            const T* base = col + (w0 + e) * 64;
            while (cand) {
                const int b = __builtin_ctzll(cand);
                const T v = key_of<FK>(base[b]);
                if (((v >= lo) & (v <= hi)) != (neg != 0)) hit |= 1ull << b;
                cand &= cand - 1;
            }
            if (e) res.y = hit;
            else res.x = hit;
        }
        reinterpret_cast<u64x2*>(out)[p] = res;
    }
}

template <typename T, typename CT, int FK = 0>
hipError_t launch_candidate_t(const T* col, const uint64_t* validity, const uint64_t* lo_bv, const uint64_t* hi_bv,
                              uint64_t n_rows, int cmp, CT c, uint64_t* out, hipStream_t stream) {
    const uint64_t nw = padded_words(n_rows);
    const dim3 grid((unsigned)std::min<uint64_t>((nw / 2 + 255) / 256, 8192)), block(256);
    if (cmp == 2)
        hipLaunchKernelGGL((candidate_check_kernel<T, CT, 2, FK>), grid, block, 0, stream, col, validity, lo_bv, hi_bv,
                           n_rows, nw, c, out);
    else if (cmp == 0)
        hipLaunchKernelGGL((candidate_check_kernel<T, CT, 0, FK>), grid, block, 0, stream, col, validity, lo_bv, hi_bv,
                           n_rows, nw, c, out);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// every key (and bin end) an int32: an int32 column compares in 32 bits
bool keys_fit32(const MultiKeyArgs& a, int cmp) {
    for (uint32_t k = 0; k < a.m; ++k)
        if (a.c[k] < INT32_MIN || a.c[k] > INT32_MAX ||
            (cmp == kCmpBetween && (a.c2[k] < INT32_MIN || a.c2[k] > INT32_MAX)))
            return false;
    return true;
}

template <int M>
hipError_t launch_compare_m(const void* col, int type, const uint64_t* validity, uint64_t n_rows, int cmp,
                            const MultiKeyArgs& a, hipStream_t stream) {
    // FLOAT / DOUBLE: the patterns' keys (FLOAT keys are int32, so are the planner's keys for it)
    if (type == kTypeFloat)
        return keys_fit32(a, cmp) ? launch_compare_multi_t<int32_t, int32_t, M, 1>(static_cast<const int32_t*>(col),
                                                                                   validity, n_rows, cmp, a, stream)
                                  : launch_compare_multi_t<int32_t, int64_t, M, 1>(static_cast<const int32_t*>(col),
                                                                                   validity, n_rows, cmp, a, stream);
    if (type == kTypeDouble)
        return launch_compare_multi_t<int64_t, int64_t, M, 2>(static_cast<const int64_t*>(col), validity, n_rows, cmp, a,
                                                              stream);
    if (type == kTypeUInt64) {
        // the keys v ^ 2^63 order as the raw values do unsigned: un-key the constants once and
        // compare the 64 bits unsigned (no per-value XOR in the loop)
        MultiKeyArgs u = a;
        for (int k = 0; k < kMultiKeys; ++k) {
            u.c[k] = (int64_t)((uint64_t)u.c[k] ^ 0x8000000000000000ull);
            u.c2[k] = (int64_t)((uint64_t)u.c2[k] ^ 0x8000000000000000ull);
        }
        return launch_compare_multi_t<uint64_t, uint64_t, M>(static_cast<const uint64_t*>(col), validity, n_rows, cmp, u,
                                                             stream);
    }
    if (type_is32(type) && keys_fit32(a, cmp))
        return launch_compare_multi_t<int32_t, int32_t, M>(static_cast<const int32_t*>(col), validity, n_rows, cmp, a,
                                                           stream);
    if (type_is32(type))
        return launch_compare_multi_t<int32_t, int64_t, M>(static_cast<const int32_t*>(col), validity, n_rows, cmp, a,
                                                           stream);
    return launch_compare_multi_t<int64_t, int64_t, M>(static_cast<const int64_t*>(col), validity, n_rows, cmp, a,
                                                       stream);
}

// ------------------------------------------------------------------ index build: column stats

// min / max / any-valid of a column (the statistics an index build needs; the reference
// keeps them per segment as BaseStatistics, used by CheckZonemap, row_group.cpp:361-371).
// out[0] = min, out[1] = max (pre-set to INT64_MAX / INT64_MIN), out[2] = valid rows.
template <typename T, int FK = 0>
__global__ __launch_bounds__(256) void column_minmax_kernel(const T* __restrict__ col,
                                                            const uint64_t* __restrict__ validity, uint64_t n,
                                                            int64_t* __restrict__ out) {
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    uint64_t cnt = 0;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (validity && !((validity[i >> 6] >> (i & 63)) & 1ull)) continue;
        const int64_t v = (int64_t)key_of<FK>(col[i]);
        mn = v < mn ? v : mn;
        mx = v > mx ? v : mx;
        ++cnt;
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const int64_t a = __shfl_xor(mn, d, 64), b = __shfl_xor(mx, d, 64);
        mn = a < mn ? a : mn;
        mx = b > mx ? b : mx;
        cnt += __shfl_xor(cnt, d, 64);
    }
    if ((threadIdx.x & 63) == 0 && cnt) {
        atomicMin(reinterpret_cast<long long*>(out), (long long)mn);
        atomicMax(reinterpret_cast<long long*>(out + 1), (long long)mx);
        atomicAdd(reinterpret_cast<unsigned long long*>(out + 2), (unsigned long long)cnt);
    }
}

// presence bitmap of the valid values: bit (v - vmin) of `bits`. Narrow ranges (≤ 2^16
// values) collect in LDS first so the few global words are OR-ed once per workgroup.
template <typename T, bool LDS, int FK = 0>
__global__ __launch_bounds__(256) void presence_kernel(const T* __restrict__ col, const uint64_t* __restrict__ validity,
                                                       uint64_t n, int64_t vmin, uint64_t range,
                                                       uint64_t* __restrict__ bits) {
    __shared__ uint64_t s_bits[LDS ? 1024 : 1];
    const uint64_t nw = (range + 63) / 64;
    if (LDS) {
        for (uint64_t w = threadIdx.x; w < nw; w += blockDim.x) s_bits[w] = 0;
        __syncthreads();
    }
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (validity && !((validity[i >> 6] >> (i & 63)) & 1ull)) continue;
        const uint64_t off = (uint64_t)((int64_t)key_of<FK>(col[i]) - vmin);
        const uint64_t bit = 1ull << (off & 63);
        if (LDS) {
            if (!(s_bits[off >> 6] & bit)) atomicOr(reinterpret_cast<unsigned long long*>(&s_bits[off >> 6]), bit);
        } else {
            atomicOr(reinterpret_cast<unsigned long long*>(&bits[off >> 6]), bit);
        }
    }
    if (LDS) {
        __syncthreads();
        for (uint64_t w = threadIdx.x; w < nw; w += blockDim.x)
            if (s_bits[w]) atomicOr(reinterpret_cast<unsigned long long*>(&bits[w]), s_bits[w]);
    }
}

// ------------------------------------------------------------------ K5: bit-unpack

// One workgroup per DuckDB bitpacking metadata group (BitpackingScanPartial,
// bitpacking.cpp:785-868): CONSTANT, CONSTANT_DELTA (first + i·delta), FOR (unpacked + min)
// and DELTA_FOR (running sum of unpacked + min_delta from delta_offset, a block scan here).
// Packed values are horizontal (fastpforlib fastpack): value i at bits [i·w, (i+1)·w) of
// little-endian 32-bit words. The group's packed words (≤ 2,048·64 bits = 16 KiB) are staged
// in LDS with coalesced loads; thread t then owns the 4-value quads t and t + 256 (values
// 4t..4t+3 and 1024+4t..1024+4t+3), so every wave store is a contiguous 16 B per lane
// (HBM-write-bound: the output is 4–8 B per value, the input w/8). U = unsigned T, the
// reference's wrap-around arithmetic.
constexpr uint32_t kBpMaxWords = 2048 * 64 / 32;  // packed 32-bit words of a 64-bit-wide group

typedef uint32_t bp_u32x4 __attribute__((ext_vector_type(4)));

// The 16-byte-aligned span of a FOR / DELTA_FOR group's packed words (they start 4-aligned; the
// upload pads the bytes by 16): nvec dwordx4 from byte a0, word 0 at s_words[sh]. CONSTANT
// groups have no span.
struct BpSpan {
    uint64_t a0;
    uint32_t sh, nvec;
};
__device__ __forceinline__ BpSpan bp_span(const BpGroup& g) {
    BpSpan sp{0, 0, 0};
    if (g.mode == 4 || g.mode == 5) {
        const uint32_t nwords = (g.count + 31) / 32 * g.width;  // validated on the host against the bytes
        sp.a0 = g.words_off & ~15ull;
        sp.sh = (uint32_t)(g.words_off - sp.a0) / 4;
        sp.nvec = (sp.sh + nwords + 3) / 4;
    }
    return sp;
}

// Unpack one group with 256 threads: thread t produces the 4-value quads t and t + 256 (values
// 4t..4t+3 and 1024+4t..1024+4t+3) and hands each to store_quad(c, v) (c = 0, 1). s_words
// (kBpMaxWords + 8 words, 16-byte aligned) stages the packed words, s_tot holds wave totals.
// STAGED: the caller already landed the group's span in s_words (and synchronised).
template <typename T, typename U, bool STAGED = false, typename Store>
__device__ __forceinline__ void unpack_group(const uint8_t* __restrict__ bytes, const BpGroup& g, uint32_t* s_words,
                                             U* s_tot, Store&& store_quad) {
    constexpr int THREADS = 256, QUADS = 2;
    const int t = threadIdx.x;
    if (g.mode == 2 || g.mode == 3) {  // CONSTANT, CONSTANT_DELTA
        const U base = (U)g.base, d = g.mode == 3 ? (U)g.aux : (U)0;
#pragma unroll
        for (int c = 0; c < QUADS; ++c) {
            U v[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = bp_norm<U>((U)(d * (U)(4u * (uint32_t)(t + THREADS * c) + j) + base), g.tnorm);
            store_quad(c, v);
        }
        return;
    }
    const U fr = (U)g.base;
    const uint32_t w = g.width;
    const bool delta = g.mode == 4;
    const U doff = delta ? (U)g.aux : (U)0;
    // packed words start 4-aligned: stage the 16-byte-aligned span that covers them with
    // dwordx4 loads (the upload pads the bytes by 16), word 0 lands at s_words[sh]
    const BpSpan sp = bp_span(g);
    const uint32_t sh = sp.sh;
    if (!STAGED) {
        const bp_u32x4* src = reinterpret_cast<const bp_u32x4*>(bytes + sp.a0);
        bp_u32x4* sw = reinterpret_cast<bp_u32x4*>(s_words);
        for (uint32_t i = t; i < sp.nvec; i += THREADS) sw[i] = __builtin_nontemporal_load(src + i);
        // (a value's window may read one word past its last bit: those bits are masked off)
        __syncthreads();
    }
    U v[QUADS][4];
#pragma unroll
    for (int c = 0; c < QUADS; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t i = 4u * (uint32_t)(t + THREADS * c) + j;
            uint64_t x = 0;
            if (w && i < g.count) {
                const uint64_t bit = (uint64_t)i * w;
                const uint32_t wi = (uint32_t)(bit >> 5), off = (uint32_t)(bit & 31);
                x = ((uint64_t)s_words[sh + wi] | (uint64_t)s_words[sh + wi + 1] << 32) >> off;
                if (off + w > 64) x |= (uint64_t)s_words[sh + wi + 2] << (64 - off);
                if (w < 64) x &= (1ull << w) - 1;
            }
            v[c][j] = bp_norm<U>((U)x + fr, g.tnorm);
        }
    if (!delta) {
#pragma unroll
        for (int c = 0; c < QUADS; ++c) store_quad(c, v[c]);
        return;
    }
    // DELTA_FOR: inclusive prefix over the group in value order: quad c = 0 covers values
    // 0..1023, c = 1 covers 1024..2047 (carry = the first half's total). Values past count add 0.
    const int lane = t & 63, wave = t >> 6;
    U carry = doff;
#pragma unroll
    for (int c = 0; c < QUADS; ++c) {
        U run = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (4u * (uint32_t)(t + THREADS * c) + j >= g.count) v[c][j] = 0;
            run += v[c][j];
            v[c][j] = run;
        }
        U incl = run;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const U y = (U)__shfl_up((uint64_t)incl, d, 64);
            if (lane >= d) incl += y;
        }
        if (lane == 63) s_tot[wave] = incl;
        __syncthreads();
        U pre = carry + incl - run, tot = 0;
#pragma unroll
        for (int w2 = 0; w2 < THREADS / 64; ++w2) {
            if (w2 < wave) pre += s_tot[w2];
            tot += s_tot[w2];
        }
        __syncthreads();  // s_tot is rewritten by the next half
        carry += tot;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[c][j] = bp_norm<U>(v[c][j] + pre, g.tnorm);
        store_quad(c, v[c]);
    }
}

template <typename T, typename U>
__global__ __launch_bounds__(256) void bitunpack_kernel(const uint8_t* __restrict__ bytes,
                                                        const BpGroup* __restrict__ groups, T* __restrict__ out) {
    constexpr int THREADS = 256;
    __shared__ __attribute__((aligned(16))) uint32_t s_words[kBpMaxWords + 8];  // + alignment shift + 3-word window
    __shared__ U s_tot[THREADS / 64];
    const BpGroup g = groups[blockIdx.x];
    const int t = threadIdx.x;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    // 4-byte values leave through a descriptor over dst[0, count) built from SGPRs, as sc1
    // (write-through) 16-byte buffer stores — the store policy the decode's copy-out measured
    // fastest (emit_ids, profiles/r02e_balbench_cache_policy.txt); each store instruction then
    // covers 1 KiB contiguously
    T* dst = out + g.row_start;
    const uintptr_t dp = reinterpret_cast<uintptr_t>(dst);
    const uint64_t db = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(dp >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)dp);
    const uint32_t cnt = (uint32_t)__builtin_amdgcn_readfirstlane(g.count);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)db, (short)0, (int)(cnt * (uint32_t)sizeof(T)), 0x00020000);
    // store quad c of this thread: values 4·(t + 256c) + 0..3
    unpack_group<T, U>(bytes, g, s_words, s_tot, [&](int c, const U (&v)[4]) {
        const uint32_t i0 = 4u * (uint32_t)(t + THREADS * c);
        if (sizeof(T) == 8 && cnt == 2048u) {
            // 8-byte values of a full group (uniform; store_quad runs with every lane active): a
            // wave's 256 values are 2 KiB, lane l owns bytes [32l, 32l + 32). Two lane exchanges
            // make each store instruction cover 1 KiB contiguously — lane l writes wave values
            // 2l, 2l + 1 (from lane l/2) and 128 + 2l, 129 + 2l (from lane 32 + l/2) — so the
            // stores can be sc1 (write-through) without half-line writes
            const int lane = t & 63;
            const bool odd = (lane & 1) != 0;
            const uint32_t wbase = 32u * (uint32_t)(THREADS * c + (t & ~63));
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int src = 32 * h + (lane >> 1);
                const unsigned long long e0 = __shfl((unsigned long long)(uint64_t)v[0], src, 64);
                const unsigned long long e1 = __shfl((unsigned long long)(uint64_t)v[1], src, 64);
                const unsigned long long f0 = __shfl((unsigned long long)(uint64_t)v[2], src, 64);
                const unsigned long long f1 = __shfl((unsigned long long)(uint64_t)v[3], src, 64);
                u64x2 o;
                o.x = odd ? f0 : e0;
                o.y = odd ? f1 : e1;
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rs, (int)(wbase + 1024u * h + 16u * lane),
                                                       0, 16);
            }
            return;
        }
        if (i0 + 4 <= cnt) {
            if (sizeof(T) == 4) {
                u32x4 o;
                o.x = (uint32_t)v[0], o.y = (uint32_t)v[1], o.z = (uint32_t)v[2], o.w = (uint32_t)v[3];
                __builtin_amdgcn_raw_buffer_store_b128(o, rs, (int)(i0 * 4u), 0, 16);
            } else {
                // 8-byte values of a partial group: a lane's quad is 32 bytes, so each store
                // instruction covers every other 16 bytes; write-through (sc1) of those half lines
                // measured 3.3 ms instead of 1.0 ms for l_discount, so these stay plain
                u64x2 o0, o1;
                o0.x = (uint64_t)v[0], o0.y = (uint64_t)v[1], o1.x = (uint64_t)v[2], o1.y = (uint64_t)v[3];
                reinterpret_cast<u64x2*>(dst + i0)[0] = o0;
                reinterpret_cast<u64x2*>(dst + i0)[1] = o1;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (i0 + j >= cnt) continue;
                if (sizeof(T) == 4)
                    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v[j], rs, (int)((i0 + j) * 4u), 0, 16);
                else
                    dst[i0 + j] = (T)v[j];
            }
        }
    });
}

// Filter straight from DuckDB BITPACKING segments (the reference's ColumnSegment::Scan →
// BitpackingScanPartial → ColumnSegment::FilterSelection chain, column_segment.cpp:378-522 /
// bitpacking.cpp:779-868, for one constant comparison). The comparison arrives as an inclusive
// range: p = (lo <= v <= hi) XOR neg (the host maps = != < <= > >= and between onto it, clamped
// to T), so testing a value is branch-free. A workgroup takes GPW consecutive groups and lands
// every group's header and packed span in LDS at once, so one load round trip covers GPW
// groups (a group is ~3 KB at 12 bits per value: one group per workgroup waited on its round
// trip). Then, group by group (not unrolled: the code stays small enough for the instruction
// cache — the fully unrolled version ran 18,800 instructions and a quarter of the bandwidth),
// thread t tests values t, t + 256, …, so a wave's 64 consecutive values are one ballot = one
// 64-row bitvector word. A FOR value of ≤ 32 bits comes straight from the staged words (one
// funnel shift); DELTA_FOR and wider FOR groups are unpacked into LDS values first, as
// bitunpack_kernel does. NULL rows never pass (validity, optional). Words wholly inside the
// group are stored; a word a group shares with its neighbour (a group whose rows do not start
// or end on a 64-row boundary) is OR-ed atomically, so `out` must be zero beforehand. Reads
// w/8 bytes per row instead of the plain column's sizeof(T).
template <typename T, typename U, int GPW>
__global__ __launch_bounds__(256) void bitpacked_compare_kernel(const uint8_t* __restrict__ bytes,
                                                                const BpGroup* __restrict__ groups, uint32_t n_groups,
                                                                const uint64_t* __restrict__ validity, T lo, T hi,
                                                                int neg, uint64_t* __restrict__ out) {
    constexpr int THREADS = 256;
    // a group's span: ≤ 2,048·8·sizeof(T) bits + the alignment shift + a 3-word read window
    constexpr uint32_t SPANW = 2048u * 8u * (uint32_t)sizeof(T) / 32u + 8u;
    constexpr int VECS = (int)((SPANW / 4 + THREADS - 1) / THREADS);
    static_assert(sizeof(BpGroup) % 4 == 0, "headers copied as words");
    constexpr int HDRW = (int)(sizeof(BpGroup) / 4);
    __shared__ __attribute__((aligned(16))) uint32_t s_words[GPW][SPANW];
    __shared__ __attribute__((aligned(16))) T s_vals[2048];
    __shared__ U s_tot[THREADS / 64];
    __shared__ BpGroup s_hdr[GPW];
    const int t = threadIdx.x;
    const int lane = t & 63;
    const uint32_t wave_u = __builtin_amdgcn_readfirstlane((uint32_t)(t >> 6));
    const uint32_t g0 = blockIdx.x * (uint32_t)GPW;
    const uint32_t ng = min((uint32_t)GPW, n_groups - g0);
    // headers (as words) and spans: every load issued before any lands
    {
        const uint32_t* hsrc = reinterpret_cast<const uint32_t*>(groups + g0);
        uint32_t hw = 0;
        if (t < (int)(ng * HDRW)) hw = hsrc[t];
        BpGroup hg[GPW];
        bp_u32x4 pf[GPW][VECS];
#pragma unroll
        for (int q = 0; q < GPW; ++q) {
            if ((uint32_t)q < ng) {
                hg[q] = groups[g0 + q];
                const BpSpan sp = bp_span(hg[q]);
                const bp_u32x4* src = reinterpret_cast<const bp_u32x4*>(bytes + sp.a0);
#pragma unroll
                for (int k = 0; k < VECS; ++k) {
                    const uint32_t i = (uint32_t)(t + THREADS * k);
                    if (i < sp.nvec) pf[q][k] = src[i];
                }
            }
        }
        if (t < (int)(ng * HDRW)) reinterpret_cast<uint32_t*>(s_hdr)[t] = hw;
#pragma unroll
        for (int q = 0; q < GPW; ++q) {
            if ((uint32_t)q < ng) {
                const BpSpan sp = bp_span(hg[q]);
                bp_u32x4* sw = reinterpret_cast<bp_u32x4*>(s_words[q]);
#pragma unroll
                for (int k = 0; k < VECS; ++k) {
                    const uint32_t i = (uint32_t)(t + THREADS * k);
                    if (i < sp.nvec) sw[i] = pf[q][k];
                }
            }
        }
    }
    __syncthreads();
#pragma unroll 1
    for (uint32_t q = 0; q < ng; ++q) {
        const BpGroup cur = s_hdr[q];
        const uint32_t* W = s_words[q];
        const uint64_t end = cur.row_start + cur.count;
        // test values t, t + 256, …: the chunk's first value and row are wave-uniform
        auto test_and_store = [&](auto&& value_of) {
#pragma unroll 1
            for (uint32_t i0 = 64u * wave_u; i0 < cur.count; i0 += 256u) {
                const uint32_t i = i0 + (uint32_t)lane;
                bool p = false;
                if (i < cur.count) {
                    const T v = value_of(i);
                    p = ((v >= lo) & (v <= hi)) != (neg != 0);
                    if (validity) {
                        const uint64_t r = cur.row_start + i;
                        p = p && ((validity[r >> 6] >> (r & 63)) & 1ull);
                    }
                }
                const uint64_t bits = __ballot(p);
                const uint64_t r0 = cur.row_start + i0;  // row of bit 0 (uniform)
                const uint32_t sh = (uint32_t)(r0 & 63);
                const uint64_t w0 = r0 >> 6;
                if (lane == 0) {
                    if (sh == 0) {
                        if (r0 + 64 <= end) out[w0] = bits;  // only this group's rows
                        else atomicOr(reinterpret_cast<unsigned long long*>(&out[w0]), (unsigned long long)bits);
                    } else {
                        atomicOr(reinterpret_cast<unsigned long long*>(&out[w0]), (unsigned long long)(bits << sh));
                        const uint64_t hi2 = bits >> (64 - sh);
                        if (hi2) atomicOr(reinterpret_cast<unsigned long long*>(&out[w0 + 1]), (unsigned long long)hi2);
                    }
                }
            }
        };
        if (cur.mode == 5 && cur.width <= 32) {
            // FOR, w ≤ 32: one funnel shift of the two words a value's bits span, a mask, the
            // frame of reference
            const uint32_t w = cur.width, sh = bp_span(cur).sh;
            const uint32_t mask = w == 32 ? ~0u : (1u << w) - 1u;
            const U fr = (U)cur.base;
            test_and_store([&](uint32_t i) -> T {
                const uint32_t bit = i * w, wi = sh + (bit >> 5);  // i·w < 2^16
                const uint32_t x = __builtin_amdgcn_alignbit(W[wi + 1], W[wi], bit & 31) & mask;
                return (T)bp_norm<U>((U)x + fr, cur.tnorm);
            });
        } else if (cur.mode == 2 || cur.mode == 3) {  // CONSTANT, CONSTANT_DELTA: no packed words
            const U base = (U)cur.base, d = cur.mode == 3 ? (U)cur.aux : (U)0;
            test_and_store([&](uint32_t i) -> T { return (T)bp_norm<U>(d * (U)i + base, cur.tnorm); });
        } else {
            // DELTA_FOR (a running sum) or FOR wider than 32 bits: unpack into LDS values first
            unpack_group<T, U, true>(bytes, cur, const_cast<uint32_t*>(W), s_tot, [&](int qq, const U (&v)[4]) {
                const uint32_t i0 = 4u * (uint32_t)(t + THREADS * qq);
                if (sizeof(T) == 4) {
                    bp_u32x4 o;
                    o.x = (uint32_t)v[0], o.y = (uint32_t)v[1], o.z = (uint32_t)v[2], o.w = (uint32_t)v[3];
                    *reinterpret_cast<bp_u32x4*>(&s_vals[i0]) = o;
                } else {
                    u64x2 o0, o1;
                    o0.x = (uint64_t)v[0], o0.y = (uint64_t)v[1], o1.x = (uint64_t)v[2], o1.y = (uint64_t)v[3];
                    reinterpret_cast<u64x2*>(&s_vals[i0])[0] = o0;
                    reinterpret_cast<u64x2*>(&s_vals[i0])[1] = o1;
                }
            });
            __syncthreads();  // values complete
            test_and_store([&](uint32_t i) -> T { return s_vals[i]; });
            __syncthreads();  // s_vals free for the next group
        }
    }
}

// One group's 64-row output words from its values (a FOR group's packed words staged in L,
// CONSTANT / CONSTANT_DELTA from its record): 64 values per step, each lane taking its value's
// bits from the staged words with one funnel shift, one ballot per step = one output word
// (bitpacked_compare_waves).
template <typename T, typename U>
__device__ __forceinline__ void compare_group_words(const BpGroup& cur, const uint32_t* L, bool packed, uint32_t w,
                                                    uint32_t mask, int lane, const uint64_t* __restrict__ validity,
                                                    T lo, T hi, int neg, uint64_t* __restrict__ out) {
    const uint64_t end = cur.row_start + cur.count;
    const U base = (U)cur.base, d = cur.mode == 3 ? (U)cur.aux : (U)0;
    const uint32_t nchunks = (cur.count + 63u) / 64u;  // ≤ 32
    // a group starting on a 64-row boundary keeps step c's word in lane c and stores the words
    // together at the end (one coalesced store; 8-byte stores from lane 0, one per step, cost
    // more than the whole read); other groups store or OR each word as it is made
    const bool aligned = (cur.row_start & 63) == 0;
    uint64_t myword = 0;
    for (uint32_t c = 0; c < nchunks; ++c) {
        const uint32_t i = c * 64u + (uint32_t)lane;
        bool p = false;
        if (i < cur.count) {
            T v;
            if (packed) {
                const uint32_t bit = i * w, wi = bit >> 5;  // i·w < 2^16
                v = (T)bp_norm<U>((U)(__builtin_amdgcn_alignbit(L[wi + 1], L[wi], bit & 31) & mask) + base, cur.tnorm);
            } else {
                v = (T)bp_norm<U>(d * (U)i + base, cur.tnorm);
            }
            p = ((v >= lo) & (v <= hi)) != (neg != 0);
            if (validity) {
                const uint64_t r = cur.row_start + i;
                p = p && ((validity[r >> 6] >> (r & 63)) & 1ull);
            }
        }
        const uint64_t bits = __ballot(p);
        if (aligned) {
            if ((uint32_t)lane == c) myword = bits;
            continue;
        }
        const uint64_t r0 = cur.row_start + 64ull * c;  // row of bit 0 (uniform)
        const uint32_t sh = (uint32_t)(r0 & 63);
        const uint64_t w0 = r0 >> 6;
        if (lane == 0) {
            if (sh == 0) {
                if (r0 + 64 <= end) out[w0] = bits;  // only this group's rows
                else atomicOr(reinterpret_cast<unsigned long long*>(&out[w0]), (unsigned long long)bits);
            } else {
                atomicOr(reinterpret_cast<unsigned long long*>(&out[w0]), (unsigned long long)(bits << sh));
                const uint64_t hi2 = bits >> (64 - sh);
                if (hi2) atomicOr(reinterpret_cast<unsigned long long*>(&out[w0 + 1]), (unsigned long long)hi2);
            }
        }
    }
    if (aligned && (uint32_t)lane < nchunks) {
        const uint64_t r0 = cur.row_start + 64ull * (uint32_t)lane;
        if (r0 + 64 <= end) out[r0 >> 6] = myword;  // only this group's rows
        else atomicOr(reinterpret_cast<unsigned long long*>(&out[r0 >> 6]), (unsigned long long)myword);
    }
}

// The same filter for columns whose groups are all FOR of ≤ MAXW bits (MAXW ≤ 32), CONSTANT or
// CONSTANT_DELTA (the modes DuckDB's AUTO picks for unsorted integer columns): one wave per group.
// The wave lands its group's packed words in its own LDS slice with coalesced 256-byte loads — all
// of them in flight at once (≤ MAXW per lane), one round trip per group — then tests 64 values per
// step, each lane taking its value's bits from the staged words with one funnel shift. One ballot
// per step = one 64-row output word, stored (or OR-ed where a group's rows share the word with a
// neighbour) by lane 0, as in bitpacked_compare_kernel. Measured before (profiles/r03w_*): the
// same wave layout loading each value's two words from global memory, eight 64-value steps in
// flight: 0.650 ms for a 600 M-row 12-bit column (the LDS kernel above 0.93 ms, K0 0.43 ms).
template <typename T, typename U, int MAXW>
__global__ __launch_bounds__(256) void bitpacked_compare_waves(const uint8_t* __restrict__ bytes,
                                                               const BpGroup* __restrict__ groups, uint32_t n_groups,
                                                               const uint64_t* __restrict__ validity, T lo, T hi,
                                                               int neg, uint64_t* __restrict__ out) {
    static_assert(MAXW >= 1 && MAXW <= 32, "FOR groups of at most 32 bits");
    constexpr uint32_t SLICE = 64u * MAXW + 4u;  // a group's words (2,048·w/32) + the read window
    __shared__ uint32_t s_w[4][SLICE];
    const int lane = threadIdx.x & 63;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const uint32_t g = blockIdx.x * 4u + wave;
    if (g >= n_groups) return;  // no workgroup barrier below: each wave works alone
    uint32_t* L = s_w[wave];
    const BpGroup cur = groups[g];
    const bool packed = cur.mode == 5 && cur.width;
    const uint32_t w = packed ? cur.width : 0u;
    const uint32_t mask = w >= 32 ? ~0u : (1u << w) - 1u;
    const uint32_t nwords = packed ? (cur.count + 31u) / 32u * w : 0u;  // ≤ 64·MAXW (host-checked)
    if (packed) {
        const uint32_t* W = reinterpret_cast<const uint32_t*>(bytes + cur.words_off);
        uint32_t x[MAXW];
#pragma unroll
        for (int m = 0; m < MAXW; ++m) {
            const uint32_t k = 64u * (uint32_t)m + (uint32_t)lane;
            x[m] = k < nwords ? __builtin_nontemporal_load(W + k) : 0u;
        }
#pragma unroll
        for (int m = 0; m < MAXW; ++m) L[64u * (uint32_t)m + (uint32_t)lane] = x[m];
        if (lane < 4) L[64u * MAXW + (uint32_t)lane] = 0u;
        // the wave's own LDS writes, read back by other lanes of the same wave: LDS operations of a
        // wave complete in order, so only the compiler must not move the reads above the writes
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    }
    compare_group_words<T, U>(cur, L, packed, w, mask, lane, validity, lo, hi, neg, out);
}

// ------------------------------------------------------------------ transfer compaction

// out[i] = (int32)(in[i] - offset) for i < min(*d_count, max_n): the DataChunk column of a
// window crosses PCIe at 4 bytes per row when every value of the column lies within 2^31 of the
// offset (the host mirror widens while it fills the chunk). 16-byte loads, 8-byte stores.
// (overflow, optional: set to 1 when some value - offset lies outside int32 — the caller's bound
// did not hold and the compacted copy must not be used)
__global__ __launch_bounds__(256) void narrow_i32_kernel(const int64_t* __restrict__ in, const uint64_t* __restrict__ d_count,
                                                          uint64_t max_n, int64_t offset, int32_t* __restrict__ out,
                                                          uint32_t* __restrict__ overflow) {
    const uint64_t n = min(*d_count, max_n);
    auto fits = [](int64_t d) { return d >= INT32_MIN && d <= INT32_MAX; };
    bool bad = false;
    for (uint64_t i = 2 * ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x); i < n; i += 2ull * gridDim.x * blockDim.x) {
        if (i + 1 < n) {
            const u64x2 v = *reinterpret_cast<const u64x2*>(in + i);
            const int64_t dx = (int64_t)((uint64_t)v.x - (uint64_t)offset), dy = (int64_t)((uint64_t)v.y - (uint64_t)offset);
            bad |= !fits(dx) || !fits(dy);
            typedef int32_t i32x2 __attribute__((ext_vector_type(2)));
            i32x2 o;
            o.x = (int32_t)dx;
            o.y = (int32_t)dy;
            *reinterpret_cast<i32x2*>(out + i) = o;
        } else {
            const int64_t d = (int64_t)((uint64_t)in[i] - (uint64_t)offset);
            bad |= !fits(d);
            out[i] = (int32_t)d;
        }
    }
    if (overflow && bad) *overflow = 1u;
}

// Transfer compaction to 1, 2 or 4 bytes: out[i] = (O)(in[i] - offset) as an unsigned O, for a
// column whose values lie in [offset, offset + 2^(8·sizeof O)); `overflow` set when one does not.
// 8 values per thread per step: four 16-byte loads, and the 8 narrowed values packed into one
// 8-byte (bytes), one 16-byte (halves) or two 16-byte (words) stores, so a wave's store covers
// 512 B – 2 KB contiguously — the shape that matters when `out` is page-locked host memory
// written across PCIe (a wave of scattered 1-byte stores ran the link at ~3 GB/s). `in` and
// `out` 16-byte aligned (launch_narrow_unsigned falls back to the scalar form otherwise).
template <typename O>
__global__ __launch_bounds__(256) void narrow_unsigned_kernel(const int64_t* __restrict__ in,
                                                              const uint64_t* __restrict__ d_count, uint64_t max_n,
                                                              int64_t offset, O* __restrict__ out,
                                                              uint32_t* __restrict__ overflow) {
    const uint64_t n = min(*d_count, max_n);
    constexpr uint64_t kMax = sizeof(O) == 4 ? 0xffffffffull : (1ull << (8 * sizeof(O))) - 1;
    bool bad = false;
    for (uint64_t i = 8 * ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x); i < n; i += 8ull * gridDim.x * blockDim.x) {
        if (i + 8 <= n) {
            const ulonglong2* src = reinterpret_cast<const ulonglong2*>(in + i);
            uint64_t d[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const ulonglong2 v = src[j];
                d[2 * j] = v.x - (uint64_t)offset;
                d[2 * j + 1] = v.y - (uint64_t)offset;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) bad |= d[j] > kMax;
            if constexpr (sizeof(O) == 1) {
                uint64_t p = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j) p |= (d[j] & 0xff) << (8 * j);
                *reinterpret_cast<uint64_t*>(out + i) = p;
            } else if constexpr (sizeof(O) == 2) {
                ulonglong2 p{0, 0};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    p.x |= (d[j] & 0xffff) << (16 * j);
                    p.y |= (d[4 + j] & 0xffff) << (16 * j);
                }
                *reinterpret_cast<ulonglong2*>(out + i) = p;
            } else {
                ulonglong2* dst = reinterpret_cast<ulonglong2*>(out + i);
                dst[0] = ulonglong2{(d[0] & 0xffffffffull) | (d[1] << 32), (d[2] & 0xffffffffull) | (d[3] << 32)};
                dst[1] = ulonglong2{(d[4] & 0xffffffffull) | (d[5] << 32), (d[6] & 0xffffffffull) | (d[7] << 32)};
            }
        } else {
            for (uint64_t k = i; k < n; ++k) {
                const uint64_t d = (uint64_t)in[k] - (uint64_t)offset;
                bad |= d > kMax;
                out[k] = (O)d;
            }
        }
    }
    if (overflow && bad) *overflow = 1u;
}

// Three bytes per value (a column whose range spans < 2^24, e.g. l_extendedprice in cents):
// value k of the output at bytes [3k, 3k + 3), little-endian. 8 values per thread per step,
// packed into three 8-byte stores (a wave's 1.5 KB contiguous). `in` 16-byte and `out` 8-byte
// aligned (launch_narrow_unsigned falls back to byte stores otherwise).
__global__ __launch_bounds__(256) void narrow_u24_kernel(const int64_t* __restrict__ in,
                                                         const uint64_t* __restrict__ d_count, uint64_t max_n,
                                                         int64_t offset, uint8_t* __restrict__ out,
                                                         uint32_t* __restrict__ overflow) {
    const uint64_t n = min(*d_count, max_n);
    constexpr uint64_t kMax = (1ull << 24) - 1;
    bool bad = false;
    for (uint64_t i = 8 * ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x); i < n; i += 8ull * gridDim.x * blockDim.x) {
        if (i + 8 <= n) {
            const ulonglong2* src = reinterpret_cast<const ulonglong2*>(in + i);
            uint64_t d[8];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const ulonglong2 v = src[j];
                d[2 * j] = v.x - (uint64_t)offset;
                d[2 * j + 1] = v.y - (uint64_t)offset;
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                bad |= d[j] > kMax;
                d[j] &= kMax;
            }
            uint64_t* dst = reinterpret_cast<uint64_t*>(out + 3 * i);
            dst[0] = d[0] | (d[1] << 24) | (d[2] << 48);
            dst[1] = (d[2] >> 16) | (d[3] << 8) | (d[4] << 32) | (d[5] << 56);
            dst[2] = (d[5] >> 8) | (d[6] << 16) | (d[7] << 40);
        } else {
            for (uint64_t k = i; k < n; ++k) {
                const uint64_t d = (uint64_t)in[k] - (uint64_t)offset;
                bad |= d > kMax;
                out[3 * k] = (uint8_t)d;
                out[3 * k + 1] = (uint8_t)(d >> 8);
                out[3 * k + 2] = (uint8_t)(d >> 16);
            }
        }
    }
    if (overflow && bad) *overflow = 1u;
}

__global__ __launch_bounds__(256) void narrow_u24_scalar_kernel(const int64_t* __restrict__ in,
                                                                const uint64_t* __restrict__ d_count, uint64_t max_n,
                                                                int64_t offset, uint8_t* __restrict__ out,
                                                                uint32_t* __restrict__ overflow) {
    const uint64_t n = min(*d_count, max_n);
    bool bad = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t d = (uint64_t)in[i] - (uint64_t)offset;
        bad |= d > 0xffffffull;
        out[3 * i] = (uint8_t)d;
        out[3 * i + 1] = (uint8_t)(d >> 8);
        out[3 * i + 2] = (uint8_t)(d >> 16);
    }
    if (overflow && bad) *overflow = 1u;
}

// The same for operands of any alignment: one value per store.
template <typename O>
__global__ __launch_bounds__(256) void narrow_unsigned_scalar_kernel(const int64_t* __restrict__ in,
                                                                     const uint64_t* __restrict__ d_count,
                                                                     uint64_t max_n, int64_t offset, O* __restrict__ out,
                                                                     uint32_t* __restrict__ overflow) {
    const uint64_t n = min(*d_count, max_n);
    constexpr uint64_t kMax = sizeof(O) == 4 ? 0xffffffffull : (1ull << (8 * sizeof(O))) - 1;
    bool bad = false;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t d = (uint64_t)in[i] - (uint64_t)offset;
        bad |= d > kMax;
        out[i] = (O)d;
    }
    if (overflow && bad) *overflow = 1u;
}

// out[i] = in[i] widened: a column registered with a narrower or unsigned type code
// (cubit_table_add_column) is held as INT32 / INT64 values. 4 values per thread per step.
template <typename S, typename D>
__global__ __launch_bounds__(256) void widen_kernel(const S* __restrict__ in, uint64_t n, D* __restrict__ out) {
    const uint64_t stride = 4ull * gridDim.x * blockDim.x;
    for (uint64_t i = 4ull * ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x); i < n; i += stride) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (i + j < n) out[i + j] = (D)in[i + j];
    }
}

// ------------------------------------------------------------------ FLOAT / DOUBLE keys

// A FLOAT / DOUBLE column is held twice: its bit patterns (probes) and their comparison keys
// (key_of<FK>), which every compare kernel reads as a plain INT32 / INT64 column — the per-value key
// in the compare loop made K0 instruction-bound (FLOAT 0.71 ms vs INT32 0.39 ms at 600 M rows).
// One streaming pass, 16-byte loads and stores.
template <int FK, typename T>
__global__ __launch_bounds__(256) void fp_keys_kernel(const T* __restrict__ raw, uint64_t n, T* __restrict__ keys) {
    constexpr int PER = 16 / sizeof(T);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * PER;
    for (uint64_t i = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * PER; i < n; i += stride) {
        if (i + PER <= n && (reinterpret_cast<uintptr_t>(raw + i) % 16) == 0 && (reinterpret_cast<uintptr_t>(keys + i) % 16) == 0) {
            u64x2 q = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(raw + i));
            T v[PER];
            __builtin_memcpy(v, &q, 16);
#pragma unroll
            for (int k = 0; k < PER; ++k) v[k] = key_of<FK>(v[k]);
            __builtin_memcpy(&q, v, 16);
            *reinterpret_cast<u64x2*>(keys + i) = q;
        } else {
            for (uint64_t k = i; k < n && k < i + PER; ++k) keys[k] = key_of<FK>(raw[k]);
        }
    }
}

// out[i] = value_key(type, v[i]): update values (bit patterns) as the keys a merge compares and
// writes into the key column
__global__ __launch_bounds__(256) void value_keys_kernel(const int64_t* __restrict__ v, uint64_t n, int type,
                                                         int64_t* __restrict__ out) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = value_key(type, v[i]);
}

// raw[rows[i]] = the merged record's bit pattern (0 for a NULL record): the pattern column beside the
// keys a merge rewrote
__global__ __launch_bounds__(256) void scatter_raw_kernel(const int64_t* __restrict__ rows, const int64_t* __restrict__ v,
                                                          const uint8_t* __restrict__ valids, uint64_t m, int is32,
                                                          void* __restrict__ raw) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += stride) {
        const int64_t x = (!valids || valids[i]) ? v[i] : 0;
        if (is32) static_cast<int32_t*>(raw)[rows[i]] = (int32_t)x;
        else static_cast<int64_t*>(raw)[rows[i]] = x;
    }
}

// ------------------------------------------------------------------ K3: probe

template <typename T>
__global__ __launch_bounds__(256) void gather_kernel(const T* __restrict__ col, const int64_t* __restrict__ rowids,
                                                     const uint64_t* __restrict__ d_count, uint64_t max_n,
                                                     int64_t row_base, int64_t* __restrict__ out) {
    const uint64_t n = min(*d_count, max_n);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        out[i] = (int64_t)__builtin_nontemporal_load(col + (__builtin_nontemporal_load(rowids + i) - row_base));
}

// K3 with NULL-ness (ColumnData::FilterScan + Vector::Slice carry the vector's validity with
// its values, column_data.cpp:305-309, vector.cpp:223-258): out[i] = col[r] for a valid row and
// 0 for a NULL one, and bit i of out_valid (LSB-first words over output positions — DuckDB's
// ValidityMask layout) says whether row r is valid. A wave takes 64 consecutive positions, so
// one ballot forms each word and lane 0 stores it: 1 bit per row beside the 8-byte value.
template <typename T>
__global__ __launch_bounds__(256) void gather_valid_kernel(const T* __restrict__ col,
                                                           const uint64_t* __restrict__ validity,
                                                           const int64_t* __restrict__ rowids,
                                                           const uint64_t* __restrict__ d_count, uint64_t max_n,
                                                           int64_t row_base, int64_t* __restrict__ out,
                                                           uint64_t* __restrict__ out_valid) {
    const uint64_t n = min(*d_count, max_n);
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    // the loop bound is the wave's first position: every lane of a wave runs the ballot together
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < n; base += stride) {
        const uint64_t i = base + lane;
        bool ok = false;
        if (i < n) {
            const int64_t r = __builtin_nontemporal_load(rowids + i) - row_base;
            ok = !validity || ((validity[r >> 6] >> (r & 63)) & 1ull);
            out[i] = ok ? (int64_t)__builtin_nontemporal_load(col + r) : 0;
        }
        const uint64_t word = __ballot(ok);
        if (lane == 0) out_valid[base >> 6] = word;
    }
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
        const int64_t r = __builtin_nontemporal_load(rowids + i) - row_base;
        acc += (__int128)__builtin_nontemporal_load(x + r) * (__int128)__builtin_nontemporal_load(y + r);
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

// Σ of the per-workgroup 128-bit partials: every lane of one wave sums a strided share (its
// loads independent, so they overlap), then a 64-lane butterfly adds the 128-bit values as
// (lo, hi) pairs with carry. (One lane walking 1,024 partials serially took ~80 µs.)
__global__ __launch_bounds__(64) void sum_partials_kernel(const int64_t* __restrict__ partials, int nblocks,
                                                          int64_t* __restrict__ out) {
    const int lane = threadIdx.x;
    __int128 s = 0;
    for (int b = lane; b < nblocks; b += 64)
        s += ((__int128)partials[2 * b + 1] << 64) | (unsigned __int128)(uint64_t)partials[2 * b];
    uint64_t lo = (uint64_t)s;
    int64_t hi = (int64_t)(s >> 64);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t olo = __shfl_xor(lo, d, 64);
        const int64_t ohi = __shfl_xor(hi, d, 64);
        const uint64_t nlo = lo + olo;
        hi = (int64_t)((uint64_t)hi + (uint64_t)ohi + (nlo < lo ? 1u : 0u));
        lo = nlo;
    }
    if (lane == 0) {
        out[0] = (int64_t)lo;
        out[1] = hi;
    }
}

// ------------------------------------------------------------------ zonemaps

// Zone classes of a bitvector (the bitmap form of a segment's min/max statistics,
// NumericStats::CheckZonemap, numeric_stats.cpp:157-228): one workgroup per zone of kZoneWords
// words, each thread ANDs and ORs 8 words (4 coalesced 16-byte loads). Only rows < n_rows count:
// words past the last row are skipped, the last word is masked. out[z - z0] bit 0 = no row set,
// bit 1 = every row set (both for a zone past the last row).
// Zone class of one bitvector per zone (bit 0: no row set, bit 1: every row set) and, with
// cnt, the zone's set rows — the per-tile counts a single-leaf decode takes its output offsets
// from (eval_decode_lookback with EvalArgs::tile_prefix).
__global__ __launch_bounds__(256) void zone_class_kernel(const uint64_t* __restrict__ bv, uint64_t n_rows,
                                                         uint32_t z0, uint8_t* __restrict__ out,
                                                         uint32_t* __restrict__ cnt) {
    __shared__ uint32_t s_cnt[4];
    const uint32_t z = z0 + blockIdx.x;
    const int t = threadIdx.x;
    const uint64_t n_words = (n_rows + 63) / 64;
    const uint64_t last_mask = (n_rows & 63) ? (1ull << (n_rows & 63)) - 1 : ~0ull;
    uint64_t all = ~0ull, any = 0;
    uint32_t ones = 0;
    const uint64_t w0 = (uint64_t)z * kZoneWords;
#pragma unroll
    for (int p = 0; p < (int)(kZoneWords / 512); ++p) {
        const uint64_t gw = w0 + (uint64_t)(p * 256 + t) * 2;
        if (gw >= n_words) continue;
        const u64x2 x = reinterpret_cast<const u64x2*>(bv + w0)[p * 256 + t];
        uint64_t a = x.x, b = x.y;
        uint64_t ma = gw == n_words - 1 ? last_mask : ~0ull;
        if (gw + 1 >= n_words) {  // b is past the last row (or a is the last word)
            all &= a | ~ma;
            any |= a & ma;
            ones += (uint32_t)__popcll(a & ma);
            continue;
        }
        const uint64_t mb = gw + 1 == n_words - 1 ? last_mask : ~0ull;
        all &= (a | ~ma) & (b | ~mb);
        any |= (a & ma) | (b & mb);
        ones += (uint32_t)(__popcll(a & ma) + __popcll(b & mb));
    }
    const uint32_t wsum = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan32(ones), 63);
    if ((t & 63) == 0) s_cnt[t >> 6] = wsum;
    const int none_set = __syncthreads_and(any == 0);
    const int all_set = __syncthreads_and(all == ~0ull);
    if (t == 0) {
        out[blockIdx.x] = (uint8_t)((none_set ? 1 : 0) | (all_set ? 2 : 0));
        if (cnt) cnt[blockIdx.x] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
    }
}

// Per-zone statistics of a raw column (the segment statistics CheckZonemap consults,
// numeric_stats.cpp:157-228): min / max over the zone's valid rows and whether any / every row
// is valid. One workgroup per zone; consecutive threads read consecutive 4-row chunks.
template <typename T, int FK = 0>
__global__ __launch_bounds__(256) void column_zone_stats_kernel(const T* __restrict__ col,
                                                                const uint64_t* __restrict__ validity, uint64_t n_rows,
                                                                int64_t* __restrict__ mn, int64_t* __restrict__ mx,
                                                                uint8_t* __restrict__ fl) {
    __shared__ int64_t s_lo[256], s_hi[256];
    __shared__ uint32_t s_n[256];
    const int t = threadIdx.x;
    const uint64_t r0 = (uint64_t)blockIdx.x * kZoneRows;
    const uint64_t r1 = min(n_rows, r0 + kZoneRows);
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    uint32_t nv = 0;
    auto take = [&](int64_t v) {
        lo = v < lo ? v : lo;
        hi = v > hi ? v : hi;
        ++nv;
    };
    // four consecutive rows per thread per step (one 16-byte load for INT32, two for INT64; a
    // zone starts on a 131,072-row boundary, so the loads are aligned), four steps in flight
#pragma unroll 4
    for (uint64_t b = r0 + 4u * (uint64_t)t; b < r1; b += 4u * 256u) {
        const uint32_t vb = validity ? (uint32_t)((validity[b >> 6] >> (b & 63)) & 15u) : 15u;
        if (b + 4 <= r1) {
            int64_t x[4];
            if (sizeof(T) == 4) {
                const bp_u32x4 q = __builtin_nontemporal_load(reinterpret_cast<const bp_u32x4*>(col + b));
                x[0] = key_of<FK>((int32_t)q.x), x[1] = key_of<FK>((int32_t)q.y), x[2] = key_of<FK>((int32_t)q.z),
                x[3] = key_of<FK>((int32_t)q.w);
            } else {
                const u64x2 q0 = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(col + b));
                const u64x2 q1 = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(col + b) + 1);
                x[0] = key_of<FK>((int64_t)q0.x), x[1] = key_of<FK>((int64_t)q0.y), x[2] = key_of<FK>((int64_t)q1.x),
                x[3] = key_of<FK>((int64_t)q1.y);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if ((vb >> j) & 1u) take(x[j]);
        } else {
            for (uint64_t r = b; r < r1; ++r)
                if ((vb >> (r - b)) & 1u) take((int64_t)key_of<FK>(col[r]));
        }
    }
    s_lo[t] = lo;
    s_hi[t] = hi;
    s_n[t] = nv;
    __syncthreads();
    for (int d = 128; d > 0; d >>= 1) {
        if (t < d) {
            s_lo[t] = s_lo[t + d] < s_lo[t] ? s_lo[t + d] : s_lo[t];
            s_hi[t] = s_hi[t + d] > s_hi[t] ? s_hi[t + d] : s_hi[t];
            s_n[t] += s_n[t + d];
        }
        __syncthreads();
    }
    if (t == 0) {
        mn[blockIdx.x] = s_lo[0];
        mx[blockIdx.x] = s_hi[0];
        fl[blockIdx.x] = (uint8_t)((s_n[0] > 0 ? 1 : 0) | (r1 > r0 && s_n[0] == r1 - r0 ? 2 : 0));
    }
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

// ------------------------------------------------------------------ index maintenance

// Append (BoundIndex::Append, bound_index.hpp:67-70): splice the n_bits bits of src (bit 0 =
// the first appended row) into dst at bit offset bit_off. One thread per destination word, so
// no word is written twice; the first word keeps its bits below bit_off (the rows already
// there) and the last keeps its bits past the splice (padding, zero). The appended rows'
// bitvector words come from the index-build compare kernel run over the appended slice alone.
__global__ __launch_bounds__(256) void splice_bits_kernel(uint64_t* __restrict__ dst, const uint64_t* __restrict__ src,
                                                          uint64_t bit_off, uint64_t n_bits) {
    const uint64_t w0 = bit_off >> 6, w1 = (bit_off + n_bits + 63) >> 6;
    const uint32_t sh = (uint32_t)(bit_off & 63);
    const uint64_t src_words = (n_bits + 63) >> 6;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t d = w0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; d < w1; d += stride) {
        const uint64_t j = d - w0;  // src word whose low bits land in d (shifted up by sh)
        uint64_t v = j < src_words ? src[j] << sh : 0ull;
        if (sh && j >= 1 && j - 1 < src_words) v |= src[j - 1] >> (64 - sh);
        // bits of d that belong to the splice: rows [max(64d, bit_off), min(64d + 64, bit_off + n_bits))
        const uint64_t lo = d == w0 ? sh : 0;
        const uint64_t end = bit_off + n_bits - 64 * d;  // > 0
        const uint64_t hi = end >= 64 ? 64 : end;
        const uint64_t m = (hi == 64 ? ~0ull : ((1ull << hi) - 1)) & ~((1ull << lo) - 1);
        dst[d] = (dst[d] & ~m) | (v & m);
    }
}

// Merge of committed updates into the base (the checkpoint of update chains, cf.
// UpdateSegment / ColumnData checkpointing; CUBIT merges its update bitvectors the same way):
// row r gets its newest merged value and NULL-ness, and every index bitvector whose predicate
// changes for r changes r's bit. Only the keys whose predicate changes are touched: for a range
// index L(k) = {v < k}, the keys in (min(old, new), max(old, new)] (binary search over the sorted
// keys); for an equality index E(old) and E(new); for bins the old and the new bin.
__device__ __forceinline__ uint32_t upper_key(const int64_t* keys, uint32_t n, int64_t v) {  // first key > v
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (keys[mid] <= v) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Merge by words (cubit_table_merge_updates): the merged records (rows ascending, one per row)
// in chunks of 64 per wave; a wave takes every 64-row word whose first record lies in its chunk
// (a word's records are contiguous, at most 64, and may run into the next chunk), one word at a
// time. The record lanes read the old values, write the new ones and the validity word; then
// every index bitvector whose membership a record can change is rewritten for the word from the
// 64 rows' merged values — one ballot per bitvector — with a plain store: no atomics, no word
// list, and each word is written once however many of its rows changed (flipping bits per record
// through atomics took 140 ms for 6 M records x ~25 range keys at SF100). Range: the keys in
// [min a, max b) of the records' symmetric differences; equality / bins: each record's old and
// new key. Rows past n_rows read as not present.
constexpr uint32_t kMergeLdsKeys = 1024;
constexpr int kMergeBatch = 4;  // words whose 64 values a wave loads together

__global__ __launch_bounds__(256) void merge_words_kernel(const int64_t* __restrict__ rows,
                                                          const int64_t* __restrict__ values,
                                                          const uint8_t* __restrict__ valids, uint64_t m,
                                                          uint64_t n_rows, void* col, int type, uint64_t* validity,
                                                          MergeIndex ix0, MergeIndex ix1) {
    // both indexes' keys and bitvector pointers in LDS (up to kMergeLdsKeys each): a word's
    // rewrite walks its keys one after another, and from global memory each step waited for a
    // dependent load of the key and of the bitvector pointer
    __shared__ int64_t s_keys[2][kMergeLdsKeys];
    __shared__ uint64_t* s_bvs[2][kMergeLdsKeys];
    for (int x = 0; x < 2; ++x) {
        const MergeIndex& ix = x ? ix1 : ix0;
        if (!ix.bvs || ix.n_keys > kMergeLdsKeys) continue;
        for (uint32_t k = threadIdx.x; k < ix.n_keys; k += blockDim.x) {
            s_keys[x][k] = ix.keys[k];
            s_bvs[x][k] = ix.bvs[k];
        }
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x / 64);
    for (uint64_t i0 = ((uint64_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64) * 64; i0 < m; i0 += waves * 64) {
        // the chunk's records and the next chunk's (a word starting here may run into it), each
        // record loaded once; a word's records then come by shuffles, and the old values of its
        // rows from the one load of the word's 64 values — one round of loads per batch of words
        const uint64_t ic = i0 + lane, inx = i0 + 64 + lane;
        const bool in_c = ic < m, in_n = inx < m;
        const int64_t row_c = in_c ? rows[ic] : -1, row_n = in_n ? rows[inx] : -1;
        const int64_t val_c = in_c ? values[ic] : 0, val_n = in_n ? values[inx] : 0;
        const int ok_c = in_c && (!valids || valids[ic]), ok_n = in_n && (!valids || valids[inx]);
        const int64_t before = i0 > 0 ? rows[i0 - 1] : -1;  // the record ahead of the chunk
        int64_t prev_row = __shfl_up(row_c, 1, 64);
        if (lane == 0) prev_row = before;
        const bool starts_word = in_c && (prev_row < 0 || ((uint64_t)prev_row >> 6) != ((uint64_t)row_c >> 6));
        uint64_t todo = __ballot(starts_word);
        while (todo) {
            uint32_t s[kMergeBatch];
            uint64_t wd[kMergeBatch];
            int nb = 0;
            for (; nb < kMergeBatch && todo; ++nb) {
                s[nb] = (uint32_t)__builtin_ctzll(todo);
                todo &= todo - 1;
                wd[nb] = (uint64_t)__shfl(row_c, (int)s[nb], 64) >> 6;
            }
            int64_t colv[kMergeBatch];
            uint64_t vw[kMergeBatch];
#pragma unroll
            for (int j = 0; j < kMergeBatch; ++j) {
                colv[j] = 0;
                vw[j] = ~0ull;
                if (j < nb) {
                    const uint64_t row = wd[j] * 64 + lane;
                    if (row < n_rows)
                        colv[j] = value_key(type, type_is32(type) ? (int64_t)static_cast<const int32_t*>(col)[row]
                                                                  : static_cast<const int64_t*>(col)[row]);
                    if (validity) vw[j] = validity[wd[j]];
                }
            }
#pragma unroll
            for (int j = 0; j < kMergeBatch; ++j) {
                if (j >= nb) break;
                const uint64_t word = wd[j];
                // the word's records: chunk lanes s[j] … and on into the next chunk (a prefix)
                const uint32_t cnt = (uint32_t)__popcll(__ballot(in_c && ((uint64_t)row_c >> 6) == word)) +
                                     (uint32_t)__popcll(__ballot(in_n && ((uint64_t)row_n >> 6) == word));
                const uint32_t q = s[j] + lane;  // this lane's record, 0 … 127 over the two chunks
                const int64_t r_a = __shfl(row_c, (int)(q & 63), 64), r_b = __shfl(row_n, (int)(q & 63), 64);
                const int64_t v_a = __shfl(val_c, (int)(q & 63), 64), v_b = __shfl(val_n, (int)(q & 63), 64);
                const int o_a = __shfl(ok_c, (int)(q & 63), 64), o_b = __shfl(ok_n, (int)(q & 63), 64);
                const bool has_rec = lane < cnt;
                const int64_t rrow = q < 64 ? r_a : r_b;
                const int64_t nv = q < 64 ? v_a : v_b;  // as stored (FLOAT / DOUBLE: the bit pattern)
                const int64_t nk = value_key(type, nv);  // as compared (colv holds keys too)
                const bool nvalid = (q < 64 ? o_a : o_b) != 0;
                const uint32_t pos = has_rec ? (uint32_t)(rrow & 63) : 0;
                const int64_t ov = __shfl(colv[j], (int)pos, 64);  // the row's old value
                const uint64_t old_vword = vw[j];
                const bool ovalid = has_rec && ((old_vword >> pos) & 1ull);
                // the records' rows and new NULL-ness as word masks (OR over the wave)
                uint64_t rec_bits = has_rec ? 1ull << pos : 0, new_bits = has_rec && nvalid ? 1ull << pos : 0;
#pragma unroll
                for (int d = 32; d >= 1; d >>= 1) {
                    rec_bits |= __shfl_xor(rec_bits, d, 64);
                    new_bits |= __shfl_xor(new_bits, d, 64);
                }
                const uint64_t vword = (old_vword & ~rec_bits) | new_bits;
                if (has_rec) {
                    if (type_is32(type)) static_cast<int32_t*>(col)[rrow] = nvalid ? (int32_t)nv : 0;
                    else static_cast<int64_t*>(col)[rrow] = nvalid ? nv : 0;
                }
                if (validity && lane == 0) validity[word] = vword;
                // each row's merged value: its record's (records ascend by row: the row's record is
                // the popcount of the record rows below it), else its old value
                const uint64_t row = word * 64 + lane;
                const bool mine = (rec_bits >> lane) & 1ull;
                const int64_t from_rec = __shfl(nk, (int)__popcll(rec_bits & ((1ull << lane) - 1ull)), 64);
                const bool present = row < n_rows && ((vword >> lane) & 1ull);
                const int64_t v = present ? (mine ? from_rec : colv[j]) : 0;
                for (int x = 0; x < 2; ++x) {
                    const MergeIndex& gix = x ? ix1 : ix0;
                    if (!gix.bvs) continue;
                    const uint32_t n = gix.n_keys;
                    const bool lds = n <= kMergeLdsKeys;
                    const MergeIndex ix{lds ? s_keys[x] : gix.keys, lds ? s_bvs[x] : gix.bvs, n, gix.encoding};
                    if (ix.encoding == 0) {  // range: L(k) = {valid, v < k}
                        // the union of the records' flipped key intervals (keys searched in LDS when
                        // cached there: called with the LDS array itself, the searches are ds_reads)
                        auto interval = [&](const int64_t* keys, uint32_t& ra, uint32_t& rb) {
                            ra = n;
                            rb = n;
                            if (ovalid && nvalid) {
                                const int64_t lo = ov < nk ? ov : nk, hi = ov < nk ? nk : ov;
                                ra = upper_key(keys, n, lo);
                                rb = upper_key(keys, n, hi);
                            } else if (ovalid) {
                                ra = upper_key(keys, n, ov);
                            } else if (nvalid) {
                                ra = upper_key(keys, n, nk);
                            }
                        };
                        uint32_t a = n, b = 0;
                        if (has_rec) {
                            uint32_t ra, rb;
                            if (lds) interval(s_keys[x], ra, rb);
                            else interval(gix.keys, ra, rb);
                            if (ra < rb) {
                                a = ra;
                                b = rb;
                            }
                        }
#pragma unroll
                        for (int d = 32; d >= 1; d >>= 1) {
                            a = min(a, (uint32_t)__shfl_xor((int)a, d, 64));
                            b = max(b, (uint32_t)__shfl_xor((int)b, d, 64));
                        }
                        if (lds) {  // explicit LDS reads (through a generic pointer they issue as flat loads)
                            for (uint32_t k = a; k < b; ++k) {
                                const uint64_t bits = __ballot(present && v < s_keys[x][k]);
                                if (lane == 0) s_bvs[x][k][word] = bits;
                            }
                        } else {
                            for (uint32_t k = a; k < b; ++k) {
                                const uint64_t bits = __ballot(present && v < ix.keys[k]);
                                if (lane == 0) ix.bvs[k][word] = bits;
                            }
                        }
                    } else {  // equality E(k) = {valid, v == k}; bins B_i = {valid, e_i <= v < e_i+1}
                        // each record's old and new bitvector (-1: none), rewritten one record at a time
                        auto which = [&](bool ok, int64_t val) -> int32_t {
                            if (!ok) return -1;
                            const uint32_t k = upper_key(ix.keys, n, val);
                            if (ix.encoding == 1) return (k > 0 && ix.keys[k - 1] == val) ? (int32_t)k - 1 : -1;
                            return (k == 0 || k == n) ? -1 : (int32_t)k - 1;
                        };
                        const int32_t ko = has_rec ? which(ovalid, ov) : -1, kn = has_rec ? which(nvalid, nk) : -1;
                        for (uint32_t jj = 0; jj < cnt; ++jj) {
                            for (int side = 0; side < 2; ++side) {
                                const int32_t k = __shfl(side ? kn : ko, (int)jj, 64);
                                if (k < 0) continue;
                                const bool in = ix.encoding == 1 ? v == ix.keys[k] : (ix.keys[k] <= v && v < ix.keys[k + 1]);
                                const uint64_t bits = __ballot(present && in);
                                if (lane == 0) ix.bvs[k][word] = bits;
                            }
                        }
                    }
                }
            }
        }
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

// Rows of insert ranges the reader may not see (UseInsertedVersion false for the range's
// insert id, chunk_info.cpp:11-19, ChunkConstantInfo / ChunkVectorInfo::inserted): clear
// [begin, end) of range blockIdx.y. Ranges are disjoint, so only a range's first and last
// word can be shared with another range (atomicAnd); inner words are stored as 0.
__global__ __launch_bounds__(256) void clear_ranges_kernel(const int64_t* __restrict__ ranges, uint64_t* __restrict__ words) {
    const uint64_t b = (uint64_t)ranges[2 * blockIdx.y], e = (uint64_t)ranges[2 * blockIdx.y + 1];
    if (b >= e) return;
    const uint64_t w0 = b >> 6, w1 = (e - 1) >> 6;
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t w = w0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w <= w1; w += stride) {
        uint64_t clear = ~0ull;
        if (w == w0) clear &= ~0ull << (b & 63);
        if (w == w1 && (e & 63)) clear &= (1ull << (e & 63)) - 1;
        if (w == w0 || w == w1) atomicAnd(reinterpret_cast<unsigned long long*>(&words[w]), ~clear);
        else words[w] = 0;
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

// production geometry: decode tiles of 512 threads × 2 pairs = 2,048 words (131,072 rows),
// STAGE 4,096 staged ids (16 KiB LDS); count tiles of 256 threads × 8 pairs = 4,096 words.
// Chosen from the interleaved variant sweep in scripts/kbench.hip.
constexpr int kDecodeThreads = 512, kDecodePairs = 2, kDecodeStage = 4096;
// eval_decode_runs: two stages of 9,984 entries (78 KiB; two workgroups per CU fill the 160 KiB)
constexpr int kRunCap = 9984;
// count tiles: 512 threads × 2 pairs = 2,048 words for K ≤ 4, × 1 pair above (two tiles in
// flight must fit the 128-VGPR budget of 4 waves per SIMD)
constexpr int count_pairs(uint32_t k) { return k <= 4 ? 2 : 1; }
constexpr int kCountGrid = 512;   // persistent count grid: 2 workgroups per CU

uint64_t decode_tile_words() { return (uint64_t)kDecodeThreads * 2 * kDecodePairs; }
uint64_t count_tile_words(uint32_t n_leaves) { return 512ull * 2 * (uint64_t)count_pairs(n_leaves); }
int decode_block_threads() { return kDecodeThreads; }

// A left-deep chain of ANDs (nops = 0,1,1,…; every op AND) evaluates as a plain conjunction.
bool is_conjunction(const EvalProgram& p) {
    if (p.n_leaves == 0 || prog_nops(p, 0) != 0) return false;
    for (uint32_t k = 1; k < p.n_leaves; ++k)
        if (prog_nops(p, (int)k) != 1 || ((p.ops >> (2 * (k - 1))) & 3u) != OP_AND) return false;
    return true;
}

uint32_t eval_form(const EvalProgram& p) {
    if (p.form == FORM_DNF || p.form == FORM_CNF || p.form == FORM_CONJ) return p.form;
    return is_conjunction(p) ? FORM_CONJ : FORM_POSTFIX;
}

// production decode (scripts/kbench.hip): the run-claimed kernel wherever a
// workgroup walks three or more tiles — one claim per filled LDS stage instead of one per pair
// (SF100-sized, 1 % / 0.75 % / 0.4 % selected at K = 1 / 2 / 3: 41 / 39 / 44 µs vs 46 / 50 / 57
// µs; K = 5 at 1.9 %: 82 vs 84 µs) — except K = 4, where at Q6's density a run holds two tiles
// and the pair kernel measured as fast or 1 % faster (73.2 vs 74.2 µs); the pair kernel for one
// or two tiles per workgroup (small inputs: one claim per workgroup either way).
// look-back kernel geometry: workgroups per CU (the grid is co-resident up to WPC·CUs tiles) and
// stage entries (32 KiB of LDS per workgroup)
constexpr int lookback_wpc(uint32_t) { return 3; }  // 80 VGPRs: no spill for K ≤ 8 (4 per CU: 64, spills)
constexpr int kLookbackStage = 8192;
uint32_t lookback_max_tiles(uint32_t n_leaves, int n_cus) {
    return std::min<uint32_t>(kLookbackMaxTiles, (uint32_t)lookback_wpc(n_leaves) * (uint32_t)n_cus);
}

int decode_kernel_for(uint32_t n_leaves, uint32_t num_tiles, unsigned grid, int kernel, bool live, int n_cus,
                      bool prefixed) {
    // known per-tile offsets: one tile per workgroup with no inter-workgroup wait, at any size
    if (prefixed && (kernel == 0 || kernel == 3)) return 3;
    if (kernel == 3 && num_tiles <= kLookbackMaxTiles) return 3;
    if (kernel == 0 && num_tiles <= lookback_max_tiles(n_leaves, n_cus)) return 3;
    // a live-tile list (zonemap skip) needs the run kernel: its stage offsets are taken from the
    // run's first tile, while the pair kernel places tile B G tiles after tile A
    if (live) return 2;
    if (kernel == 1 || kernel == 2) return kernel;
    return num_tiles > 2ull * grid ? 2 : 1;
}

template <int K, int FORM>
void launch_decode_kf(const EvalArgs& a, uint64_t* dir, unsigned grid, hipStream_t s, hipEvent_t e0, hipEvent_t e1,
                      int kernel, int n_cus) {
    const int which = decode_kernel_for(K, a.num_tiles, grid, kernel, a.live != nullptr, n_cus, a.tile_prefix != nullptr);
    if (which == 3)
        hipExtLaunchKernelGGL((eval_decode_lookback<K, FORM, kLookbackStage, lookback_wpc(K)>), dim3(a.num_tiles),
                              dim3(512), 0, s, e0, e1, 0, a, dir);
    else if (which == 2)
        hipExtLaunchKernelGGL((eval_decode_runs<K, kDecodePairs, kRunCap, kDecodeThreads, FORM>), dim3(grid),
                              dim3(kDecodeThreads), 0, s, e0, e1, 0, a, dir);
    else
        hipExtLaunchKernelGGL((eval_decode_pairs<K, kDecodePairs, kDecodeStage, kDecodeThreads, 0, FORM>), dim3(grid),
                              dim3(kDecodeThreads), 0, s, e0, e1, 0, a, dir);
}

template <int K>
hipError_t launch_decode_k(const EvalArgs& a, uint64_t* dir, unsigned grid, hipStream_t s, hipEvent_t e0,
                           hipEvent_t e1, int kernel, int n_cus) {
    switch (eval_form(a.prog)) {
    case FORM_CONJ: launch_decode_kf<K, FORM_CONJ>(a, dir, grid, s, e0, e1, kernel, n_cus); break;
    case FORM_DNF: launch_decode_kf<K, FORM_DNF>(a, dir, grid, s, e0, e1, kernel, n_cus); break;
    case FORM_CNF: launch_decode_kf<K, FORM_CNF>(a, dir, grid, s, e0, e1, kernel, n_cus); break;
    default: launch_decode_kf<K, FORM_POSTFIX>(a, dir, grid, s, e0, e1, kernel, n_cus); break;
    }
    return hipGetLastError();
}

template <int K, int FORM>
void launch_count_kf(const EvalArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    const unsigned grid = std::min<unsigned>(a.num_tiles, (unsigned)kCountGrid);
    // result words: plain stores. sc1 buffer stores (SAUX 16) measured 37.7 vs 38.8 µs for a K = 2
    // materialise at SF100 size (profiles/r02k_balbench_materialise.txt); not enabled until the GPU
    // suite has run with them
    hipExtLaunchKernelGGL((eval_count_kernel<K, count_pairs(K), FORM>), dim3(grid), dim3(512), 0, s, e0, e1, 0, a);
}

template <int K>
hipError_t launch_count_k(const EvalArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    switch (eval_form(a.prog)) {
    case FORM_CONJ: launch_count_kf<K, FORM_CONJ>(a, s, e0, e1); break;
    case FORM_DNF: launch_count_kf<K, FORM_DNF>(a, s, e0, e1); break;
    case FORM_CNF: launch_count_kf<K, FORM_CNF>(a, s, e0, e1); break;
    default: launch_count_kf<K, FORM_POSTFIX>(a, s, e0, e1); break;
    }
    return hipGetLastError();
}

hipError_t launch_eval_decode(const EvalArgs& a, uint64_t* dir, unsigned grid, hipStream_t s, hipEvent_t e0,
                              hipEvent_t e1, int kernel, int n_cus) {
    if (decode_kernel_for(a.prog.n_leaves, a.num_tiles, grid, kernel, a.live != nullptr, n_cus,
                          a.tile_prefix != nullptr) == 3 &&
        (a.num_tiles == 0 || (!a.tile_prefix && (a.flags == nullptr || a.epoch == 0))))
        return hipErrorInvalidValue;  // the look-back kernel needs the context's flags and an epoch
    switch (a.prog.n_leaves) {
    case 1: return launch_decode_k<1>(a, dir, grid, s, e0, e1, kernel, n_cus);
    case 2: return launch_decode_k<2>(a, dir, grid, s, e0, e1, kernel, n_cus);
    case 3: return launch_decode_k<3>(a, dir, grid, s, e0, e1, kernel, n_cus);
    case 4: return launch_decode_k<4>(a, dir, grid, s, e0, e1, kernel, n_cus);
    case 5: return launch_decode_k<5>(a, dir, grid, s, e0, e1, kernel, n_cus);
    case 6: return launch_decode_k<6>(a, dir, grid, s, e0, e1, kernel, n_cus);
    case 7: return launch_decode_k<7>(a, dir, grid, s, e0, e1, kernel, n_cus);
    case 8: return launch_decode_k<8>(a, dir, grid, s, e0, e1, kernel, n_cus);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_eval_count(const EvalArgs& a, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
    switch (a.prog.n_leaves) {
    case 1: return launch_count_k<1>(a, s, e0, e1);
    case 2: return launch_count_k<2>(a, s, e0, e1);
    case 3: return launch_count_k<3>(a, s, e0, e1);
    case 4: return launch_count_k<4>(a, s, e0, e1);
    case 5: return launch_count_k<5>(a, s, e0, e1);
    case 6: return launch_count_k<6>(a, s, e0, e1);
    case 7: return launch_count_k<7>(a, s, e0, e1);
    case 8: return launch_count_k<8>(a, s, e0, e1);
    default: return hipErrorInvalidValue;
    }
}

hipError_t launch_order_runs(const uint64_t* dir, uint32_t n_tiles, uint64_t* dst_off, const int64_t* src,
                             uint64_t capacity, int64_t* dst, hipStream_t s) {
    (void)dst_off;
    if (n_tiles == 0) return hipSuccess;
    const uint32_t tpw = std::max<uint32_t>(1, std::min<uint32_t>(8, n_tiles / 1024));
    const unsigned grid = (n_tiles + tpw - 1) / tpw;
    hipLaunchKernelGGL(order_runs_kernel<0>, dim3(grid), dim3(256), 0, s, dir, n_tiles, tpw, src, capacity, dst);
    return hipGetLastError();
}

hipError_t launch_compare_bitvector(const void* col, int type, const uint64_t* validity, uint64_t n_rows, int cmp,
                                    int64_t constant, uint64_t* out_words, hipStream_t stream, int64_t constant2) {
    MultiKeyArgs a{};
    a.m = 1;
    a.c[0] = constant;
    a.c2[0] = constant2;
    a.out[0] = out_words;
    return launch_compare_m<1>(col, type, validity, n_rows, cmp, a, stream);
}

hipError_t launch_candidate_check(const void* col, int type, const uint64_t* validity, const uint64_t* lo_bv,
                                  const uint64_t* hi_bv, uint64_t n_rows, int cmp, int64_t constant,
                                  uint64_t* out_words, hipStream_t stream) {
    if (type == kTypeFloat)
        return constant >= INT32_MIN && constant <= INT32_MAX
                   ? launch_candidate_t<int32_t, int32_t, 1>(static_cast<const int32_t*>(col), validity, lo_bv, hi_bv,
                                                             n_rows, cmp, (int32_t)constant, out_words, stream)
                   : launch_candidate_t<int32_t, int64_t, 1>(static_cast<const int32_t*>(col), validity, lo_bv, hi_bv,
                                                             n_rows, cmp, constant, out_words, stream);
    if (type == kTypeDouble)
        return launch_candidate_t<int64_t, int64_t, 2>(static_cast<const int64_t*>(col), validity, lo_bv, hi_bv, n_rows,
                                                       cmp, constant, out_words, stream);
    if (type == kTypeUInt64)  // unsigned compare against the un-keyed constant
        return launch_candidate_t<uint64_t, uint64_t>(static_cast<const uint64_t*>(col), validity, lo_bv, hi_bv, n_rows,
                                                      cmp, (uint64_t)constant ^ 0x8000000000000000ull, out_words, stream);
    if (type_is32(type) && constant >= INT32_MIN && constant <= INT32_MAX)
        return launch_candidate_t<int32_t, int32_t>(static_cast<const int32_t*>(col), validity, lo_bv, hi_bv, n_rows,
                                                    cmp, (int32_t)constant, out_words, stream);
    if (type_is32(type))
        return launch_candidate_t<int32_t, int64_t>(static_cast<const int32_t*>(col), validity, lo_bv, hi_bv, n_rows,
                                                    cmp, constant, out_words, stream);
    return launch_candidate_t<int64_t, int64_t>(static_cast<const int64_t*>(col), validity, lo_bv, hi_bv, n_rows, cmp,
                                                constant, out_words, stream);
}

hipError_t launch_compare_bitvectors(const void* col, int type, const uint64_t* validity, uint64_t n_rows, int cmp,
                                     const MultiKeyArgs& args, hipStream_t stream) {
    if (args.m == 0) return hipSuccess;
    if (args.m > (uint32_t)kMultiKeys) return hipErrorInvalidValue;
    MultiKeyArgs a = args;
    for (uint32_t k = a.m; k < (uint32_t)kMultiKeys; ++k) {  // the kernel evaluates every slot
        a.c[k] = a.c[a.m - 1];
        a.c2[k] = a.c2[a.m - 1];
        a.out[k] = nullptr;
    }
    // the smallest key count that covers m: the ballots per word grow with it
    if (a.m == 1) return launch_compare_m<1>(col, type, validity, n_rows, cmp, a, stream);
    if (a.m <= 4) return launch_compare_m<4>(col, type, validity, n_rows, cmp, a, stream);
    if (a.m <= 8) return launch_compare_m<8>(col, type, validity, n_rows, cmp, a, stream);
    return launch_compare_m<kMultiKeys>(col, type, validity, n_rows, cmp, a, stream);
}

hipError_t launch_column_minmax(const void* col, int type, const uint64_t* validity, uint64_t n_rows, int64_t* out3,
                                hipStream_t stream) {
    const dim3 grid(grid_for(n_rows, 2048)), block(256);
    if (type == kTypeFloat)
        hipLaunchKernelGGL((column_minmax_kernel<int32_t, 1>), grid, block, 0, stream, static_cast<const int32_t*>(col),
                           validity, n_rows, out3);
    else if (type == kTypeDouble)
        hipLaunchKernelGGL((column_minmax_kernel<int64_t, 2>), grid, block, 0, stream, static_cast<const int64_t*>(col),
                           validity, n_rows, out3);
    else if (type == kTypeUInt64)
        hipLaunchKernelGGL((column_minmax_kernel<int64_t, 3>), grid, block, 0, stream, static_cast<const int64_t*>(col),
                           validity, n_rows, out3);
    else if (type_is32(type))
        hipLaunchKernelGGL(column_minmax_kernel<int32_t>, grid, block, 0, stream, static_cast<const int32_t*>(col),
                           validity, n_rows, out3);
    else
        hipLaunchKernelGGL(column_minmax_kernel<int64_t>, grid, block, 0, stream, static_cast<const int64_t*>(col),
                           validity, n_rows, out3);
    return hipGetLastError();
}

hipError_t launch_presence(const void* col, int type, const uint64_t* validity, uint64_t n_rows, int64_t vmin,
                           uint64_t range, uint64_t* bits, hipStream_t stream) {
    const dim3 grid(grid_for(n_rows, 2048)), block(256);
    const bool lds = range <= 65536;
#define CUBIT_PRESENCE(T, L, FK)                                                                                   \
    hipLaunchKernelGGL((presence_kernel<T, L, FK>), grid, block, 0, stream, static_cast<const T*>(col), validity, \
                       n_rows, vmin, range, bits)
    if (type == kTypeFloat) {  // a FLOAT column's keys span less than 2^32 (a DOUBLE's are sorted on the host)
        if (lds) CUBIT_PRESENCE(int32_t, true, 1);
        else CUBIT_PRESENCE(int32_t, false, 1);
    } else if (type == kTypeDouble) {
        if (lds) CUBIT_PRESENCE(int64_t, true, 2);
        else CUBIT_PRESENCE(int64_t, false, 2);
    } else if (type == kTypeUInt64) {
        if (lds) CUBIT_PRESENCE(int64_t, true, 3);
        else CUBIT_PRESENCE(int64_t, false, 3);
    } else if (type_is32(type)) {
        if (lds) CUBIT_PRESENCE(int32_t, true, 0);
        else CUBIT_PRESENCE(int32_t, false, 0);
    } else {
        if (lds) CUBIT_PRESENCE(int64_t, true, 0);
        else CUBIT_PRESENCE(int64_t, false, 0);
    }
#undef CUBIT_PRESENCE
    return hipGetLastError();
}

hipError_t launch_narrow_i32(const int64_t* in, const uint64_t* d_count, uint64_t max_n, int64_t offset, int32_t* out,
                             hipStream_t stream, uint32_t* overflow) {
    if (max_n == 0) return hipSuccess;
    hipLaunchKernelGGL(narrow_i32_kernel, dim3(grid_for((max_n + 1) / 2)), dim3(256), 0, stream, in, d_count, max_n,
                       offset, out, overflow);
    return hipGetLastError();
}

template <typename O>
static void narrow_unsigned_launch(const int64_t* in, const uint64_t* d_count, uint64_t max_n, int64_t offset, O* out,
                                   uint32_t* overflow, hipStream_t stream) {
    const bool aligned = reinterpret_cast<uintptr_t>(in) % 16 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0;
    if (aligned)
        hipLaunchKernelGGL(narrow_unsigned_kernel<O>, dim3(grid_for((max_n + 7) / 8)), dim3(256), 0, stream, in, d_count,
                           max_n, offset, out, overflow);
    else
        hipLaunchKernelGGL(narrow_unsigned_scalar_kernel<O>, dim3(grid_for(max_n)), dim3(256), 0, stream, in, d_count,
                           max_n, offset, out, overflow);
}

hipError_t launch_narrow_unsigned(const int64_t* in, const uint64_t* d_count, uint64_t max_n, int64_t offset, int width,
                                  void* out, uint32_t* overflow, hipStream_t stream) {
    if (max_n == 0) return hipSuccess;
    if (width == 1)
        narrow_unsigned_launch(in, d_count, max_n, offset, static_cast<uint8_t*>(out), overflow, stream);
    else if (width == 2)
        narrow_unsigned_launch(in, d_count, max_n, offset, static_cast<uint16_t*>(out), overflow, stream);
    else if (width == 4)
        narrow_unsigned_launch(in, d_count, max_n, offset, static_cast<uint32_t*>(out), overflow, stream);
    else if (width == 3) {
        uint8_t* o = static_cast<uint8_t*>(out);
        if (reinterpret_cast<uintptr_t>(in) % 16 == 0 && reinterpret_cast<uintptr_t>(o) % 8 == 0)
            hipLaunchKernelGGL(narrow_u24_kernel, dim3(grid_for((max_n + 7) / 8)), dim3(256), 0, stream, in, d_count,
                               max_n, offset, o, overflow);
        else
            hipLaunchKernelGGL(narrow_u24_scalar_kernel, dim3(grid_for(max_n)), dim3(256), 0, stream, in, d_count, max_n,
                               offset, o, overflow);
    } else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_widen(const void* in, int src_type, uint64_t n, void* out, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const dim3 grid(grid_for((n + 3) / 4)), block(256);
    switch (src_type) {
    case CUBIT_TYPE_INT8:
        hipLaunchKernelGGL((widen_kernel<int8_t, int32_t>), grid, block, 0, stream, static_cast<const int8_t*>(in), n,
                           static_cast<int32_t*>(out));
        break;
    case CUBIT_TYPE_INT16:
        hipLaunchKernelGGL((widen_kernel<int16_t, int32_t>), grid, block, 0, stream, static_cast<const int16_t*>(in), n,
                           static_cast<int32_t*>(out));
        break;
    case CUBIT_TYPE_UINT8:
        hipLaunchKernelGGL((widen_kernel<uint8_t, int32_t>), grid, block, 0, stream, static_cast<const uint8_t*>(in), n,
                           static_cast<int32_t*>(out));
        break;
    case CUBIT_TYPE_UINT16:
        hipLaunchKernelGGL((widen_kernel<uint16_t, int32_t>), grid, block, 0, stream, static_cast<const uint16_t*>(in), n,
                           static_cast<int32_t*>(out));
        break;
    case CUBIT_TYPE_UINT32:
        hipLaunchKernelGGL((widen_kernel<uint32_t, int64_t>), grid, block, 0, stream, static_cast<const uint32_t*>(in), n,
                           static_cast<int64_t*>(out));
        break;
    case CUBIT_TYPE_UINT64:  // the bits as they are; the caller checks every valid value is below 2^63
        hipLaunchKernelGGL((widen_kernel<uint64_t, int64_t>), grid, block, 0, stream, static_cast<const uint64_t*>(in), n,
                           static_cast<int64_t*>(out));
        break;
    default:
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_fp_keys(const void* raw, int type, uint64_t n, void* keys, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (type == kTypeFloat)
        hipLaunchKernelGGL((fp_keys_kernel<1, int32_t>), dim3(grid_for((n + 3) / 4)), dim3(256), 0, stream,
                           static_cast<const int32_t*>(raw), n, static_cast<int32_t*>(keys));
    else if (type == kTypeDouble)
        hipLaunchKernelGGL((fp_keys_kernel<2, int64_t>), dim3(grid_for((n + 1) / 2)), dim3(256), 0, stream,
                           static_cast<const int64_t*>(raw), n, static_cast<int64_t*>(keys));
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_value_keys(const int64_t* v, uint64_t n, int type, int64_t* out, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(value_keys_kernel, dim3(grid_for(n)), dim3(256), 0, stream, v, n, type, out);
    return hipGetLastError();
}

hipError_t launch_scatter_raw(const int64_t* rows, const int64_t* v, const uint8_t* valids, uint64_t m, int type,
                              void* raw, hipStream_t stream) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(scatter_raw_kernel, dim3(grid_for(m)), dim3(256), 0, stream, rows, v, valids, m,
                       type_is32(type) ? 1 : 0, raw);
    return hipGetLastError();
}

hipError_t launch_gather(const void* col, int type, const int64_t* rowids, const uint64_t* d_count, uint64_t max_n,
                         int64_t row_base, int64_t* out, hipStream_t stream) {
    const dim3 grid(grid_for(max_n, 8192)), block(256);
    // the values as stored: a FLOAT pattern zero-extended, a DOUBLE pattern as it is
    if (type == kTypeFloat)
        hipLaunchKernelGGL(gather_kernel<uint32_t>, grid, block, 0, stream, static_cast<const uint32_t*>(col), rowids,
                           d_count, max_n, row_base, out);
    else if (type_is32(type))
        hipLaunchKernelGGL(gather_kernel<int32_t>, grid, block, 0, stream, static_cast<const int32_t*>(col), rowids,
                           d_count, max_n, row_base, out);
    else
        hipLaunchKernelGGL(gather_kernel<int64_t>, grid, block, 0, stream, static_cast<const int64_t*>(col), rowids,
                           d_count, max_n, row_base, out);
    return hipGetLastError();
}

hipError_t launch_gather_valid(const void* col, int type, const uint64_t* validity, const int64_t* rowids,
                               const uint64_t* d_count, uint64_t max_n, int64_t row_base, int64_t* out,
                               uint64_t* out_valid, hipStream_t stream) {
    const dim3 grid(grid_for(max_n, 8192)), block(256);
    if (type == kTypeFloat)
        hipLaunchKernelGGL(gather_valid_kernel<uint32_t>, grid, block, 0, stream, static_cast<const uint32_t*>(col),
                           validity, rowids, d_count, max_n, row_base, out, out_valid);
    else if (type_is32(type))
        hipLaunchKernelGGL(gather_valid_kernel<int32_t>, grid, block, 0, stream, static_cast<const int32_t*>(col),
                           validity, rowids, d_count, max_n, row_base, out, out_valid);
    else
        hipLaunchKernelGGL(gather_valid_kernel<int64_t>, grid, block, 0, stream, static_cast<const int64_t*>(col),
                           validity, rowids, d_count, max_n, row_base, out, out_valid);
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

unsigned sum_product_grid(unsigned n_cus) { return std::min<unsigned>(2 * n_cus, (unsigned)kSumBlocks); }

template <int K, int M>
void launch_sum_km(const EvalArgs& a, const SumArgs& s, unsigned grid, hipStream_t st) {
    switch (eval_form(a.prog)) {
    case FORM_CONJ: hipLaunchKernelGGL((eval_sum_product<K, M, FORM_CONJ>), dim3(grid), dim3(512), 0, st, a, s); break;
    case FORM_DNF: hipLaunchKernelGGL((eval_sum_product<K, M, FORM_DNF>), dim3(grid), dim3(512), 0, st, a, s); break;
    case FORM_CNF: hipLaunchKernelGGL((eval_sum_product<K, M, FORM_CNF>), dim3(grid), dim3(512), 0, st, a, s); break;
    default: hipLaunchKernelGGL((eval_sum_product<K, M, FORM_POSTFIX>), dim3(grid), dim3(512), 0, st, a, s); break;
    }
}

template <int K>
void launch_sum_k(const EvalArgs& a, const SumArgs& s, unsigned grid, hipStream_t st) {
    switch (s.b ? 0 : s.n_decode) {
    case 0: launch_sum_km<K, 0>(a, s, grid, st); break;
    case 1: launch_sum_km<K, 1>(a, s, grid, st); break;
    case 2: launch_sum_km<K, 2>(a, s, grid, st); break;
    default: launch_sum_km<K, 3>(a, s, grid, st); break;
    }
}

hipError_t launch_eval_sum_product(const EvalArgs& a, const SumArgs& s, unsigned grid, int64_t* out, hipStream_t st) {
    if (!s.b && s.n_decode > (uint32_t)kMaxDecode) return hipErrorInvalidValue;
    switch (a.prog.n_leaves) {
    case 1: launch_sum_k<1>(a, s, grid, st); break;
    case 2: launch_sum_k<2>(a, s, grid, st); break;
    case 3: launch_sum_k<3>(a, s, grid, st); break;
    case 4: launch_sum_k<4>(a, s, grid, st); break;
    case 5: launch_sum_k<5>(a, s, grid, st); break;
    case 6: launch_sum_k<6>(a, s, grid, st); break;
    case 7: launch_sum_k<7>(a, s, grid, st); break;
    case 8: launch_sum_k<8>(a, s, grid, st); break;
    default: return hipErrorInvalidValue;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(64), 0, st, s.partials, (int)grid, out);
    return hipGetLastError();
}

hipError_t launch_sum_product_arrays(const int64_t* x, const int64_t* y, const uint64_t* d_count, uint64_t max_n,
                                     int64_t* partials, int64_t* out, hipStream_t stream) {
    hipLaunchKernelGGL(sum_product_arrays_kernel, dim3(kSumBlocks), dim3(256), 0, stream, x, y, d_count, max_n,
                       partials);
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(64), 0, stream, partials, kSumBlocks, out);
    return hipGetLastError();
}

hipError_t launch_bitunpack(const uint8_t* bytes, const BpGroup* groups, uint64_t n_groups, int type, void* out,
                            hipStream_t stream, hipEvent_t start, hipEvent_t stop) {
    if (n_groups == 0) return hipSuccess;
    if (n_groups > 0x7fffffffull) return hipErrorInvalidValue;
    if (type == 0)
        hipExtLaunchKernelGGL((bitunpack_kernel<int32_t, uint32_t>), dim3((unsigned)n_groups), dim3(256), 0, stream,
                              start, stop, 0, bytes, groups, static_cast<int32_t*>(out));
    else
        hipExtLaunchKernelGGL((bitunpack_kernel<int64_t, uint64_t>), dim3((unsigned)n_groups), dim3(256), 0, stream,
                              start, stop, 0, bytes, groups, static_cast<int64_t*>(out));
    return hipGetLastError();
}

// ------------------------------------------------------------------ dictionary encode
// Strings (bytes + offsets, in device memory) → codes of an order-preserving dictionary (its
// entries sorted, bytes + offsets on the device): one lane per string, a binary search comparing
// bytes as unsigned then lengths (string_t's order, the host dictionary's). A NULL row gets code
// 0; a valid string the dictionary lacks gets -1 and counts into *missing.
__device__ __forceinline__ int dict_cmp(const uint8_t* a, uint64_t na, const uint8_t* b, uint64_t nb) {
    const uint64_t m = na < nb ? na : nb;
    for (uint64_t i = 0; i < m; ++i)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return na < nb ? -1 : na > nb ? 1 : 0;
}

__global__ __launch_bounds__(256) void dict_encode_kernel(const uint8_t* __restrict__ bytes,
                                                          const uint64_t* __restrict__ offs, uint64_t n,
                                                          const uint64_t* __restrict__ validity,
                                                          const uint8_t* __restrict__ dbytes,
                                                          const uint64_t* __restrict__ doffs, uint64_t dn,
                                                          int32_t* __restrict__ codes,
                                                          unsigned long long* __restrict__ missing) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t miss = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (validity && !((validity[i >> 6] >> (i & 63)) & 1ull)) {
            codes[i] = 0;
            continue;
        }
        const uint8_t* s = bytes + offs[i];
        const uint64_t ns = offs[i + 1] - offs[i];
        uint64_t lo = 0, hi = dn;  // first entry >= s
        while (lo < hi) {
            const uint64_t mid = (lo + hi) / 2;
            if (dict_cmp(dbytes + doffs[mid], doffs[mid + 1] - doffs[mid], s, ns) < 0) lo = mid + 1;
            else hi = mid;
        }
        const bool found = lo < dn && dict_cmp(dbytes + doffs[lo], doffs[lo + 1] - doffs[lo], s, ns) == 0;
        codes[i] = found ? (int32_t)lo : -1;
        miss += found ? 0u : 1u;
    }
    // one add per wave that saw a miss
    for (int o = 32; o > 0; o >>= 1) miss += __shfl_down(miss, o, 64);
    if ((threadIdx.x & 63) == 0 && miss) atomicAdd(missing, (unsigned long long)miss);
}

hipError_t launch_dict_encode(const uint8_t* bytes, const uint64_t* offs, uint64_t n, const uint64_t* validity,
                              const uint8_t* dbytes, const uint64_t* doffs, uint64_t dn, int32_t* codes,
                              unsigned long long* missing, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 256 * 32);
    hipLaunchKernelGGL(dict_encode_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, bytes, offs, n, validity, dbytes,
                       doffs, dn, codes, missing);
    return hipGetLastError();
}

// ------------------------------------------------------------------ RLE expand
// DuckDB RLE segments (src/storage/compression/rle.cpp) expanded into a plain column. The host
// has parsed every segment into runs — the run values (already widened to the column's type) and
// each run's end row (exclusive, cumulative over the partition; zero-length runs, which the
// reference writes after a run of exactly 65,535 rows, repeat the previous end). Workgroups take
// 2,048-row tiles in turn; a tile's runs, from its first row's through its last row's, are known
// beforehand (rle_tile_first_kernel, a lane per tile). A tile inside one run or across one
// boundary is filled straight from those two runs; otherwise its runs are staged in LDS and each
// lane finds the run of its first of 8 consecutive rows by binary search and walks on from it.
// Every lane writes its 8 rows as 16-byte stores.
// tile_first[b] = the first run ending past row 2,048·b (b = 0 … tiles; n_runs past the end): one
// lane per tile, so the dependent loads of the searches overlap across the whole grid
__global__ __launch_bounds__(256) void rle_tile_first_kernel(const uint64_t* __restrict__ ends, uint64_t n_runs,
                                                             uint64_t n_tiles, uint64_t* __restrict__ tile_first) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b > n_tiles) return;
    const uint64_t r = b * 2048;
    uint64_t lo = 0, hi = n_runs;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (ends[mid] > r) hi = mid;
        else lo = mid + 1;
    }
    tile_first[b] = lo;
}

template <typename T, int PER>
__device__ __forceinline__ void rle_store(T* __restrict__ out, uint64_t r0, uint64_t t1, const T (&v)[PER]) {
    if (r0 + PER <= t1) {  // 32 / 64 contiguous bytes per lane, 16-byte stores
        using V = __attribute__((ext_vector_type(4))) uint32_t;
        V* o = reinterpret_cast<V*>(out + r0);
#pragma unroll
        for (int q = 0; q < (int)(PER * sizeof(T) / 16); ++q) {
            V w;
            __builtin_memcpy(&w, reinterpret_cast<const char*>(v) + 16 * q, 16);
            o[q] = w;
        }
    } else {
        for (int k = 0; k < PER && r0 + k < t1; ++k) out[r0 + k] = v[k];
    }
}

template <typename T>
__global__ __launch_bounds__(256) void rle_expand_kernel(const T* __restrict__ vals, const uint64_t* __restrict__ ends,
                                                         const uint64_t* __restrict__ tile_first, uint64_t n_runs,
                                                         uint64_t n_rows, T* __restrict__ out) {
    constexpr int TILE = 2048, PER = 8, WIN = 2064;  // a tile holds at most 2,048 non-empty runs (+ one empty)
    __shared__ uint64_t s_end[WIN];
    __shared__ T s_val[WIN];
    const uint64_t n_tiles = (n_rows + TILE - 1) / TILE;
    for (uint64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {  // tile-uniform control flow
        const uint64_t t0 = tile * TILE;
        const uint64_t t1 = t0 + TILE < n_rows ? t0 + TILE : n_rows;
        const uint64_t r0 = t0 + (uint64_t)threadIdx.x * PER;
        // the tile's runs: from the first ending past t0 through the first ending past t1 (one
        // more than needed when a run ends at t1 exactly), within the partition's runs
        const uint64_t first = tile_first[tile];
        const uint64_t stop = tile_first[tile + 1] < n_runs ? tile_first[tile + 1] + 1 : n_runs;
        const uint64_t cnt = stop - first;
        T v[PER];
        if (cnt <= 2) {  // inside one run or across one boundary (long runs): no staging
            const uint64_t e0 = ends[first];
            const T a = vals[first], b = cnt == 2 ? vals[first + 1] : a;
#pragma unroll
            for (int k = 0; k < PER; ++k) v[k] = r0 + k < e0 ? a : b;
            if (r0 < t1) rle_store<T, PER>(out, r0, t1, v);
            continue;
        }
        if (cnt <= (uint64_t)WIN) {
            // the tile's runs in LDS; each lane expands 8 consecutive rows: one search, then a walk
            for (uint32_t i = threadIdx.x; i < cnt; i += blockDim.x) {
                s_end[i] = ends[first + i];
                s_val[i] = vals[first + i];
            }
            __syncthreads();
            if (r0 < t1) {
                uint32_t lo = 0, hi = (uint32_t)cnt - 1;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) / 2;
                    if (s_end[mid] > r0) hi = mid;
                    else lo = mid + 1;
                }
#pragma unroll
                for (int k = 0; k < PER; ++k) {
                    while (lo + 1 < cnt && s_end[lo] <= r0 + k) ++lo;
                    v[k] = s_val[lo];
                }
                rle_store<T, PER>(out, r0, t1, v);
            }
            __syncthreads();  // the LDS is the next tile's
            continue;
        }
        // more runs than the window (not produced by DuckDB's writer): windows of runs in turn
        uint64_t f = first, row = t0;
        while (row < t1 && f < n_runs) {
            const uint64_t c = n_runs - f < (uint64_t)WIN ? n_runs - f : (uint64_t)WIN;
            for (uint32_t i = threadIdx.x; i < c; i += blockDim.x) {
                s_end[i] = ends[f + i];
                s_val[i] = vals[f + i];
            }
            __syncthreads();
            const uint64_t covered = s_end[c - 1] < t1 ? s_end[c - 1] : t1;
            for (uint64_t r = row + threadIdx.x; r < covered; r += blockDim.x) {
                uint32_t lo = 0, hi = (uint32_t)c - 1;
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) / 2;
                    if (s_end[mid] > r) hi = mid;
                    else lo = mid + 1;
                }
                out[r] = s_val[lo];
            }
            row = covered;
            f += c;
            __syncthreads();
        }
    }
}

hipError_t launch_rle_expand(const void* vals, const uint64_t* ends, uint64_t n_runs, uint64_t n_rows, int type,
                             uint64_t* tile_first, void* out, hipStream_t stream, hipEvent_t start, hipEvent_t stop) {
    if (n_rows == 0) return hipSuccess;
    const uint64_t tiles = (n_rows + 2047) / 2048;
    if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
    // timed from the first kernel's start to the second's end
    hipExtLaunchKernelGGL(rle_tile_first_kernel, dim3((unsigned)((tiles + 1 + 255) / 256)), dim3(256), 0, stream, start,
                          nullptr, 0, ends, n_runs, tiles, tile_first);
    const unsigned grid = (unsigned)std::min<uint64_t>(tiles, 256 * 16);  // 16 workgroups per CU, tiles in turn
    if (type == 0)
        hipExtLaunchKernelGGL(rle_expand_kernel<int32_t>, dim3(grid), dim3(256), 0, stream, nullptr, stop, 0,
                              static_cast<const int32_t*>(vals), ends, tile_first, n_runs, n_rows,
                              static_cast<int32_t*>(out));
    else
        hipExtLaunchKernelGGL(rle_expand_kernel<int64_t>, dim3(grid), dim3(256), 0, stream, nullptr, stop, 0,
                              static_cast<const int64_t*>(vals), ends, tile_first, n_runs, n_rows,
                              static_cast<int64_t*>(out));
    return hipGetLastError();
}

// A comparison (CUBIT_CMP_* or kCmpBetween) as the inclusive range [lo, hi] of passing values,
// complemented when neg (!=); empty: lo > hi. clamp32 narrows it to INT32 values.
struct CmpRange {
    int64_t lo = INT64_MIN, hi = INT64_MAX;
    int neg = 0;
    void clamp32(int32_t& lo32, int32_t& hi32) const {
        const bool empty = lo > hi || lo > INT32_MAX || hi < INT32_MIN;
        lo32 = empty ? 1 : (int32_t)std::max<int64_t>(lo, INT32_MIN);
        hi32 = empty ? 0 : (int32_t)std::min<int64_t>(hi, INT32_MAX);
    }
};
CmpRange cmp_range(int cmp, int64_t constant, int64_t constant2) {
    CmpRange r;
    switch (cmp) {
    case 0: r.lo = r.hi = constant; break;                                            // =
    case 1: r.lo = r.hi = constant; r.neg = 1; break;                                 // !=
    case 2: if (constant == INT64_MIN) { r.lo = 1; r.hi = 0; } else r.hi = constant - 1; break;  // <
    case 3: r.hi = constant; break;                                                   // <=
    case 4: if (constant == INT64_MAX) { r.lo = 1; r.hi = 0; } else r.lo = constant + 1; break;  // >
    case 5: r.lo = constant; break;                                                   // >=
    default:                                                                          // c <= v < c2
        r.lo = constant;
        if (constant2 == INT64_MIN) { r.lo = 1; r.hi = 0; } else r.hi = constant2 - 1;
        break;
    }
    return r;
}

hipError_t launch_masked_compare(const void* col, int type, const uint64_t* validity, const uint64_t* mask,
                                 uint64_t n_rows, int cmp, int64_t constant, uint64_t* out, hipStream_t stream) {
    const uint64_t nw = padded_words(n_rows);
    const CmpRange r = cmp_range(cmp, constant, 0);
    const dim3 grid(grid_for(nw / 2)), block(256);
    if (type_is32(type)) {
        int32_t lo32, hi32;
        r.clamp32(lo32, hi32);
        if (type == kTypeFloat)
            hipLaunchKernelGGL((masked_compare_kernel<int32_t, 1>), grid, block, 0, stream,
                               static_cast<const int32_t*>(col), validity, mask, nw, lo32, hi32, r.neg, out);
        else
            hipLaunchKernelGGL(masked_compare_kernel<int32_t>, grid, block, 0, stream, static_cast<const int32_t*>(col),
                               validity, mask, nw, lo32, hi32, r.neg, out);
    } else if (type == kTypeDouble) {
        hipLaunchKernelGGL((masked_compare_kernel<int64_t, 2>), grid, block, 0, stream, static_cast<const int64_t*>(col),
                           validity, mask, nw, r.lo, r.hi, r.neg, out);
    } else if (type == kTypeUInt64) {
        hipLaunchKernelGGL(masked_compare_kernel<uint64_t>, grid, block, 0, stream, static_cast<const uint64_t*>(col),
                           validity, mask, nw, (uint64_t)r.lo ^ 0x8000000000000000ull,
                           (uint64_t)r.hi ^ 0x8000000000000000ull, r.neg, out);
    } else {
        hipLaunchKernelGGL(masked_compare_kernel<int64_t>, grid, block, 0, stream, static_cast<const int64_t*>(col),
                           validity, mask, nw, r.lo, r.hi, r.neg, out);
    }
    return hipGetLastError();
}

hipError_t launch_bitpacked_compare(const uint8_t* bytes, const BpGroup* groups, uint64_t n_groups, int type,
                                    const uint64_t* validity, int cmp, int64_t constant, int64_t constant2,
                                    uint64_t* out, hipStream_t stream, int simple_width) {
    if (n_groups == 0) return hipSuccess;
    if (n_groups > 0x7fffffffull) return hipErrorInvalidValue;
    const CmpRange rg = cmp_range(cmp, constant, constant2);
    const int64_t lo = rg.lo, hi = rg.hi;
    const int neg = rg.neg;
    const uint32_t ng = (uint32_t)n_groups;
    if (simple_width > 0) {  // every group FOR ≤ 32 bits / CONSTANT / CONSTANT_DELTA: one wave per group
        const dim3 grid((ng + 3) / 4);
        if (type == 0) {
            int32_t lo32, hi32;
            rg.clamp32(lo32, hi32);
            if (simple_width <= 16)
                hipLaunchKernelGGL((bitpacked_compare_waves<int32_t, uint32_t, 16>), grid, dim3(256), 0, stream, bytes,
                                   groups, ng, validity, lo32, hi32, neg, out);
            else
                hipLaunchKernelGGL((bitpacked_compare_waves<int32_t, uint32_t, 32>), grid, dim3(256), 0, stream, bytes,
                                   groups, ng, validity, lo32, hi32, neg, out);
        } else {
            if (simple_width <= 16)
                hipLaunchKernelGGL((bitpacked_compare_waves<int64_t, uint64_t, 16>), grid, dim3(256), 0, stream, bytes,
                                   groups, ng, validity, lo, hi, neg, out);
            else
                hipLaunchKernelGGL((bitpacked_compare_waves<int64_t, uint64_t, 32>), grid, dim3(256), 0, stream, bytes,
                                   groups, ng, validity, lo, hi, neg, out);
        }
        return hipGetLastError();
    }
    if (type == 0) {
        int32_t lo32, hi32;
        rg.clamp32(lo32, hi32);
        constexpr int GPW = 4;  // groups per workgroup, their loads all in flight together
        hipLaunchKernelGGL((bitpacked_compare_kernel<int32_t, uint32_t, GPW>), dim3((ng + GPW - 1) / GPW), dim3(256),
                           0, stream, bytes, groups, ng, validity, lo32, hi32, neg, out);
    } else {
        constexpr int GPW = 2;  // 16 KiB spans
        hipLaunchKernelGGL((bitpacked_compare_kernel<int64_t, uint64_t, GPW>), dim3((ng + GPW - 1) / GPW), dim3(256),
                           0, stream, bytes, groups, ng, validity, lo, hi, neg, out);
    }
    return hipGetLastError();
}

hipError_t launch_fill_valid(uint64_t* words, uint64_t n_rows, hipStream_t stream) {
    const uint64_t nw = padded_words(n_rows);
    hipLaunchKernelGGL(fill_valid_kernel, dim3(grid_for(nw)), dim3(256), 0, stream, words, n_rows, nw);
    return hipGetLastError();
}

hipError_t launch_zone_classes(const uint64_t* bv, uint64_t n_rows, uint32_t z0, uint32_t nz, uint8_t* out,
                               hipStream_t stream, uint32_t* cnt) {
    if (nz == 0) return hipSuccess;
    hipLaunchKernelGGL(zone_class_kernel, dim3(nz), dim3(256), 0, stream, bv, n_rows, z0, out, cnt);
    return hipGetLastError();
}

hipError_t launch_column_zone_stats(const void* col, int type, const uint64_t* validity, uint64_t n_rows, uint32_t nz,
                                    int64_t* mn, int64_t* mx, uint8_t* fl, hipStream_t stream) {
    if (nz == 0) return hipSuccess;
    if (type == kTypeFloat)
        hipLaunchKernelGGL((column_zone_stats_kernel<int32_t, 1>), dim3(nz), dim3(256), 0, stream,
                           static_cast<const int32_t*>(col), validity, n_rows, mn, mx, fl);
    else if (type == kTypeDouble)
        hipLaunchKernelGGL((column_zone_stats_kernel<int64_t, 2>), dim3(nz), dim3(256), 0, stream,
                           static_cast<const int64_t*>(col), validity, n_rows, mn, mx, fl);
    else if (type == kTypeUInt64)
        hipLaunchKernelGGL((column_zone_stats_kernel<int64_t, 3>), dim3(nz), dim3(256), 0, stream,
                           static_cast<const int64_t*>(col), validity, n_rows, mn, mx, fl);
    else if (type_is32(type))
        hipLaunchKernelGGL(column_zone_stats_kernel<int32_t>, dim3(nz), dim3(256), 0, stream,
                           static_cast<const int32_t*>(col), validity, n_rows, mn, mx, fl);
    else
        hipLaunchKernelGGL(column_zone_stats_kernel<int64_t>, dim3(nz), dim3(256), 0, stream,
                           static_cast<const int64_t*>(col), validity, n_rows, mn, mx, fl);
    return hipGetLastError();
}

hipError_t launch_visibility(const int64_t* del_rows, const uint64_t* del_ids, uint64_t n_del, uint64_t n_rows,
                             uint64_t start_time, uint64_t transaction_id, uint64_t* words, hipStream_t stream,
                             const int64_t* hidden_ranges, uint32_t n_hidden) {
    hipError_t e = launch_fill_valid(words, n_rows, stream);
    if (e != hipSuccess) return e;
    for (uint32_t r0 = 0; r0 < n_hidden; r0 += 65535) {
        const unsigned ny = (unsigned)std::min<uint32_t>(65535, n_hidden - r0);
        hipLaunchKernelGGL(clear_ranges_kernel, dim3(64, ny), dim3(256), 0, stream, hidden_ranges + 2 * (uint64_t)r0,
                           words);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (n_del == 0) return hipSuccess;
    hipLaunchKernelGGL(visibility_kernel, dim3(grid_for(n_del)), dim3(256), 0, stream, del_rows, del_ids, n_del,
                       start_time, transaction_id, words);
    return hipGetLastError();
}

hipError_t launch_splice_bits(uint64_t* dst, const uint64_t* src, uint64_t bit_off, uint64_t n_bits,
                              hipStream_t stream) {
    if (n_bits == 0) return hipSuccess;
    const uint64_t words = ((bit_off + n_bits + 63) >> 6) - (bit_off >> 6);
    hipLaunchKernelGGL(splice_bits_kernel, dim3(grid_for(words)), dim3(256), 0, stream, dst, src, bit_off, n_bits);
    return hipGetLastError();
}

hipError_t launch_merge_words(const int64_t* rows, const int64_t* values, const uint8_t* valids, uint64_t m,
                              uint64_t n_rows, void* col, int type, uint64_t* validity, MergeIndex ix0, MergeIndex ix1,
                              hipStream_t stream) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(merge_words_kernel, dim3(grid_for(m)), dim3(256), 0, stream, rows, values, valids, m,
                       n_rows, col, type, validity, ix0, ix1);
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
