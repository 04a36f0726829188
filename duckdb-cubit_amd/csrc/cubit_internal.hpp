// Internal interfaces shared by the HIP kernels (cubit_kernels.hip) and the C ABI /
// planner (cubit_capi.hip). Not installed; the public surface is include/cubit_gpu.h.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace cubit {

// DuckDB storage geometry (src/include/duckdb/common/vector_size.hpp:16-20,
// src/include/duckdb/storage/storage_info.hpp:20). Both are whole 64-bit words, so vector
// and row-group boundaries never split a bitvector word.
constexpr uint64_t kVectorSize = 2048;
constexpr uint64_t kRowGroupSize = 122880;
static_assert(kVectorSize % 64 == 0 && kVectorSize / 64 == 32, "vector must be 32 words");
static_assert(kRowGroupSize % 64 == 0 && kRowGroupSize / 64 == 1920, "row group must be 1920 words");

// Filter kernel geometry: 256-thread workgroups; each thread owns PAIRS 16-byte word pairs
// per leaf (one dwordx4 load per pair; a wave-instruction moves 1 KiB). Bitvectors are padded
// to kPadWords so every tile shape reads in bounds.
constexpr int kThreads = 256;
constexpr uint64_t kPadWords = 16384;  // 1,048,576 rows
constexpr int kMaxLeaves = 8;
constexpr int kMaxOps = 16;  // 2 bits each in EvalProgram::ops

enum : uint32_t { OP_AND = 1, OP_OR = 2, OP_ANDNOT = 3 };

// A postfix program whose leaves appear in order 0..n_leaves-1: leaf k is pushed
// (complemented if bit k of `negate`), then nops(k) binary ops are applied. The op counts
// (4 bits per leaf) and opcodes (2 bits per op) are packed into words so the kernel decodes
// them with scalar shifts (a runtime-indexed byte array in the kernel arguments compiles to
// vector loads, each followed by an s_waitcnt vmcnt(0) that drains every outstanding load).
// Evaluation forms: the general postfix interpreter, or a branch-free two-level form chosen
// by the planner's emitter (leaves ordered by group, gstart bit k = leaf k opens a group).
enum : uint32_t { FORM_POSTFIX = 0, FORM_CONJ = 1, FORM_DNF = 2, FORM_CNF = 3 };

struct EvalProgram {
    const uint64_t* leaf[kMaxLeaves];
    uint32_t negate;
    uint32_t n_leaves;
    uint32_t nops;    // 4 bits per leaf
    uint32_t ops;     // 2 bits per op
    uint32_t form;    // FORM_*; FORM_POSTFIX runs the postfix program (is_conjunction upgrades)
    uint32_t gstart;  // FORM_DNF / FORM_CNF group starts
};

inline uint32_t prog_nops(const EvalProgram& p, int k) { return (p.nops >> (4 * k)) & 15u; }

// Column value types as the kernels see them: INT32 / INT64 values, or FLOAT / DOUBLE bit patterns
// (4 / 8 bytes) compared through their order key (cubit_fp_key, include/cubit_gpu.h: NaN one key
// above +inf, -x → -pattern(x), so -0.0 == +0.0 — DuckDB's floating-point operators,
// comparison_operators.hpp:100-146). Type codes as in cubit_gpu.h.
// VARCHAR columns hold int32 codes of an order-preserving dictionary (cubit_dict): compared as
// INT32 values, the codes order as the strings do.
// UBIGINT (UINT64) columns hold the unsigned values' bits, compared through the key v ^ 2^63 (the
// unsigned order as a signed one).
constexpr int kTypeInt32 = 0, kTypeInt64 = 1, kTypeUInt64 = 7, kTypeFloat = 8, kTypeDouble = 9, kTypeVarchar = 10;
__host__ __device__ __forceinline__ bool type_is32(int type) {
    return type == kTypeInt32 || type == kTypeFloat || type == kTypeVarchar;
}
__host__ __device__ __forceinline__ bool type_is_fp(int type) { return type == kTypeFloat || type == kTypeDouble; }
// the type a table's compare kernels see for a column: FLOAT / DOUBLE columns keep their keys as an
// INT32 / INT64 column beside the patterns
__host__ __device__ __forceinline__ int key_type(int type) {
    return type == kTypeFloat ? kTypeInt32 : type == kTypeDouble ? kTypeInt64 : type;
}
// values compared through a key other than themselves (FLOAT, DOUBLE, UBIGINT)
__host__ __device__ __forceinline__ bool type_is_keyed(int type) { return type_is_fp(type) || type == kTypeUInt64; }
__host__ __device__ __forceinline__ int32_t fp_key32(uint32_t u) {
    const uint32_t mag = u & 0x7fffffffu;
    if (mag > 0x7f800000u) return 0x7fc00000;
    return (u >> 31) ? -(int32_t)mag : (int32_t)mag;
}
__host__ __device__ __forceinline__ int64_t fp_key64(uint64_t u) {
    const uint64_t mag = u & 0x7fffffffffffffffull;
    if (mag > 0x7ff0000000000000ull) return (int64_t)0x7ff8000000000000ull;
    return (u >> 63) ? -(int64_t)mag : (int64_t)mag;
}
// the comparison key of a value as the ABI carries it (FLOAT: the zero-extended 32-bit pattern)
__host__ __device__ __forceinline__ int64_t value_key(int type, int64_t v) {
    if (type == kTypeFloat) return fp_key32((uint32_t)v);
    if (type == kTypeDouble) return fp_key64((uint64_t)v);
    if (type == kTypeUInt64) return (int64_t)((uint64_t)v ^ 0x8000000000000000ull);
    return v;
}
// kernels templated on the key kind FK (0: the value itself, 1: FLOAT pattern, 2: DOUBLE pattern,
// 3: UBIGINT bits)
template <int FK, typename T>
__host__ __device__ __forceinline__ T key_of(T raw) {
    if constexpr (FK == 1) return (T)fp_key32((uint32_t)raw);
    else if constexpr (FK == 2) return (T)fp_key64((uint64_t)raw);
    else if constexpr (FK == 3) return (T)((uint64_t)raw ^ 0x8000000000000000ull);
    else return raw;
}

inline uint64_t padded_words(uint64_t n_rows) {
    const uint64_t w = (n_rows + 63) / 64;
    return ((w + kPadWords - 1) / kPadWords) * kPadWords;
}

struct EvalArgs {
    EvalProgram prog;
    uint64_t n_rows;
    uint64_t n_words;  // ceil(n_rows / 64)
    int64_t row_base;
    int64_t* rowids;
    uint64_t capacity;
    uint64_t* count;         // result: the number of qualifying rows (written at kernel end)
    uint64_t* result_words;  // optional evaluated bitvector
    uint32_t num_tiles;
    // claim ticket (context-owned, kTicketWords words, zero between launches): running claim
    // counter + arrival counters. The last workgroup to finish publishes *count and re-zeroes
    // the ticket, so no memset launch precedes a scan (finish_ticket, cubit_kernels.hip).
    uint64_t* ticket;
    // zonemap skip (device, ascending): the tiles to evaluate, num_tiles entries; null = every
    // tile 0 … num_tiles-1. The planner leaves out the tiles whose zone classes prove the program
    // false on every row (RowGroup::CheckZonemap, row_group.cpp:361-371, over bitvector zones).
    const uint32_t* live;
    // eval_decode_lookback: context-owned flag words (kLookbackMaxTiles, zeroed once) and the
    // launch's epoch (> 0, one per launch on the context), which tags every flag it publishes
    uint64_t* flags;
    uint64_t epoch;
    // polls of one flag before the polling thread counts that tile itself (0 = the kernel's
    // default; cubit_ctx_set_lookback_spins forces the recount path in tests)
    uint32_t spin_limit;
    // eval_decode_lookback: exclusive prefix of every tile's qualifying rows, known before the
    // launch (a program of one index bitvector: its per-zone counts, a zone being one decode
    // tile), or null. With it no workgroup publishes or waits, at any tile count.
    const uint64_t* tile_prefix;
};
// eval_decode_lookback: one workgroup per tile, at most this many tiles per launch (6.0e8 rows).
// Every workgroup reads the counts of all earlier tiles, so the flag reads grow with the square
// of the tile count: at 4,578 tiles (SF100) the kernel takes 68.5 µs against 64.7 µs for the
// run-claimed decode; larger launches are not measured, so ordered scans past this size keep the
// run-claimed decode + ordering pass.
constexpr uint32_t kLookbackMaxTiles = 4608;
// Zonemaps: one zone = one decode tile (2,048 words = 131,072 rows). Class byte per zone:
// bit 0 = no row of the zone is set, bit 1 = every row of the zone is set (a zone past the
// last row has both).
constexpr uint64_t kZoneWords = 2048;
constexpr uint64_t kZoneRows = kZoneWords * 64;
constexpr uint32_t kTicketStride = 64;  // words (512 B) between ticket counters
constexpr uint32_t kTicketGroups = 8;
constexpr uint32_t kTicketWords = kTicketStride * (kTicketGroups + 2);

// launchers (cubit_kernels.hip); all asynchronous on `stream`
uint64_t decode_tile_words();  // words per eval_decode_tiles tile
uint64_t count_tile_words(uint32_t n_leaves);  // words per eval_count_kernel tile
int decode_block_threads();
// evaluate + decode into per-tile runs; dir (optional) gets {start, length} per tile
// ev0 / ev1 (optional): events stamped by the kernel dispatch itself (hipExtLaunchKernel), so
// their elapsed time is the kernel's execution, as rocprofv3's kernel trace reports it
// kernel: 0 = by the measured policy (launch_decode_kf), 1 = pair-claimed, 2 = run-claimed,
// 3 = look-back (one tile per workgroup, runs in tile order: small partitions by policy —
// lookback_max_tiles — and ordered scans up to kLookbackMaxTiles); decode_kernel_for resolves
// it for a launch
int decode_kernel_for(uint32_t n_leaves, uint32_t num_tiles, unsigned grid, int kernel, bool live = false,
                      int n_cus = 256, bool prefixed = false);
// the largest tile count the measured policy decodes with the look-back kernel (grid = tiles)
uint32_t lookback_max_tiles(uint32_t n_leaves, int n_cus);
hipError_t launch_eval_decode(const EvalArgs& a, uint64_t* dir, unsigned grid, hipStream_t stream,
                              hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr, int kernel = 0, int n_cus = 256);
// zone classes of a bitvector (class byte per zone, see kZoneWords) for zones [z0, z0 + nz),
// and (cnt non-null) each zone's set rows
hipError_t launch_zone_classes(const uint64_t* bv, uint64_t n_rows, uint32_t z0, uint32_t nz, uint8_t* out,
                               hipStream_t stream, uint32_t* cnt = nullptr);
// per-zone min / max of a raw column's valid rows; fl bit 0 = some row valid, bit 1 = every row
hipError_t launch_column_zone_stats(const void* col, int type, const uint64_t* validity, uint64_t n_rows, uint32_t nz,
                                    int64_t* mn, int64_t* mx, uint8_t* fl, hipStream_t stream);
// evaluate + count (and/or write the result bitvector)
hipError_t launch_eval_count(const EvalArgs& a, hipStream_t stream, hipEvent_t ev0 = nullptr,
                             hipEvent_t ev1 = nullptr);
// lay per-tile runs out in row order: dst[dst_off[i] ...] = src[dir run i]
hipError_t launch_order_runs(const uint64_t* dir, uint32_t n_tiles, uint64_t* dst_off, const int64_t* src,
                             uint64_t capacity, int64_t* dst, hipStream_t stream);
// cmp = CUBIT_CMP_* (0..5) or kCmpBetween (constant <= v < constant2)
constexpr int kCmpBetween = 6;
hipError_t launch_compare_bitvector(const void* col, int type, const uint64_t* validity, uint64_t n_rows, int cmp,
                                    int64_t constant, uint64_t* out_words, hipStream_t stream, int64_t constant2 = 0);
// candidate check of a constant inside one bin [k_lo, k_hi) of a range index: cand =
// hi_bv \ lo_bv (lo_bv null = ∅, hi_bv null = every valid row); out = (cmp LT: lo_bv ∪)
// {r ∈ cand : v[r] cmp constant}; cmp ∈ {CUBIT_CMP_EQ, CUBIT_CMP_LT}
hipError_t launch_candidate_check(const void* col, int type, const uint64_t* validity, const uint64_t* lo_bv,
                                  const uint64_t* hi_bv, uint64_t n_rows, int cmp, int64_t constant,
                                  uint64_t* out_words, hipStream_t stream);
// selection narrowing: out = mask ∩ valid ∩ {v cmp constant}, the column read at mask rows only
hipError_t launch_masked_compare(const void* col, int type, const uint64_t* validity, const uint64_t* mask,
                                 uint64_t n_rows, int cmp, int64_t constant, uint64_t* out, hipStream_t stream);
// K0 over several keys in one pass of the column (index build): out[k] = cmp(v, c[k], c2[k]),
// cmp ∈ {EQ, LT, between}
constexpr int kMultiKeys = 16;
struct MultiKeyArgs {
    int64_t c[kMultiKeys];
    int64_t c2[kMultiKeys];
    uint64_t* out[kMultiKeys];
    uint32_t m;
};
hipError_t launch_compare_bitvectors(const void* col, int type, const uint64_t* validity, uint64_t n_rows, int cmp,
                                     const MultiKeyArgs& a, hipStream_t stream);
// index-build statistics (out3 = {min, max, valid count}, pre-set by the caller) and the
// presence bitmap of the valid values (bit v - vmin, `range` bits, zeroed by the caller)
hipError_t launch_column_minmax(const void* col, int type, const uint64_t* validity, uint64_t n_rows, int64_t* out3,
                                hipStream_t stream);
hipError_t launch_presence(const void* col, int type, const uint64_t* validity, uint64_t n_rows, int64_t vmin,
                           uint64_t range, uint64_t* bits, hipStream_t stream);
// K5: DuckDB BITPACKING groups → plain values. One record per 2,048-value metadata group
// (mode: 2 CONSTANT, 3 CONSTANT_DELTA, 4 DELTA_FOR, 5 FOR — BitpackingMode).
// The host reads each group's header (the T-sized fields before the packed words) into the
// record, so a workgroup's only dependent load chain is record → packed words.
struct BpGroup {
    uint64_t words_off;  // byte offset of the packed words (FOR / DELTA_FOR)
    uint64_t row_start;  // first row of the group
    uint64_t base;       // CONSTANT value | CONSTANT_DELTA first | FOR minimum | DELTA_FOR min_delta (T bits)
    uint64_t aux;        // CONSTANT_DELTA delta | DELTA_FOR delta_offset (T bits)
    uint32_t count;      // rows in the group (≤ 2,048)
    uint8_t mode;
    // the segments' T when narrower than the column's values (an 8- / 16-bit T in an INT32
    // column, UINT32 in an INT64 column): its bits | 0x80 when signed; 0 = T is the column's
    // type. Decoded values are taken mod 2^bits and sign- or zero-extended (bp_norm), which is
    // T's own wrap-around arithmetic
    uint8_t tnorm;
    uint16_t width;      // bit width of the packed values (FOR / DELTA_FOR)
};
hipError_t launch_bitunpack(const uint8_t* bytes, const BpGroup* groups, uint64_t n_groups, int type, void* out,
                            hipStream_t stream, hipEvent_t start = nullptr, hipEvent_t stop = nullptr);
// strings → codes of a sorted dictionary, all on the device (NULL rows 0; a missing string -1,
// counted into *missing)
hipError_t launch_dict_encode(const uint8_t* bytes, const uint64_t* offs, uint64_t n, const uint64_t* validity,
                              const uint8_t* dbytes, const uint64_t* doffs, uint64_t dn, int32_t* codes,
                              unsigned long long* missing, hipStream_t stream);
// DuckDB RLE segments parsed into runs (values of the column's type, cumulative exclusive run
// ends) expanded into the column (type 0: INT32, else INT64); tile_first: scratch of
// (n_rows + 2047) / 2048 + 1 words
hipError_t launch_rle_expand(const void* vals, const uint64_t* ends, uint64_t n_runs, uint64_t n_rows, int type,
                             uint64_t* tile_first, void* out, hipStream_t stream, hipEvent_t start, hipEvent_t stop);
// K5 + K0 fused: {valid rows whose value cmp constant} straight from the BITPACKING groups
// (cmp = CUBIT_CMP_* or kCmpBetween); out must be zero (words shared by two groups are OR-ed)
// simple_width > 0: every group is FOR of ≤ 32 bits, CONSTANT or CONSTANT_DELTA, and the widest
// FOR group has ≤ simple_width bits (bitpacked_compare_waves); 0: the LDS kernel
hipError_t launch_bitpacked_compare(const uint8_t* bytes, const BpGroup* groups, uint64_t n_groups, int type,
                                    const uint64_t* validity, int cmp, int64_t constant, int64_t constant2,
                                    uint64_t* out, hipStream_t stream, int simple_width = 0);
// out[i] = (int32)(in[i] - offset), i < min(*d_count, max_n) (transfer compaction of a column)
// out[i] = (unsigned width-byte)(in[i] - offset), width 1 / 2 / 4; *overflow = 1 when a value
// falls outside [offset, offset + 2^(8·width))
hipError_t launch_narrow_unsigned(const int64_t* in, const uint64_t* d_count, uint64_t max_n, int64_t offset, int width,
                                  void* out, uint32_t* overflow, hipStream_t stream);
// a narrower / unsigned column (CUBIT_TYPE_INT8 … UINT64) widened to its INT32 / INT64 storage
hipError_t launch_widen(const void* in, int src_type, uint64_t n, void* out, hipStream_t stream);
hipError_t launch_narrow_i32(const int64_t* in, const uint64_t* d_count, uint64_t max_n, int64_t offset, int32_t* out,
                             hipStream_t stream, uint32_t* overflow = nullptr);
// FLOAT / DOUBLE columns: keys[i] = the comparison key of pattern raw[i] (the column the compare
// kernels read); out[i] = value_key(type, v[i]); raw[rows[i]] = v[i] (0 where valids[i] = 0)
hipError_t launch_fp_keys(const void* raw, int type, uint64_t n, void* keys, hipStream_t stream);
hipError_t launch_value_keys(const int64_t* v, uint64_t n, int type, int64_t* out, hipStream_t stream);
hipError_t launch_scatter_raw(const int64_t* rows, const int64_t* v, const uint8_t* valids, uint64_t m, int type,
                              void* raw, hipStream_t stream);
hipError_t launch_gather(const void* col, int type, const int64_t* rowids, const uint64_t* d_count, uint64_t max_n,
                         int64_t row_base, int64_t* out, hipStream_t stream);
// the probe with NULL-ness: values (0 at NULL rows) and out_valid bit i = row rowids[i] valid
// (⌈min(*d_count, max_n) / 64⌉ words written; validity nullptr = every row valid)
hipError_t launch_gather_valid(const void* col, int type, const uint64_t* validity, const int64_t* rowids,
                               const uint64_t* d_count, uint64_t max_n, int64_t row_base, int64_t* out,
                               uint64_t* out_valid, hipStream_t stream);
hipError_t launch_gather_sum_product(const int64_t* a, const int64_t* b, const int64_t* rowids,
                                     const uint64_t* d_count, uint64_t max_n, int64_t row_base, int64_t* partials,
                                     int64_t* out, hipStream_t stream);
constexpr int kSumBlocks = 1024;  // partials buffer holds 2 * kSumBlocks int64

// Fused filter + probe + reduce: sum(a[r] * b[r]) over the qualifying rows r (K1+K3).
// b = nullptr: b is decoded from its range index, b = v0 + Σ_j delta[j]·[r ∉ dleaf[j]]
// (dleaf[j] = L(v_j), the filter pins b to v0 < v1 < … ≤ kMaxDecode+1 values).
constexpr int kMaxDecode = 3;
struct SumArgs {
    const int64_t* a;
    const uint64_t* a_valid;  // optional
    const int64_t* b;         // nullptr → decode
    const uint64_t* b_valid;  // optional (gather mode)
    const uint64_t* dleaf[kMaxDecode];
    int64_t delta[kMaxDecode];
    int64_t v0;
    uint32_t n_decode;
    int64_t* partials;  // 2 int64 (lo, hi) per workgroup
    // a read from its DuckDB BITPACKING segments instead of the plain column (null = plain):
    // the packed bytes, the group records (BpGroup, row order) and per 2,048-row vector the
    // index of the group holding its first row. CONSTANT / CONSTANT_DELTA / FOR groups are
    // random-accessible (value i = base (+ aux·i | + its w bits at bit i·w)); a row of a
    // DELTA_FOR group is read from a_plain (the unpacked column), as its value needs the prefix
    // of its group.
    const uint8_t* a_bytes;
    const BpGroup* a_groups;
    const uint32_t* a_vgroup;
    const int64_t* a_plain;
    uint64_t a_n_groups;
};
// grid = persistent workgroups; partials must hold 2·grid int64; out = {lo, hi}
hipError_t launch_eval_sum_product(const EvalArgs& a, const SumArgs& s, unsigned grid, int64_t* out, hipStream_t stream);
unsigned sum_product_grid(unsigned n_cus);
// sum over i < *d_count of x[i]·y[i] (MVCC fallback of the fused path)
hipError_t launch_sum_product_arrays(const int64_t* x, const int64_t* y, const uint64_t* d_count, uint64_t max_n,
                                     int64_t* partials, int64_t* out, hipStream_t stream);

// MVCC (K4)
// visibility: words = valid-row mask, then clear rows whose delete is visible to txn
hipError_t launch_visibility(const int64_t* del_rows, const uint64_t* del_ids, uint64_t n_del, uint64_t n_rows,
                             uint64_t start_time, uint64_t transaction_id, uint64_t* words, hipStream_t stream,
                             const int64_t* hidden_ranges = nullptr, uint32_t n_hidden = 0);
// mark rows with an update visible to txn into `mask` (atomicOr)
hipError_t launch_update_mask(const int64_t* upd_rows, const uint64_t* upd_versions, uint64_t n_upd,
                              uint64_t start_time, uint64_t transaction_id, uint64_t* mask, hipStream_t stream);
hipError_t launch_fill_valid(uint64_t* words, uint64_t n_rows, hipStream_t stream);

// Index maintenance. Append: splice n_bits bits of src (bit 0 = first appended row) into dst
// at bit offset bit_off (dst words outside the splice untouched). Merge: base values of the
// merged rows replaced (rows become valid) and the bits of every index bitvector whose
// predicate changes for a row flipped. encoding: 0 range L(k) = {v < k}, 1 equality, 2 bins
// (keys = edges, n_keys - 1 bitvectors); bvs = nullptr: no index.
struct MergeIndex {
    const int64_t* keys;  // device, sorted
    uint64_t* const* bvs; // device array of bitvector pointers
    uint32_t n_keys;
    int32_t encoding;
};
hipError_t launch_splice_bits(uint64_t* dst, const uint64_t* src, uint64_t bit_off, uint64_t n_bits,
                              hipStream_t stream);
// merge by 64-row words: the m merged records' rows ascend, each row once; valids: per record
// 1 = the value, 0 = NULL (nullptr: every row valid; a NULL needs `validity`)
hipError_t launch_merge_words(const int64_t* rows, const int64_t* values, const uint8_t* valids, uint64_t m,
                              uint64_t n_rows, void* col, int type, uint64_t* validity, MergeIndex ix0, MergeIndex ix1,
                              hipStream_t stream);
}  // namespace cubit
