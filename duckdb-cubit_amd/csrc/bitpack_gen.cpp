// Bench input: DuckDB BITPACKING segment images of a column (the layout K5 consumes), built
// in parallel on the host. This is synthetic-input generation for bench.py's K5 leg, not a
// restatement of the reference compressor (that one is oracle/bitpacking_ref.c, test-only):
// every 2,048-value group is written as CONSTANT when min == max and as FOR otherwise, the
// two modes the reference's AUTO choice gives TPC-H lineitem's unsorted columns
// (BitpackingState::Flush, src/storage/compression/bitpacking.cpp:220-320).
// Segment image (bitpacking.cpp:474-540): 8-byte header = end of the metadata words; group
// data from byte 8 upward; one metadata word per group (data offset | mode << 24) growing
// down, compacted behind the 8-aligned data when the segment is closed. Segments never span
// a 122,880-row row group (each row group has its own column segments), so row groups pack
// independently, one thread per range of row groups.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

constexpr uint64_t kGroup = 2048;
constexpr uint64_t kRowGroup = 122880;
constexpr uint32_t kModeConstant = 2, kModeFor = 5;

struct Seg {
    uint64_t off, rows;
};

// GetEffectiveWidth (src/include/duckdb/common/bitpacking.hpp): widths within tsize bits of
// the type's width round up to the full width
int for_width(uint64_t range, int tsize) {
    int w = range ? 64 - __builtin_clzll(range) : 0;
    return w + tsize > 8 * tsize ? 8 * tsize : w;
}

struct Packer {
    const uint8_t* vals;
    int tsize;
    uint64_t block;
    std::vector<uint8_t> out;
    std::vector<Seg> segs;
    std::vector<uint8_t> blk;
    uint64_t data = 8, meta = 0, rows = 0;

    int64_t at(uint64_t i) const {
        if (tsize == 4) {
            int32_t x;
            std::memcpy(&x, vals + 4 * i, 4);
            return x;
        }
        int64_t x;
        std::memcpy(&x, vals + 8 * i, 8);
        return x;
    }
    void begin() {
        blk.assign(block, 0);
        data = 8;
        meta = block;
        rows = 0;
    }
    void close() {
        if (rows == 0) return;
        const uint64_t meta_at = (data + 7) / 8 * 8, meta_size = block - meta;
        std::memmove(blk.data() + meta_at, blk.data() + meta, meta_size);
        const uint64_t header = meta_at + meta_size;
        std::memcpy(blk.data(), &header, 8);
        out.resize((out.size() + 7) / 8 * 8);
        segs.push_back({out.size(), rows});
        out.insert(out.end(), blk.begin(), blk.begin() + header);
        begin();
    }
    bool fits(uint64_t bytes) const { return (data + bytes + 7) / 8 * 8 + (block - meta) + 4 <= block - 8; }
    void put(int64_t v) {
        std::memcpy(blk.data() + data, &v, tsize);  // little-endian: the low tsize bytes
        data += tsize;
    }
    void group(uint64_t b, uint64_t count) {
        int64_t mn = at(b), mx = mn;
        for (uint64_t i = 1; i < count; ++i) {
            const int64_t x = at(b + i);
            mn = std::min(mn, x);
            mx = std::max(mx, x);
        }
        const uint64_t umask = tsize == 4 ? 0xffffffffull : ~0ull;
        const int w = for_width(((uint64_t)mx - (uint64_t)mn) & umask, tsize);
        const uint64_t packed = mn == mx ? 0 : (count + 31) / 32 * 32 * (uint64_t)w / 8;
        const uint64_t bytes = mn == mx ? (uint64_t)tsize : 2 * (uint64_t)tsize + packed;
        if (!fits(bytes)) close();
        meta -= 4;
        const uint32_t enc = (uint32_t)(data & 0x00ffffffu) | ((mn == mx ? kModeConstant : kModeFor) << 24);
        std::memcpy(blk.data() + meta, &enc, 4);
        put(mn);
        if (mn != mx) {
            put(w);
            uint32_t* words = reinterpret_cast<uint32_t*>(blk.data() + data);  // 4-aligned
            const uint64_t mask = w == 64 ? ~0ull : (1ull << w) - 1;
            for (uint64_t i = 0; i < count; ++i) {
                const uint64_t x = ((uint64_t)at(b + i) - (uint64_t)mn) & mask;
                const uint64_t bit = i * (uint64_t)w;
                const uint32_t wi = (uint32_t)(bit >> 5), off = (uint32_t)(bit & 31);
                words[wi] |= (uint32_t)(x << off);
                if (off + w > 32) words[wi + 1] |= (uint32_t)(x >> (32 - off));
                if (off + w > 64) words[wi + 2] |= (uint32_t)(x >> (64 - off));
            }
            data += packed;
        }
        rows += count;
    }
};

}  // namespace

extern "C" {

// Pack n values (tsize 4 or 8) into segments of block_size bytes. Writes the images to out
// (capacity out_cap), segment i at seg_off[i] (8-aligned) holding seg_rows[i] rows, and
// returns the number of segments, or 0 when out_cap / max_segs is too small or the input is
// invalid. *out_bytes = bytes used.
uint32_t cubit_bitpack_for(const void* values, int tsize, uint64_t n, uint64_t block_size, uint8_t* out,
                           uint64_t out_cap, uint64_t* seg_off, uint64_t* seg_rows, uint32_t max_segs,
                           uint64_t* out_bytes, int nthreads) {
    if (!values || !out || !seg_off || !seg_rows || !out_bytes || (tsize != 4 && tsize != 8) || n == 0 ||
        block_size < 64 * 1024 || block_size > (1u << 24))
        return 0;
    const uint64_t n_rg = (n + kRowGroup - 1) / kRowGroup;
    if (nthreads <= 0) nthreads = (int)std::max(1u, std::min(std::thread::hardware_concurrency(), 16u));
    nthreads = (int)std::min<uint64_t>((uint64_t)nthreads, n_rg);
    std::vector<Packer> parts(nthreads);
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) {
        th.emplace_back([&, t] {
            Packer& p = parts[t];
            p.vals = static_cast<const uint8_t*>(values);
            p.tsize = tsize;
            p.block = block_size;
            p.begin();
            const uint64_t rb = n_rg * t / nthreads, re = n_rg * (t + 1) / nthreads;
            for (uint64_t rg = rb; rg < re; ++rg) {
                const uint64_t r0 = rg * kRowGroup, r1 = std::min(n, r0 + kRowGroup);
                for (uint64_t g = r0; g < r1; g += kGroup) p.group(g, std::min(kGroup, r1 - g));
                p.close();
            }
        });
    }
    for (auto& x : th) x.join();
    uint64_t used = 0;
    uint32_t ns = 0;
    for (const Packer& p : parts) {
        used = (used + 7) / 8 * 8;
        if (used + p.out.size() > out_cap || ns + p.segs.size() > max_segs) return 0;
        std::memcpy(out + used, p.out.data(), p.out.size());
        for (const Seg& s : p.segs) {
            seg_off[ns] = used + s.off;
            seg_rows[ns] = s.rows;
            ++ns;
        }
        used += p.out.size();
    }
    *out_bytes = used;
    return ns;
}

}  // extern "C"
