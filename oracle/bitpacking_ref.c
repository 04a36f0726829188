/*
 * ORACLE — test infrastructure only (never linked into the product). A plain-C restatement of
 * DuckDB v1.1.2's BITPACKING column compression, so tests can build real segments in that
 * format and check the GPU unpack (K5) against a CPU decode of the same bytes.
 *
 * Restated from src/storage/compression/bitpacking.cpp:
 *   metadata word = group data offset | mode << 24                     (EncodeMeta, :62-75)
 *   BitpackingState::Update / Flush: per 2,048-value group choose       (:100-320)
 *     CONSTANT        (all NULL or min == max; AUTO or forced)
 *     CONSTANT_DELTA  (all valid, one distinct delta; not forced FOR/DELTA_FOR)
 *     DELTA_FOR       (delta width < signed value width; not forced FOR)
 *     FOR             (max - min does not overflow)
 *   writers: CONSTANT [T] | CONSTANT_DELTA [T first][T delta] |
 *            DELTA_FOR [T min_delta][T width][T delta_offset][packed] |
 *            FOR [T min][T width][packed]                              (BitpackingWriter, :375-435)
 *   segments: 8-byte header, group data growing up, metadata words growing down from the block
 *            end, compacted behind the 8-aligned data on flush; header = end of metadata
 *            (CanStore / CreateEmptySegment / FlushSegment, :474-540)
 *   scan: LoadNextGroup / BitpackingScanPartial / DeltaDecode          (:585-870)
 * and from src/include/duckdb/common/bitpacking.hpp: 32-value algorithm groups packed
 * horizontally (value i of a group at bits [i·w, (i+1)·w) of little-endian 32-bit words,
 * fastpforlib fastpack), MinimumBitWidth / GetEffectiveWidth (:84-210).
 * Values are INT32 (DATE, INTEGER, DECIMAL ≤ 9) or INT64 (BIGINT, DECIMAL 10..18).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "cpu_ref.h"

#define BP_GROUP 2048
#define BP_ALG 32

/* BitpackingMode (src/include/duckdb/storage/compression/bitpacking.hpp:15) */
enum { BP_INVALID = 0, BP_AUTO = 1, BP_CONSTANT = 2, BP_CONSTANT_DELTA = 3, BP_DELTA_FOR = 4, BP_FOR = 5 };

/* ---------------------------------------------------------------- width helpers */

/* unsigned bits of v (v ≥ 0), through GetEffectiveWidth */
static int eff_width(int w, int tsize) {
    const int bits = tsize * 8;
    return (w + tsize > bits) ? bits : w;
}
static int width_unsigned(uint64_t v, int tsize) {
    int w = 0;
    while (v) {
        w++;
        v >>= 1;
    }
    return w == 0 ? 0 : eff_width(w, tsize);
}
/* MinimumBitWidth<T signed>(value, value) for value ≥ 0: one sign bit more */
static int width_signed_nonneg(int64_t v, int tsize) {
    if (v == 0) return 0;
    int w = 1;
    uint64_t x = (uint64_t)v;
    while (x) {
        w++;
        x >>= 1;
    }
    return eff_width(w, tsize);
}

static int64_t tmin(int tsize) { return tsize == 4 ? INT32_MIN : INT64_MIN; }
static int64_t tmax(int tsize) { return tsize == 4 ? INT32_MAX : INT64_MAX; }
static int sub_ok(int64_t a, int64_t b, int tsize, int64_t *out) {
    if (tsize == 4) {
        const int64_t r = a - b;
        if (r < INT32_MIN || r > INT32_MAX) return 0;
        *out = r;
        return 1;
    }
    return !__builtin_sub_overflow(a, b, out);
}
static uint64_t umask(int tsize) { return tsize == 4 ? 0xffffffffull : ~0ull; }

/* ---------------------------------------------------------------- packing */

static void pack_values(uint8_t *dst, const uint64_t *v, uint64_t count, int w) {
    const uint64_t n = (count + BP_ALG - 1) / BP_ALG * BP_ALG;
    const uint64_t bytes = n * (uint64_t)w / 8;
    memset(dst, 0, bytes);
    if (w == 0) return;
    uint32_t *words = (uint32_t *)dst;
    const uint64_t mask = w == 64 ? ~0ull : ((1ull << w) - 1);
    for (uint64_t i = 0; i < n; i++) {
        uint64_t x = (i < count ? v[i] : 0) & mask;
        uint64_t bit = i * (uint64_t)w;
        int left = w;
        while (left > 0) {
            const uint64_t wi = bit >> 5;
            const int off = (int)(bit & 31);
            const int take = (32 - off) < left ? (32 - off) : left;
            words[wi] |= (uint32_t)((x & ((take == 64) ? ~0ull : ((1ull << take) - 1))) << off);
            x >>= take;
            bit += (uint64_t)take;
            left -= take;
        }
    }
}

static uint64_t unpack_value(const uint8_t *src, uint64_t i, int w) {
    if (w == 0) return 0;
    const uint32_t *words = (const uint32_t *)src;
    uint64_t bit = i * (uint64_t)w, x = 0;
    int got = 0;
    while (got < w) {
        const uint64_t wi = bit >> 5;
        const int off = (int)(bit & 31);
        const int take = (32 - off) < (w - got) ? (32 - off) : (w - got);
        const uint64_t part = ((uint64_t)words[wi] >> off) & ((1ull << take) - 1);
        x |= part << got;
        got += take;
        bit += (uint64_t)take;
    }
    return x;
}

/* ---------------------------------------------------------------- compressor */

typedef struct {
    uint8_t *out;          /* whole output (all segments) */
    uint64_t out_cap;
    uint64_t out_used;     /* bytes of finished segments */
    uint64_t block_size;
    uint8_t *blk;          /* current segment image (block_size bytes) */
    uint64_t data_off;     /* next free data byte */
    uint64_t meta_off;     /* lowest metadata byte */
    uint64_t seg_rows;
    uint64_t *seg_off, *seg_size, *seg_count;
    uint32_t n_segs, max_segs;
    int tsize;
    int failed;
} bp_writer;

static void store_t(uint8_t *p, int64_t v, int tsize) {
    if (tsize == 4) {
        int32_t x = (int32_t)v;
        memcpy(p, &x, 4);
    } else {
        memcpy(p, &v, 8);
    }
}

static void seg_begin(bp_writer *w) {
    memset(w->blk, 0, w->block_size);
    w->data_off = 8;
    w->meta_off = w->block_size;
    w->seg_rows = 0;
}

static void seg_flush(bp_writer *w) {
    const uint64_t meta_at = (w->data_off + 7) / 8 * 8;
    const uint64_t meta_size = w->block_size - w->meta_off;
    const uint64_t total = meta_at + meta_size;
    memmove(w->blk + meta_at, w->blk + w->meta_off, meta_size);
    const uint64_t header = meta_at + meta_size;
    memcpy(w->blk, &header, 8);
    /* segments start 8-aligned in the concatenated image (each is a block of its own in the
     * reference, so every field stays aligned to its width) */
    w->out_used = (w->out_used + 7) / 8 * 8;
    if (w->n_segs >= w->max_segs || w->out_used + total > w->out_cap) {
        w->failed = 1;
        return;
    }
    memcpy(w->out + w->out_used, w->blk, total);
    w->seg_off[w->n_segs] = w->out_used;
    w->seg_size[w->n_segs] = total;
    w->seg_count[w->n_segs] = w->seg_rows;
    w->n_segs++;
    w->out_used += total;
}

static int can_store(const bp_writer *w, uint64_t data_bytes, uint64_t meta_bytes) {
    const uint64_t req_data = (data_bytes + 7) / 8 * 8;
    const uint64_t req_meta = w->block_size - (w->meta_off - w->data_off) + meta_bytes;
    return req_data + req_meta <= w->block_size - 8;
}

static void reserve(bp_writer *w, uint64_t data_bytes) {
    if (!can_store(w, data_bytes, 4)) {
        seg_flush(w);
        seg_begin(w);
    }
}

static void write_meta(bp_writer *w, int mode) {
    const uint32_t enc = (uint32_t)(w->data_off & 0x00ffffff) | ((uint32_t)mode << 24);
    w->meta_off -= 4;
    memcpy(w->blk + w->meta_off, &enc, 4);
}

static void put_t(bp_writer *w, int64_t v) {
    store_t(w->blk + w->data_off, v, w->tsize);
    w->data_off += (uint64_t)w->tsize;
}

typedef struct {
    int64_t buf[BP_GROUP + 1]; /* buf[0] = the "previous value" slot (stays 0) */
    int64_t delta[BP_GROUP];
    int valid[BP_GROUP];
    uint64_t idx;
    int64_t minimum, maximum, min_delta, max_delta, min_max_diff, min_max_delta_diff, delta_offset;
    int all_valid, all_invalid, can_delta, can_for;
    int mode;
} bp_state;

static void st_reset(bp_state *s, int tsize) {
    s->minimum = tmax(tsize);
    s->maximum = tmin(tsize);
    s->min_delta = tmax(tsize);
    s->max_delta = tmin(tsize);
    s->delta_offset = 0;
    s->all_valid = 1;
    s->all_invalid = 1;
    s->can_delta = 0;
    s->can_for = 0;
    s->idx = 0;
    s->min_max_diff = 0;
    s->min_max_delta_diff = 0;
}

/* Flush one group (BitpackingState::Flush); 0 = the column cannot be bitpacked */
static int st_flush(bp_state *s, bp_writer *w) {
    const int ts = w->tsize;
    int64_t *cb = s->buf + 1;
    if (s->idx == 0) return 1;
    if ((s->all_invalid || s->maximum == s->minimum) && (s->mode == BP_AUTO || s->mode == BP_CONSTANT)) {
        reserve(w, (uint64_t)ts);
        write_meta(w, BP_CONSTANT);
        put_t(w, s->maximum);
        w->seg_rows += s->idx;
        return 1;
    }
    s->can_for = sub_ok(s->maximum, s->minimum, ts, &s->min_max_diff);
    /* CalculateDeltaStats (T signed: the T_S maximum check never fires) */
    if (s->idx >= 2 && s->all_valid) {
        int64_t bogus;
        const int can_all = sub_ok(s->minimum, s->maximum, ts, &bogus) && sub_ok(s->maximum, s->minimum, ts, &bogus);
        int ok = 1;
        for (uint64_t i = 0; i < s->idx; i++) {
            if (can_all) {
                s->delta[i] = ts == 4 ? (int64_t)(int32_t)((uint32_t)cb[i] - (uint32_t)cb[(int64_t)i - 1])
                                      : (int64_t)((uint64_t)cb[i] - (uint64_t)cb[(int64_t)i - 1]);
            } else if (!sub_ok(cb[i], cb[(int64_t)i - 1], ts, &s->delta[i])) {
                ok = 0;
                break;
            }
        }
        if (ok) {
            s->can_delta = 1;
            for (uint64_t i = 1; i < s->idx; i++) {
                if (s->delta[i] > s->max_delta) s->max_delta = s->delta[i];
                if (s->delta[i] < s->min_delta) s->min_delta = s->delta[i];
            }
            s->delta[0] = s->min_delta;
            s->can_delta = s->can_delta && sub_ok(s->max_delta, s->min_delta, ts, &s->min_max_delta_diff);
            s->can_delta = s->can_delta && sub_ok(cb[0], s->min_delta, ts, &s->delta_offset);
        }
    }
    if (s->can_delta) {
        if (s->max_delta == s->min_delta && s->mode != BP_FOR && s->mode != BP_DELTA_FOR) {
            reserve(w, 2 * (uint64_t)ts);
            write_meta(w, BP_CONSTANT_DELTA);
            put_t(w, cb[0]);
            put_t(w, s->max_delta);
            w->seg_rows += s->idx;
            return 1;
        }
        const int dw = width_unsigned((uint64_t)s->min_max_delta_diff & umask(ts), ts);
        const int rw = width_signed_nonneg(s->min_max_diff, ts);
        if (dw < rw && s->mode != BP_FOR) {
            uint64_t u[BP_GROUP];
            for (uint64_t i = 0; i < s->idx; i++) u[i] = ((uint64_t)s->delta[i] - (uint64_t)s->min_delta) & umask(ts);
            const uint64_t bp = (s->idx + BP_ALG - 1) / BP_ALG * BP_ALG * (uint64_t)dw / 8;
            reserve(w, bp + 3 * (uint64_t)ts);
            write_meta(w, BP_DELTA_FOR);
            put_t(w, s->min_delta);
            put_t(w, dw);
            put_t(w, s->delta_offset);
            pack_values(w->blk + w->data_off, u, s->idx, dw);
            w->data_off += bp;
            w->seg_rows += s->idx;
            return 1;
        }
    }
    if (s->can_for) {
        const int fw = width_unsigned((uint64_t)s->min_max_diff, ts);
        uint64_t u[BP_GROUP];
        for (uint64_t i = 0; i < s->idx; i++) u[i] = ((uint64_t)cb[i] - (uint64_t)s->minimum) & umask(ts);
        const uint64_t bp = (s->idx + BP_ALG - 1) / BP_ALG * BP_ALG * (uint64_t)fw / 8;
        reserve(w, bp + 2 * (uint64_t)ts);
        write_meta(w, BP_FOR);
        put_t(w, s->minimum);
        put_t(w, fw);
        pack_values(w->blk + w->data_off, u, s->idx, fw);
        w->data_off += bp;
        w->seg_rows += s->idx;
        return 1;
    }
    return 0;
}

int oracle_bp_compress(const void *values, int tsize, const uint8_t *valid, uint64_t n, int mode, uint64_t block_size,
                       uint8_t *out, uint64_t out_cap, uint64_t *seg_off, uint64_t *seg_size, uint64_t *seg_count,
                       uint32_t max_segs, uint32_t *n_segs) {
    if ((tsize != 4 && tsize != 8) || !values || !out || !n_segs) return -1;
    bp_writer w;
    memset(&w, 0, sizeof(w));
    w.out = out;
    w.out_cap = out_cap;
    w.block_size = block_size;
    w.blk = (uint8_t *)malloc(block_size);
    w.seg_off = seg_off;
    w.seg_size = seg_size;
    w.seg_count = seg_count;
    w.max_segs = max_segs;
    w.tsize = tsize;
    bp_state *s = (bp_state *)calloc(1, sizeof(bp_state));
    if (!w.blk || !s) {
        free(w.blk);
        free(s);
        return -1;
    }
    s->mode = mode;
    st_reset(s, tsize);
    seg_begin(&w);
    int ok = 1;
    for (uint64_t r = 0; r < n && ok; r++) {
        const int v_ok = valid ? valid[r] != 0 : 1;
        const int64_t v = tsize == 4 ? (int64_t)((const int32_t *)values)[r] : ((const int64_t *)values)[r];
        s->valid[s->idx] = v_ok;
        s->all_valid = s->all_valid && v_ok;
        s->all_invalid = s->all_invalid && !v_ok;
        if (v_ok) {
            s->buf[1 + s->idx] = v;
            if (v < s->minimum) s->minimum = v;
            if (v > s->maximum) s->maximum = v;
        }
        s->idx++;
        if (s->idx == BP_GROUP) {
            ok = st_flush(s, &w);
            st_reset(s, tsize);
        }
    }
    if (ok) ok = st_flush(s, &w);
    if (ok) seg_flush(&w);
    free(w.blk);
    free(s);
    if (!ok) return 1;    /* not bitpackable (the reference picks another compression) */
    if (w.failed) return -2;
    *n_segs = w.n_segs;
    return 0;
}

/* ---------------------------------------------------------------- CPU decode */

static int64_t load_t(const uint8_t *p, int tsize) {
    if (tsize == 4) {
        int32_t x;
        memcpy(&x, p, 4);
        return x;
    }
    int64_t x;
    memcpy(&x, p, 8);
    return x;
}

/* Sequential scan of the segments (LoadNextGroup + BitpackingScanPartial). */
int oracle_bp_decode(const uint8_t *bytes, const uint64_t *seg_off, const uint64_t *seg_count, uint32_t n_segs,
                     int tsize, void *out_values) {
    uint64_t row = 0;
    for (uint32_t sg = 0; sg < n_segs; sg++) {
        const uint8_t *base = bytes + seg_off[sg];
        uint64_t meta_end;
        memcpy(&meta_end, base, 8);
        const uint8_t *meta = base + meta_end - 4;
        for (uint64_t done = 0; done < seg_count[sg]; done += BP_GROUP, meta -= 4) {
            uint32_t enc;
            memcpy(&enc, meta, 4);
            const int mode = (int)(enc >> 24);
            const uint8_t *g = base + (enc & 0x00ffffff);
            const uint64_t cnt = seg_count[sg] - done < BP_GROUP ? seg_count[sg] - done : BP_GROUP;
            int64_t for_v = 0, c = 0, doff = 0;
            int w = 0;
            const uint8_t *packed = g;
            if (mode == BP_CONSTANT) {
                c = load_t(g, tsize);
            } else if (mode == BP_CONSTANT_DELTA) {
                for_v = load_t(g, tsize);
                c = load_t(g + tsize, tsize);
            } else if (mode == BP_FOR || mode == BP_DELTA_FOR) {
                for_v = load_t(g, tsize);
                w = (int)(uint8_t)load_t(g + tsize, tsize);
                packed = g + 2 * tsize;
                if (mode == BP_DELTA_FOR) {
                    doff = load_t(packed, tsize);
                    packed += tsize;
                }
            } else {
                return -1;
            }
            uint64_t run = (uint64_t)doff;
            for (uint64_t i = 0; i < cnt; i++) {
                uint64_t v;
                if (mode == BP_CONSTANT) v = (uint64_t)c;
                else if (mode == BP_CONSTANT_DELTA) v = (uint64_t)c * i + (uint64_t)for_v;
                else if (mode == BP_FOR) v = unpack_value(packed, i, w) + (uint64_t)for_v;
                else {
                    run += unpack_value(packed, i, w) + (uint64_t)for_v;
                    v = run;
                }
                if (tsize == 4) ((int32_t *)out_values)[row + i] = (int32_t)(uint32_t)v;
                else ((int64_t *)out_values)[row + i] = (int64_t)v;
            }
            row += cnt;
        }
    }
    return 0;
}

/* mode of every group, in row order (tests check the reference's mode choice) */
int oracle_bp_group_modes(const uint8_t *bytes, const uint64_t *seg_off, const uint64_t *seg_count, uint32_t n_segs,
                          uint8_t *modes, uint64_t cap) {
    uint64_t k = 0;
    for (uint32_t sg = 0; sg < n_segs; sg++) {
        const uint8_t *base = bytes + seg_off[sg];
        uint64_t meta_end;
        memcpy(&meta_end, base, 8);
        const uint8_t *meta = base + meta_end - 4;
        for (uint64_t done = 0; done < seg_count[sg]; done += BP_GROUP, meta -= 4) {
            uint32_t enc;
            memcpy(&enc, meta, 4);
            if (k < cap) modes[k] = (uint8_t)(enc >> 24);
            k++;
        }
    }
    return (int)k;
}
