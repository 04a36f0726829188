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
 * Values are any of the integral physical types the reference bit-packs: INT8 … INT64 and
 * UINT8 … UINT64 (TINYINT … BIGINT, UTINYINT … UBIGINT, DATE, DECIMAL ≤ 18).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "cpu_ref.h"

#define BP_GROUP 2048
#define BP_ALG 32

/* BitpackingMode (src/include/duckdb/storage/compression/bitpacking.hpp:15) */
enum { BP_INVALID = 0, BP_AUTO = 1, BP_CONSTANT = 2, BP_CONSTANT_DELTA = 3, BP_DELTA_FOR = 4, BP_FOR = 5 };

/* ---------------------------------------------------------------- the value type T */

/* T is one of DuckDB's bitpacked physical types: 1, 2, 4 or 8 bytes, signed or unsigned
 * (bitpacking.cpp:951-977 GetBitpackingFunction: INT8..INT64, UINT8..UINT64). The caller's
 * ttype = byte size | 0x100 when unsigned. Values travel as T's bits, zero-extended to 64;
 * T_S is the signed type of T's size (the deltas, MakeSigned<T>). */
typedef struct {
    int tsize, bits, sgn;
    uint64_t mask;
} bp_t;

static int bp_ttype_ok(int ttype) {
    const int sz = ttype & 0xff;
    return (ttype & ~0x1ff) == 0 && (sz == 1 || sz == 2 || sz == 4 || sz == 8);
}
static bp_t bp_type(int ttype) {
    bp_t t;
    t.tsize = ttype & 0xff;
    t.bits = 8 * t.tsize;
    t.sgn = !(ttype & 0x100);
    t.mask = t.bits == 64 ? ~0ull : ((1ull << t.bits) - 1);
    return t;
}
/* the signed value of T_S bits x */
static int64_t sx(uint64_t x, int bits) { return bits == 64 ? (int64_t)x : (int64_t)(x << (64 - bits)) >> (64 - bits); }
/* a < b in T's order */
static int t_lt(bp_t t, uint64_t a, uint64_t b) { return t.sgn ? sx(a, t.bits) < sx(b, t.bits) : a < b; }
static uint64_t t_max(bp_t t) { return t.sgn ? t.mask >> 1 : t.mask; }
static uint64_t t_min(bp_t t) { return t.sgn ? (t.mask >> 1) + 1 : 0; }
/* TrySubtractOperator in T_S: a - b of T_S bits, 0 when it overflows T_S */
static int sub_s(bp_t t, uint64_t a, uint64_t b, uint64_t *out) {
    const int64_t x = sx(a, t.bits), y = sx(b, t.bits);
    int64_t r;
    if (__builtin_sub_overflow(x, y, &r)) return 0;
    if (t.bits < 64 && (r < -(1ll << (t.bits - 1)) || r > (1ll << (t.bits - 1)) - 1)) return 0;
    *out = (uint64_t)r & t.mask;
    return 1;
}
/* TrySubtractOperator in T */
static int sub_t(bp_t t, uint64_t a, uint64_t b, uint64_t *out) {
    if (t.sgn) return sub_s(t, a, b, out);
    if (a < b) return 0;
    *out = a - b;
    return 1;
}

/* ---------------------------------------------------------------- width helpers */

/* GetEffectiveWidth (bitpacking.hpp:202-210) */
static int eff_width(int w, bp_t t) { return (w + t.tsize > t.bits) ? t.bits : w; }
/* MinimumBitWidth<T, false>(v) (bitpacking.hpp:139-188, is_signed = false) */
static int width_u(bp_t t, uint64_t v) {
    v &= t.mask;
    int w = 0;
    while (v) {
        w++;
        v >>= 1;
    }
    return w == 0 ? 0 : eff_width(w, t);
}
/* MinimumBitWidth<T>(v) with T's own signedness: signed T takes |v| plus a sign bit, and the
 * full width for T's minimum */
static int width_t(bp_t t, uint64_t v) {
    if (!t.sgn) return width_u(t, v);
    const int64_t x = sx(v & t.mask, t.bits);
    if ((v & t.mask) == t_min(t)) return t.bits;
    uint64_t a = (uint64_t)(x < 0 ? -x : x);
    if (a == 0) return 0;
    int w = 1;
    while (a) {
        w++;
        a >>= 1;
    }
    return eff_width(w, t);
}

/* ---------------------------------------------------------------- packing */

/* 32-bit little-endian word i of a packed run (any byte alignment: narrow T's headers leave
 * the run unaligned) */
static uint32_t get_word(const uint8_t *p, uint64_t i) {
    uint32_t x;
    memcpy(&x, p + 4 * i, 4);
    return x;
}
static void or_word(uint8_t *p, uint64_t i, uint32_t v) {
    uint32_t x;
    memcpy(&x, p + 4 * i, 4);
    x |= v;
    memcpy(p + 4 * i, &x, 4);
}

static void pack_values(uint8_t *dst, const uint64_t *v, uint64_t count, int w) {
    const uint64_t n = (count + BP_ALG - 1) / BP_ALG * BP_ALG;
    const uint64_t bytes = n * (uint64_t)w / 8;
    memset(dst, 0, bytes);
    if (w == 0) return;
    const uint64_t mask = w == 64 ? ~0ull : ((1ull << w) - 1);
    for (uint64_t i = 0; i < n; i++) {
        uint64_t x = (i < count ? v[i] : 0) & mask;
        uint64_t bit = i * (uint64_t)w;
        int left = w;
        while (left > 0) {
            const uint64_t wi = bit >> 5;
            const int off = (int)(bit & 31);
            const int take = (32 - off) < left ? (32 - off) : left;
            or_word(dst, wi, (uint32_t)((x & ((1ull << take) - 1)) << off));
            x >>= take;
            bit += (uint64_t)take;
            left -= take;
        }
    }
}

static uint64_t unpack_value(const uint8_t *src, uint64_t i, int w) {
    if (w == 0) return 0;
    uint64_t bit = i * (uint64_t)w, x = 0;
    int got = 0;
    while (got < w) {
        const uint64_t wi = bit >> 5;
        const int off = (int)(bit & 31);
        const int take = (32 - off) < (w - got) ? (32 - off) : (w - got);
        const uint64_t part = ((uint64_t)get_word(src, wi) >> off) & ((1ull << take) - 1);
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
    bp_t t;
    int failed;
} bp_writer;

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
     * reference) */
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

/* WriteData<T>: T's bytes, unaligned (little-endian: the low tsize bytes of the bits) */
static void put_t(bp_writer *w, uint64_t v) {
    memcpy(w->blk + w->data_off, &v, (size_t)w->t.tsize);
    w->data_off += (uint64_t)w->t.tsize;
}

typedef struct {
    uint64_t buf[BP_GROUP + 1]; /* T bits; buf[0] = the "previous value" slot (stays 0) */
    uint64_t delta[BP_GROUP];   /* T_S bits */
    int valid[BP_GROUP];
    uint64_t idx;
    uint64_t minimum, maximum, min_max_diff;                          /* T */
    uint64_t min_delta, max_delta, min_max_delta_diff, delta_offset;  /* T_S */
    int all_valid, all_invalid, can_delta, can_for;
    int mode;
} bp_state;

static void st_reset(bp_state *s, bp_t t) {
    s->minimum = t_max(t);
    s->maximum = t_min(t);
    s->min_delta = t.mask >> 1;    /* T_S maximum */
    s->max_delta = (t.mask >> 1) + 1;  /* T_S minimum */
    s->delta_offset = 0;
    s->all_valid = 1;
    s->all_invalid = 1;
    s->can_delta = 0;
    s->can_for = 0;
    s->idx = 0;
    s->min_max_diff = 0;
    s->min_max_delta_diff = 0;
}

/* Flush one group (BitpackingState::Flush, bitpacking.cpp:231-296); 0 = the column cannot be
 * bitpacked */
static int st_flush(bp_state *s, bp_writer *w) {
    const bp_t t = w->t;
    const uint64_t ts = (uint64_t)t.tsize;
    uint64_t *cb = s->buf + 1;
    if (s->idx == 0) return 1;
    if ((s->all_invalid || s->maximum == s->minimum) && (s->mode == BP_AUTO || s->mode == BP_CONSTANT)) {
        reserve(w, ts);
        write_meta(w, BP_CONSTANT);
        put_t(w, s->maximum);
        w->seg_rows += s->idx;
        return 1;
    }
    s->can_for = sub_t(t, s->maximum, s->minimum, &s->min_max_diff); /* CalculateFORStats */
    /* CalculateDeltaStats (:155-214): unsigned T above T_S's maximum never delta-encodes; a
     * NULL or a single value neither. Every delta is a T_S subtraction (for signed T whose
     * max - min fits T_S the reference skips the overflow check: none can occur). */
    const int above_ts = !t.sgn && s->maximum > (t.mask >> 1);
    if (!above_ts && s->idx >= 2 && s->all_valid) {
        int ok = 1;
        for (uint64_t i = 0; i < s->idx; i++) {
            if (!sub_s(t, cb[i], cb[(int64_t)i - 1], &s->delta[i])) {
                ok = 0;
                break;
            }
        }
        if (ok) {
            s->can_delta = 1;
            for (uint64_t i = 1; i < s->idx; i++) {
                if (sx(s->delta[i], t.bits) > sx(s->max_delta, t.bits)) s->max_delta = s->delta[i];
                if (sx(s->delta[i], t.bits) < sx(s->min_delta, t.bits)) s->min_delta = s->delta[i];
            }
            s->delta[0] = s->min_delta;
            s->can_delta = s->can_delta && sub_s(t, s->max_delta, s->min_delta, &s->min_max_delta_diff);
            s->can_delta = s->can_delta && sub_s(t, cb[0], s->min_delta, &s->delta_offset);
        }
    }
    if (s->can_delta) {
        if (s->max_delta == s->min_delta && s->mode != BP_FOR && s->mode != BP_DELTA_FOR) {
            reserve(w, 2 * ts);
            write_meta(w, BP_CONSTANT_DELTA);
            put_t(w, cb[0]);
            put_t(w, s->max_delta);
            w->seg_rows += s->idx;
            return 1;
        }
        const int dw = width_u(t, s->min_max_delta_diff);
        const int rw = width_t(t, s->min_max_diff);
        if (dw < rw && s->mode != BP_FOR) {
            uint64_t u[BP_GROUP];
            for (uint64_t i = 0; i < s->idx; i++) u[i] = (s->delta[i] - s->min_delta) & t.mask;
            const uint64_t bp = (s->idx + BP_ALG - 1) / BP_ALG * BP_ALG * (uint64_t)dw / 8;
            reserve(w, bp + 3 * ts);
            write_meta(w, BP_DELTA_FOR);
            put_t(w, s->min_delta);
            put_t(w, (uint64_t)dw);
            put_t(w, s->delta_offset);
            pack_values(w->blk + w->data_off, u, s->idx, dw);
            w->data_off += bp;
            w->seg_rows += s->idx;
            return 1;
        }
    }
    if (s->can_for) {
        const int fw = width_u(t, s->min_max_diff);
        uint64_t u[BP_GROUP];
        for (uint64_t i = 0; i < s->idx; i++) u[i] = (cb[i] - s->minimum) & t.mask;
        const uint64_t bp = (s->idx + BP_ALG - 1) / BP_ALG * BP_ALG * (uint64_t)fw / 8;
        reserve(w, bp + 2 * ts);
        write_meta(w, BP_FOR);
        put_t(w, s->minimum);
        put_t(w, (uint64_t)fw);
        pack_values(w->blk + w->data_off, u, s->idx, fw);
        w->data_off += bp;
        w->seg_rows += s->idx;
        return 1;
    }
    return 0;
}

int oracle_bp_compress(const void *values, int ttype, const uint8_t *valid, uint64_t n, int mode, uint64_t block_size,
                       uint8_t *out, uint64_t out_cap, uint64_t *seg_off, uint64_t *seg_size, uint64_t *seg_count,
                       uint32_t max_segs, uint32_t *n_segs) {
    if (!bp_ttype_ok(ttype) || !values || !out || !n_segs) return -1;
    const bp_t t = bp_type(ttype);
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
    w.t = t;
    bp_state *s = (bp_state *)calloc(1, sizeof(bp_state));
    if (!w.blk || !s) {
        free(w.blk);
        free(s);
        return -1;
    }
    s->mode = mode;
    st_reset(s, t);
    seg_begin(&w);
    int ok = 1;
    for (uint64_t r = 0; r < n && ok; r++) { /* BitpackingState::Update (:298-318) */
        const int v_ok = valid ? valid[r] != 0 : 1;
        uint64_t v = 0;
        memcpy(&v, (const uint8_t *)values + r * (uint64_t)t.tsize, (size_t)t.tsize);
        s->valid[s->idx] = v_ok;
        s->all_valid = s->all_valid && v_ok;
        s->all_invalid = s->all_invalid && !v_ok;
        if (v_ok) {
            s->buf[1 + s->idx] = v;
            if (t_lt(t, v, s->minimum)) s->minimum = v;
            if (t_lt(t, s->maximum, v)) s->maximum = v;
        }
        s->idx++;
        if (s->idx == BP_GROUP) {
            ok = st_flush(s, &w);
            st_reset(s, t);
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

static uint64_t load_t(const uint8_t *p, bp_t t) {
    uint64_t x = 0;
    memcpy(&x, p, (size_t)t.tsize);
    return x;
}

/* Sequential scan of the segments (LoadNextGroup + BitpackingScanPartial, :585-868): every
 * value in T's arithmetic (mod 2^bits), written as T. */
int oracle_bp_decode(const uint8_t *bytes, const uint64_t *seg_off, const uint64_t *seg_count, uint32_t n_segs,
                     int ttype, void *out_values) {
    if (!bp_ttype_ok(ttype)) return -1;
    const bp_t t = bp_type(ttype);
    const uint64_t ts = (uint64_t)t.tsize;
    uint8_t *outb = (uint8_t *)out_values;
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
            uint64_t for_v = 0, c = 0, doff = 0;
            int w = 0;
            const uint8_t *packed = g;
            if (mode == BP_CONSTANT) {
                c = load_t(g, t);
            } else if (mode == BP_CONSTANT_DELTA) {
                for_v = load_t(g, t);
                c = load_t(g + ts, t);
            } else if (mode == BP_FOR || mode == BP_DELTA_FOR) {
                for_v = load_t(g, t);
                w = (int)(uint8_t)load_t(g + ts, t); /* the width is stored as a T */
                packed = g + 2 * ts;
                if (mode == BP_DELTA_FOR) {
                    doff = load_t(packed, t);
                    packed += ts;
                }
                if (w > t.bits) return -1;
            } else {
                return -1;
            }
            uint64_t run = doff;
            for (uint64_t i = 0; i < cnt; i++) {
                uint64_t v;
                if (mode == BP_CONSTANT) v = c;
                else if (mode == BP_CONSTANT_DELTA) v = c * i + for_v;
                else if (mode == BP_FOR) v = unpack_value(packed, i, w) + for_v;
                else {
                    run += unpack_value(packed, i, w) + for_v;
                    v = run;
                }
                v &= t.mask;
                memcpy(outb + (row + i) * ts, &v, (size_t)ts);
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
