/*
 * ORACLE — test infrastructure only. Nothing on the product path links, loads or calls
 * this file; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg do.
 *
 * A plain-C restatement of the reference CPU scan path (DuckDB v1.1.2, mounted at
 * /root/reference) that the HIP path must reproduce bit-exactly:
 *
 *   RowGroup::TemplatedScan<TABLE_SCAN_REGULAR>   src/storage/table/row_group.cpp:447-604
 *     - 2,048-row vectors, 122,880-row row groups   common/vector_size.hpp:16-20, storage_info.hpp:20
 *     - MVCC visibility sel                           row_group.cpp:469-475, chunk_info.cpp:11-19,123-161
 *     - per-column filter loop over one shared sel    row_group.cpp:537-550
 *     - early skip when nothing survives              row_group.cpp:551-568
 *     - row-id synthesis start+current_row+sel[i]     row_group.cpp:573-580
 *   ColumnData::Select → ColumnSegment::FilterSelection  column_data.cpp:296-303,
 *                                                    column_segment.cpp:378-522
 *     - CONJUNCTION_OR: union with O(k^2) dedupe, child order (NOT sorted)   :381-409
 *     - CONJUNCTION_AND: successive narrowing                                 :410-416
 *     - CONSTANT_COMPARISON: TemplatedFilterSelection branchless compaction   :261-349
 *     - IS_NULL / IS_NOT_NULL                                                 :351-376, 506-520
 *   UpdateSegment::FetchUpdates / UpdatesForTransaction (visible value of an updated row)
 *                                                    update_segment.cpp:101-174, update_info.hpp:44-55
 *   ExpressionExecutor::Select for a residual cross-column AND/OR tree (PhysicalFilter above
 *   the scan, since OR filters are not pushed in this snapshot: filter_combiner.cpp:624)
 *                                                    execute_conjunction.cpp:56-142,
 *                                                    physical_filter.cpp:42-53
 *   ColumnData::FetchRow (index_scan probe)           row_group_collection.cpp:264-288
 *
 * Plus a CPU bitmap evaluator (64-bit words, AND/OR/ANDNOT, tzcnt decode) used as the
 * algorithmic sibling of the GPU kernels.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "cpu_ref.h"

#define VEC 2048            /* STANDARD_VECTOR_SIZE */
#define ROW_GROUP 122880    /* STANDARD_ROW_GROUPS_SIZE */

static const uint64_t NOT_DELETED_ID = UINT64_MAX - 1; /* src/common/constants.cpp:16 */

/* ------------------------------------------------------------------ helpers */

static inline int row_valid(const ocol *c, uint64_t row) {
    if (!c->validity) return 1;
    return (int)((c->validity[row >> 6] >> (row & 63)) & 1ULL);
}

/* TransactionVersionOperator::UseInsertedVersion (chunk_info.cpp:11-14) */
static inline int use_inserted(uint64_t start_time, uint64_t tid, uint64_t id) {
    return id < start_time || id == tid;
}

/* Floating-point comparisons with DuckDB's semantics (src/common/vector_operations/
 * comparison_operators.cpp:17-88): NaN equals NaN and is greater than every other value; other
 * values compare as IEEE (so -0.0 == +0.0). LessThan(a, b) = GreaterThan(b, a). */
static inline int fp_isnan(double x) { return x != x; }
static inline int fp_eq(double a, double b) { return (fp_isnan(a) && fp_isnan(b)) || a == b; }
static inline int fp_gt(double a, double b) {
    if (fp_isnan(b)) return 0;
    if (fp_isnan(a)) return 1;
    return a > b;
}
static inline int fp_ge(double a, double b) {
    if (fp_isnan(b)) return fp_isnan(a);
    if (fp_isnan(a)) return 1;
    return a >= b;
}
static inline double fp_value(int type, int64_t bits) {
    if (type == OTYPE_FLOAT) {
        uint32_t u = (uint32_t)bits;
        float f;
        memcpy(&f, &u, 4);
        return (double)f;
    }
    double d;
    memcpy(&d, &bits, 8);
    return d;
}
static inline int cmp_fp(int cmp, double v, double c) {
    switch (cmp) {
    case 0: return fp_eq(v, c);
    case 1: return !fp_eq(v, c);
    case 2: return fp_gt(c, v);
    case 3: return fp_ge(c, v);
    case 4: return fp_gt(v, c);
    default: return fp_ge(v, c);
    }
}

static inline int cmp_op(int cmp, int64_t v, int64_t c) {
    switch (cmp) {
    case OCMP_EQ: return v == c;
    case OCMP_NE: return v != c;
    case OCMP_LT: return v < c;
    case OCMP_LE: return v <= c;
    case OCMP_GT: return v > c;
    case OCMP_GE: return v >= c;
    default: return 0;
    }
}

/* string_t comparisons (src/include/duckdb/common/types/string_type.hpp:143-206, Equals /
 * GreaterThan): the bytes compared as unsigned (the byte-swapped prefix, then memcmp), a string
 * that is a prefix of the other is the smaller one */
static inline int str_order(const ostring *a, const ostring *b) {
    const uint64_t m = a->size < b->size ? a->size : b->size;
    const int r = m ? memcmp(a->data, b->data, m) : 0;
    if (r) return r < 0 ? -1 : 1;
    return a->size < b->size ? -1 : a->size > b->size ? 1 : 0;
}
static inline int cmp_str(int cmp, int64_t v, int64_t c) {
    const int o = str_order((const ostring *)(intptr_t)v, (const ostring *)(intptr_t)c);
    switch (cmp) {
    case OCMP_EQ: return o == 0;
    case OCMP_NE: return o != 0;
    case OCMP_LT: return o < 0;
    case OCMP_LE: return o <= 0;
    case OCMP_GT: return o > 0;
    default: return o >= 0;
    }
}

/* hugeint_t / uhugeint_t comparisons (hugeint.cpp / uhugeint.cpp operators: upper, then lower
 * unsigned) as the compiler's 128-bit integers */
static inline int cmp_huge(int type, int cmp, int64_t v, int64_t c) {
    const ohuge *a = (const ohuge *)(intptr_t)v, *b = (const ohuge *)(intptr_t)c;
    int o;
    if (type == OTYPE_INT128) {
        const __int128 x = (__int128)(((unsigned __int128)a->upper << 64) | a->lower);
        const __int128 y = (__int128)(((unsigned __int128)b->upper << 64) | b->lower);
        o = x < y ? -1 : x > y;
    } else {
        const unsigned __int128 x = ((unsigned __int128)a->upper << 64) | a->lower;
        const unsigned __int128 y = ((unsigned __int128)b->upper << 64) | b->lower;
        o = x < y ? -1 : x > y;
    }
    switch (cmp) {
    case OCMP_EQ: return o == 0;
    case OCMP_NE: return o != 0;
    case OCMP_LT: return o < 0;
    case OCMP_LE: return o <= 0;
    case OCMP_GT: return o > 0;
    default: return o >= 0;
    }
}
static inline int is_addr_type(int type) {
    return type == OTYPE_VARCHAR || type == OTYPE_INT128 || type == OTYPE_UINT128;
}

/* a comparison of values of column type `type` (FP: bit patterns; VARCHAR / INT128 / UINT128:
 * ostring / ohuge addresses) */
static inline int cmp_typed(int type, int cmp, int64_t v, int64_t c) {
    if (type == OTYPE_VARCHAR) return cmp_str(cmp, v, c);
    if (type == OTYPE_INT128 || type == OTYPE_UINT128) return cmp_huge(type, cmp, v, c);
    if (type == OTYPE_UINT64) {
        const uint64_t a = (uint64_t)v, b = (uint64_t)c;
        switch (cmp) {
        case OCMP_EQ: return a == b;
        case OCMP_NE: return a != b;
        case OCMP_LT: return a < b;
        case OCMP_LE: return a <= b;
        case OCMP_GT: return a > b;
        default: return a >= b;
        }
    }
    if (type == OTYPE_FLOAT || type == OTYPE_DOUBLE) return cmp_fp(cmp, fp_value(type, v), fp_value(type, c));
    return cmp_op(cmp, v, c);
}

/* the stored value of row r as int64 (FP: its bit pattern, FLOAT zero-extended) */
static inline int64_t col_value(const ocol *c, uint64_t r) {
    switch (c->type) {
    case OTYPE_INT32: return (int64_t)((const int32_t *)c->data)[r];
    case OTYPE_VARCHAR: return (int64_t)(intptr_t)((const ostring *)c->data + r);
    case OTYPE_INT128:
    case OTYPE_UINT128: return (int64_t)(intptr_t)((const ohuge *)c->data + r);
    case OTYPE_FLOAT: {
        uint32_t u;
        memcpy(&u, (const float *)c->data + r, 4);
        return (int64_t)u;
    }
    default: return ((const int64_t *)c->data)[r];  /* INT64, DOUBLE bits */
    }
}

/* end (exclusive) of the prefix-order subtree rooted at node i */
static int subtree_end(const ofilter *nodes, int i) {
    int n = nodes[i].n_children, j = i + 1;
    for (int k = 0; k < n; k++) j = subtree_end(nodes, j);
    return j;
}

/* One vector of a column as the scan sees it: values (updates merged for this txn) and
 * validity. Mirrors ColumnData::ScanVector + FetchUpdates (column_data.cpp:229-235). Without
 * updates the vector references the column data in place (an uncompressed in-memory
 * segment scan is zero-copy) and keeps its physical type. */
typedef struct {
    int type;              /* OTYPE_* of the column */
    int wide;              /* data is int64[] of values / FP bit patterns (the merged copy) */
    const void *data;      /* first value of the vector */
    const uint8_t *valid;  /* NULL = all valid */
    int64_t vals[VEC];     /* merged copy when the vector has updates (type becomes INT64) */
    uint8_t valid_buf[VEC];
} vecbuf;

static void load_vector(const ocol *c, uint64_t first_row, uint64_t count, const omvcc *tx, vecbuf *out) {
    int has_upd = 0;
    uint64_t st = tx ? tx->start_time : UINT64_MAX - 2, tid = tx ? tx->transaction_id : UINT64_MAX - 2;
    for (uint64_t u = 0; u < c->n_updates; u++) {
        int64_t r = c->upd_rows[u];
        if (r >= (int64_t)first_row && r < (int64_t)(first_row + count) && use_inserted(st, tid, c->upd_version[u])) {
            has_upd = 1;
            break;
        }
    }
    if (c->validity) {
        for (uint64_t i = 0; i < count; i++) out->valid_buf[i] = (uint8_t)row_valid(c, first_row + i);
        out->valid = out->valid_buf;
    } else {
        out->valid = NULL;
    }
    out->type = c->type;
    if (!has_upd) {
        out->wide = 0;
        out->data = c->type == OTYPE_INT32 || c->type == OTYPE_FLOAT
                        ? (const void *)((const int32_t *)c->data + first_row)
                        : c->type == OTYPE_VARCHAR ? (const void *)((const ostring *)c->data + first_row)
                        : c->type == OTYPE_INT128 || c->type == OTYPE_UINT128
                            ? (const void *)((const ohuge *)c->data + first_row)
                            : (const void *)((const int64_t *)c->data + first_row);
        return;
    }
    for (uint64_t i = 0; i < count; i++) out->vals[i] = col_value(c, first_row + i);
    if (!out->valid) {
        memset(out->valid_buf, 1, count);
        out->valid = out->valid_buf;
    }
    /* update records are chronological; the visible value is the newest visible one
     * (UpdatesForTransaction applies undo images newest→oldest: update_info.hpp:44-55). The
     * validity column keeps its own chain, written by the same UPDATE (InitializeUpdateValidity,
     * update_segment.cpp:588-600) and merged into the mask the same way (UpdateMergeValidity
     * :94-99): a SET NULL record clears the row's bit. */
    for (uint64_t u = 0; u < c->n_updates; u++) {
        int64_t r = c->upd_rows[u];
        if (r < (int64_t)first_row || r >= (int64_t)(first_row + count)) continue;
        if (!use_inserted(st, tid, c->upd_version[u])) continue;
        const int ok = c->upd_valid ? c->upd_valid[u] != 0 : 1;
        out->vals[r - first_row] = ok ? c->upd_values[u] : 0;
        out->valid_buf[r - first_row] = (uint8_t)ok;
    }
    out->wide = 1;
    out->data = out->vals;
}

static inline int64_t vec_value(const vecbuf *v, uint32_t idx) {
    if (v->wide) return ((const int64_t *)v->data)[idx];
    switch (v->type) {
    case OTYPE_INT32: return (int64_t)((const int32_t *)v->data)[idx];
    case OTYPE_FLOAT: return (int64_t)((const uint32_t *)v->data)[idx];
    case OTYPE_VARCHAR: return (int64_t)(intptr_t)((const ostring *)v->data + idx);
    case OTYPE_INT128:
    case OTYPE_UINT128: return (int64_t)(intptr_t)((const ohuge *)v->data + idx);
    default: return ((const int64_t *)v->data)[idx];
    }
}
static inline int vec_valid(const vecbuf *v, uint32_t idx) { return v->valid ? v->valid[idx] : 1; }

/* TemplatedFilterSelection<T, OP, HAS_NULL> (column_segment.cpp:261-276): one loop per
 * (type, comparison, has-null) so the compare is branch-free in the loop body. */
#define TFS_LOOP(T, EXPR)                                                   \
    do {                                                                    \
        const T *vec = (const T *)v->data;                                  \
        const T pred = (T)c;                                                \
        if (v->valid) {                                                     \
            for (uint64_t a = 0; a < approved; a++) {                       \
                uint32_t idx = sel[a];                                      \
                T x = vec[idx];                                             \
                int pass = v->valid[idx] && (EXPR);                         \
                sel[rc] = idx;                                              \
                rc += (uint64_t)pass;                                       \
            }                                                               \
        } else {                                                            \
            for (uint64_t a = 0; a < approved; a++) {                       \
                uint32_t idx = sel[a];                                      \
                T x = vec[idx];                                             \
                int pass = (EXPR);                                          \
                sel[rc] = idx;                                              \
                rc += (uint64_t)pass;                                       \
            }                                                               \
        }                                                                   \
    } while (0)

#define TFS_CMP(T)                                      \
    switch (cmp) {                                      \
    case OCMP_EQ: TFS_LOOP(T, x == pred); break;        \
    case OCMP_NE: TFS_LOOP(T, x != pred); break;        \
    case OCMP_LT: TFS_LOOP(T, x < pred); break;         \
    case OCMP_LE: TFS_LOOP(T, x <= pred); break;        \
    case OCMP_GT: TFS_LOOP(T, x > pred); break;         \
    default: TFS_LOOP(T, x >= pred); break;             \
    }

static uint64_t templated_filter_selection(const vecbuf *v, int cmp, int64_t c, uint32_t *sel, uint64_t approved) {
    uint64_t rc = 0;
    if (is_addr_type(v->type)) {
        /* FilterSelectionSwitch<string_t / hugeint_t / uhugeint_t> (column_segment.cpp:278-349) */
        for (uint64_t a = 0; a < approved; a++) {
            uint32_t idx = sel[a];
            int pass = vec_valid(v, idx) && cmp_typed(v->type, cmp, vec_value(v, idx), c);
            sel[rc] = idx;
            rc += (uint64_t)pass;
        }
        return rc;
    }
    if (v->type == OTYPE_FLOAT || v->type == OTYPE_DOUBLE) {
        /* FilterSelectionSwitch<float / double> with DuckDB's floating-point operators */
        const double pred = fp_value(v->type, c);
        for (uint64_t a = 0; a < approved; a++) {
            uint32_t idx = sel[a];
            int pass = vec_valid(v, idx) && cmp_fp(cmp, fp_value(v->type, vec_value(v, idx)), pred);
            sel[rc] = idx;
            rc += (uint64_t)pass;
        }
        return rc;
    }
    if (v->type == OTYPE_UINT64) {  /* FilterSelectionSwitch<uint64_t>: unsigned compares */
        TFS_CMP(uint64_t)
        return rc;
    }
    if (v->wide) {
        TFS_CMP(int64_t)
        return rc;
    }
    if (v->type == OTYPE_INT32) {
        /* a constant outside the int32 domain: the comparison is decided by its sign */
        if (c > INT32_MAX || c < INT32_MIN) {
            int above = c > INT32_MAX;
            int pass_all = (cmp == OCMP_NE) || (above ? (cmp == OCMP_LT || cmp == OCMP_LE)
                                                      : (cmp == OCMP_GT || cmp == OCMP_GE));
            for (uint64_t a = 0; a < approved; a++) {
                uint32_t idx = sel[a];
                sel[rc] = idx;
                rc += (uint64_t)(pass_all && vec_valid(v, idx));
            }
            return rc;
        }
        TFS_CMP(int32_t)
    } else {
        TFS_CMP(int64_t)
    }
    return rc;
}

/* ColumnSegment::FilterSelection restated over a loaded vector. sel is modified in place,
 * returns the new approved count. */
static uint64_t filter_selection(const ofilter *nodes, int i, const vecbuf *v, uint32_t *sel, uint64_t approved) {
    const ofilter *f = &nodes[i];
    switch (f->kind) {
    case OF_OR: {
        uint32_t result[VEC];
        uint64_t total = 0;
        int child = i + 1;
        for (int k = 0; k < f->n_children; k++) {
            uint32_t tmp[VEC];
            memcpy(tmp, sel, approved * sizeof(uint32_t));
            uint64_t tc = filter_selection(nodes, child, v, tmp, approved);
            for (uint64_t a = 0; a < tc; a++) {
                uint32_t idx = tmp[a];
                int is_new = 1;
                for (uint64_t b = 0; b < total; b++) {
                    if (result[b] == idx) { is_new = 0; break; }
                }
                if (is_new) result[total++] = idx;
            }
            child = subtree_end(nodes, child);
        }
        memcpy(sel, result, total * sizeof(uint32_t));
        return total;
    }
    case OF_AND: {
        int child = i + 1;
        for (int k = 0; k < f->n_children; k++) {
            approved = filter_selection(nodes, child, v, sel, approved);
            child = subtree_end(nodes, child);
        }
        return approved;
    }
    case OF_CONST:
        /* TemplatedFilterSelection: branchless compaction, NULL never passes */
        return templated_filter_selection(v, f->cmp, f->constant, sel, approved);
    case OF_IS_NULL:
    case OF_IS_NOT_NULL: {
        uint64_t rc = 0;
        int want = f->kind == OF_IS_NOT_NULL;
        for (uint64_t a = 0; a < approved; a++) {
            uint32_t idx = sel[a];
            sel[rc] = idx;
            rc += (uint64_t)(vec_valid(v, idx) == want);
        }
        return rc;
    }
    default:
        return 0;
    }
}

/* ExpressionExecutor::Select for a cross-column tree (execute_conjunction.cpp:56-142;
 * comparisons: execute_comparison.cpp, NULL compares false). Writes true rows (sel order)
 * into true_sel and false rows into false_sel, returns true count. */
static uint64_t expr_select(const ofilter *nodes, int i, vecbuf *const *vbufs, const uint32_t *sel, uint64_t count,
                            uint32_t *true_sel, uint32_t *false_sel) {
    const ofilter *f = &nodes[i];
    if (f->kind == OF_AND) {
        uint32_t cur[VEC], tmp_true[VEC], tmp_false[VEC];
        memcpy(cur, sel, count * sizeof(uint32_t));
        uint64_t cur_count = count, false_count = 0;
        int child = i + 1;
        for (int k = 0; k < f->n_children; k++) {
            uint64_t t = expr_select(nodes, child, vbufs, cur, cur_count, tmp_true, tmp_false);
            uint64_t fc = cur_count - t;
            for (uint64_t a = 0; a < fc; a++) false_sel[false_count++] = tmp_false[a];
            memcpy(cur, tmp_true, t * sizeof(uint32_t));
            cur_count = t;
            child = subtree_end(nodes, child);
            if (cur_count == 0) {
                /* remaining children are skipped (execute_conjunction.cpp:88-90) */
                break;
            }
        }
        memcpy(true_sel, cur, cur_count * sizeof(uint32_t));
        return cur_count;
    }
    if (f->kind == OF_OR) {
        uint32_t cur[VEC], tmp_true[VEC], tmp_false[VEC];
        memcpy(cur, sel, count * sizeof(uint32_t));
        uint64_t cur_count = count, result_count = 0;
        int child = i + 1;
        for (int k = 0; k < f->n_children; k++) {
            uint64_t t = expr_select(nodes, child, vbufs, cur, cur_count, tmp_true, tmp_false);
            if (t > 0) {
                for (uint64_t a = 0; a < t; a++) true_sel[result_count++] = tmp_true[a];
                cur_count -= t;
                memcpy(cur, tmp_false, cur_count * sizeof(uint32_t));
            }
            child = subtree_end(nodes, child);
        }
        memcpy(false_sel, cur, cur_count * sizeof(uint32_t));
        return result_count;
    }
    /* leaf: comparison / null test on one column */
    const vecbuf *v = vbufs[f->column];
    uint64_t tc = 0, fc = 0;
    for (uint64_t a = 0; a < count; a++) {
        uint32_t idx = sel[a];
        int pass;
        if (f->kind == OF_CONST) pass = vec_valid(v, idx) && cmp_typed(v->type, f->cmp, vec_value(v, idx), f->constant);
        else if (f->kind == OF_IS_NULL) pass = !vec_valid(v, idx);
        else pass = vec_valid(v, idx);
        if (pass) true_sel[tc++] = idx;
        else false_sel[fc++] = idx;
    }
    return tc;
}

static int cmp_u32(const void *a, const void *b) {
    uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
    return (x > y) - (x < y);
}

/* MVCC visibility for one vector (ChunkVectorInfo::TemplatedGetSelVector) */
static uint64_t visibility_sel(const omvcc *tx, uint64_t first_row, uint64_t count, uint32_t *sel, int *all) {
    *all = 1;
    if (!tx || (!tx->inserted && !tx->deleted)) {
        for (uint64_t i = 0; i < count; i++) sel[i] = (uint32_t)i;
        return count;
    }
    uint64_t c = 0;
    for (uint64_t i = 0; i < count; i++) {
        uint64_t r = first_row + i;
        uint64_t ins = tx->inserted ? tx->inserted[r] : 0;
        uint64_t del = tx->deleted ? tx->deleted[r] : NOT_DELETED_ID;
        if (use_inserted(tx->start_time, tx->transaction_id, ins) &&
            !use_inserted(tx->start_time, tx->transaction_id, del))
            sel[c++] = (uint32_t)i;
    }
    if (c != count) *all = 0;
    return c;
}

/* ----------------------------------------------------------- scan one range */

typedef struct {
    const oscan *s;
    uint64_t vec_begin, vec_end; /* vector indices in [vec_begin, vec_end) */
    int64_t *out;                /* may be NULL: count only */
    uint64_t out_cap;
    uint64_t count;
    uint64_t sum_rowid;
} scan_job;

static void scan_range(scan_job *j) {
    const oscan *s = j->s;
    vecbuf *bufs[OMAX_COLS];
    vecbuf *storage = (vecbuf *)malloc(sizeof(vecbuf) * (size_t)s->n_cols);
    for (int c = 0; c < s->n_cols; c++) bufs[c] = &storage[c];
    uint32_t sel[VEC], tsel[VEC], fsel[VEC];
    j->count = 0;
    j->sum_rowid = 0;
    for (uint64_t vi = j->vec_begin; vi < j->vec_end; vi++) {
        uint64_t first = vi * VEC;
        if (first >= s->n_rows) break;
        uint64_t max_count = s->n_rows - first < VEC ? s->n_rows - first : VEC;
        int all;
        uint64_t approved = visibility_sel(s->tx, first, max_count, sel, &all);
        if (approved == 0) continue;
        /* pushed per-column filters, in (adaptive) permutation order */
        for (int p = 0; p < s->n_pushed && approved; p++) {
            int col = s->pushed[p].column;
            load_vector(&s->cols[col], first, max_count, s->tx, bufs[col]);
            approved = filter_selection(s->nodes, s->pushed[p].root, bufs[col], sel, approved);
        }
        if (approved == 0) continue;
        /* residual cross-column tree (PhysicalFilter above the scan) */
        if (s->residual_root >= 0) {
            for (int c = 0; c < s->n_cols; c++) load_vector(&s->cols[c], first, max_count, s->tx, bufs[c]);
            approved = expr_select(s->nodes, s->residual_root, bufs, sel, approved, tsel, fsel);
            memcpy(sel, tsel, approved * sizeof(uint32_t));
        }
        if (approved == 0) continue;
        if (s->canonical) qsort(sel, approved, sizeof(uint32_t), cmp_u32);
        /* row-id synthesis: start + current_row + sel[i] (row_group.cpp:573-580) */
        for (uint64_t a = 0; a < approved; a++) {
            int64_t rid = s->row_base + (int64_t)(first + sel[a]);
            if (j->out && j->count < j->out_cap) j->out[j->count] = rid;
            j->count++;
            j->sum_rowid += (uint64_t)rid;
        }
    }
    free(storage);
}

int64_t oracle_table_scan(const oscan *s, int64_t *out_rowids, uint64_t out_cap) {
    if (!s || s->n_cols > OMAX_COLS) return -1;
    scan_job j = {s, 0, (s->n_rows + VEC - 1) / VEC, out_rowids, out_cap, 0, 0};
    scan_range(&j);
    return (int64_t)j.count;
}

/* ---------------------------------------- morsel-driven parallel scan (timing) */

typedef struct {
    const oscan *s;
    uint64_t n_groups;
    volatile uint64_t next; /* shared cursor (row_group_collection.cpp:174-224) */
    pthread_mutex_t lock;
    uint64_t count, sum_rowid;
} mt_state;

static void *mt_worker(void *arg) {
    mt_state *st = (mt_state *)arg;
    int64_t chunk[VEC * 60];
    uint64_t cnt = 0, sum = 0;
    for (;;) {
        pthread_mutex_lock(&st->lock);
        uint64_t g = st->next++;
        pthread_mutex_unlock(&st->lock);
        if (g >= st->n_groups) break;
        scan_job j = {st->s, g * (ROW_GROUP / VEC), (g + 1) * (ROW_GROUP / VEC), chunk, VEC * 60, 0, 0};
        scan_range(&j);
        cnt += j.count;
        sum += j.sum_rowid;
    }
    pthread_mutex_lock(&st->lock);
    st->count += cnt;
    st->sum_rowid += sum;
    pthread_mutex_unlock(&st->lock);
    return NULL;
}

int64_t oracle_table_scan_mt(const oscan *s, int nthreads, uint64_t *sum_rowid) {
    if (!s || s->n_cols > OMAX_COLS) return -1;
    if (nthreads < 1) nthreads = 1;
    mt_state st;
    st.s = s;
    st.n_groups = (s->n_rows + ROW_GROUP - 1) / ROW_GROUP;
    st.next = 0;
    st.count = 0;
    st.sum_rowid = 0;
    pthread_mutex_init(&st.lock, NULL);
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * (size_t)nthreads);
    for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, mt_worker, &st);
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&st.lock);
    if (sum_rowid) *sum_rowid = st.sum_rowid;
    return (int64_t)st.count;
}

/* ------------------------------------------------------------- probe / fetch */

/* ColumnData::FetchRow per row id (index_scan path) with updates for the txn; NULL → 0
 * value with valid flag cleared. */
int oracle_fetch(const ocol *c, const omvcc *tx, const int64_t *rowids, uint64_t n, int64_t row_base,
                 int64_t *out_vals, uint8_t *out_valid) {
    uint64_t st = tx ? tx->start_time : UINT64_MAX - 2, tid = tx ? tx->transaction_id : UINT64_MAX - 2;
    /* each row's update records, in list (= chronological) order: a stable bucketing by row, so
     * a fetch costs O(rows + records) instead of rows × records (test-speed only; same result) */
    uint64_t max_row = 0;
    for (uint64_t u = 0; u < c->n_updates; u++)
        if ((uint64_t)c->upd_rows[u] > max_row) max_row = (uint64_t)c->upd_rows[u];
    uint64_t *first = NULL, *order = NULL;
    if (c->n_updates) {
        first = (uint64_t *)calloc(max_row + 2, sizeof(uint64_t));
        order = (uint64_t *)malloc(c->n_updates * sizeof(uint64_t));
        if (!first || !order) {
            free(first);
            free(order);
            return -1;
        }
        for (uint64_t u = 0; u < c->n_updates; u++) first[(uint64_t)c->upd_rows[u] + 1]++;
        for (uint64_t r = 0; r <= max_row; r++) first[r + 1] += first[r];
        uint64_t *fill = (uint64_t *)malloc((max_row + 1) * sizeof(uint64_t));
        if (!fill) {
            free(first);
            free(order);
            return -1;
        }
        memcpy(fill, first, (max_row + 1) * sizeof(uint64_t));
        for (uint64_t u = 0; u < c->n_updates; u++) order[fill[(uint64_t)c->upd_rows[u]]++] = u;
        free(fill);
    }
    for (uint64_t i = 0; i < n; i++) {
        uint64_t r = (uint64_t)(rowids[i] - row_base);
        int64_t v = col_value(c, r);
        int valid = row_valid(c, r);
        if (c->n_updates && r <= max_row) {
            for (uint64_t k = first[r]; k < first[r + 1]; k++) {
                const uint64_t u = order[k];
                if (use_inserted(st, tid, c->upd_version[u])) { /* the newest visible record wins */
                    v = c->upd_values[u];
                    valid = c->upd_valid ? c->upd_valid[u] != 0 : 1; /* FetchRowValidity :357-370 */
                }
            }
        }
        out_vals[i] = valid ? v : 0;
        if (out_valid) out_valid[i] = (uint8_t)valid;
    }
    free(first);
    free(order);
    return 0;
}

/* Q6 aggregate sum(l_extendedprice * l_discount) over row ids, as a 128-bit integer
 * (DECIMAL(38,4) storage), returned as lo/hi words. */
void oracle_sum_product(const int64_t *a, const int64_t *b, const int64_t *rowids, uint64_t n, int64_t row_base,
                        uint64_t *lo, int64_t *hi) {
    __int128 acc = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t r = (uint64_t)(rowids[i] - row_base);
        acc += (__int128)a[r] * (__int128)b[r];
    }
    *lo = (uint64_t)acc;
    *hi = (int64_t)(acc >> 64);
}

/* ----------------------------------------------------------- bitmap evaluator */

/* Postfix program over 64-bit-word bitvectors: the CPU sibling of the GPU evaluator. */
int64_t oracle_bitmap_eval(const uint64_t *const *leaves, const int32_t *prog, int n_prog, uint64_t n_rows,
                           int64_t row_base, int64_t *out, uint64_t out_cap, uint64_t *result_words) {
    uint64_t n_words = (n_rows + 63) / 64;
    uint64_t count = 0;
    uint64_t stack[64];
    for (uint64_t w = 0; w < n_words; w++) {
        int sp = 0;
        for (int p = 0; p < n_prog; p++) {
            int32_t op = prog[p];
            if (op >= 0) {
                stack[sp++] = leaves[op][w];
            } else if (op == OB_NOT) {
                stack[sp - 1] = ~stack[sp - 1];
            } else {
                uint64_t b = stack[--sp], a = stack[--sp];
                uint64_t r = op == OB_AND ? (a & b) : op == OB_OR ? (a | b) : (a & ~b);
                stack[sp++] = r;
            }
        }
        uint64_t word = stack[0];
        if (w == n_words - 1 && (n_rows & 63)) word &= (1ULL << (n_rows & 63)) - 1;
        if (result_words) result_words[w] = word;
        while (word) {
            int b = __builtin_ctzll(word);
            if (out && count < out_cap) out[count] = row_base + (int64_t)(w * 64 + (uint64_t)b);
            count++;
            word &= word - 1;
        }
    }
    return (int64_t)count;
}

/* Reference-semantics bitvector of one predicate over a column (what the GPU K0 kernel
 * builds): bit r = valid(r) && v[r] CMP c. */
void oracle_build_bitvector(const ocol *c, uint64_t n_rows, int cmp, int64_t constant, uint64_t *words) {
    uint64_t n_words = (n_rows + 63) / 64;
    memset(words, 0, n_words * 8);
    for (uint64_t r = 0; r < n_rows; r++) {
        if (row_valid(c, r) && cmp_typed(c->type, cmp, col_value(c, r), constant)) words[r >> 6] |= 1ULL << (r & 63);
    }
}

/* DuckDB Hash(int64) = MurmurHash64 (src/include/duckdb/common/types/hash.hpp:17-24,
 * src/common/types/hash.cpp:18-21); bit_xor over row ids is the survey's fingerprint. */
uint64_t oracle_xor_hash(const int64_t *rowids, uint64_t n) {
    uint64_t h = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t x = (uint64_t)rowids[i];
        x ^= x >> 32;
        x *= 0xd6e8feb86659fd93ULL;
        x ^= x >> 32;
        x *= 0xd6e8feb86659fd93ULL;
        x ^= x >> 32;
        h ^= x;
    }
    return h;
}
