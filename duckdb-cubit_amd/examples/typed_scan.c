/*
 * typed_scan — the typed columns through the C ABI alone (no Python, no PyTorch): what a DuckDB
 * extension does with FLOAT / DOUBLE, UBIGINT, VARCHAR and HUGEINT / UHUGEINT columns and their
 * pushed comparisons (tests/test_gpu_c_example.py feeds it the reference's own filter cases).
 *
 *   typed_scan < spec
 *
 * The spec, one item per line:
 *   column <type>                 type: integer bigint ubigint float double varchar hugeint uhugeint
 *   row <v0> <v1> …               one value per column: NULL, or a literal (numbers as written,
 *                                 nan / inf / -inf; VARCHAR as x<hex bytes>, "x" = the empty string)
 *   index <col> range|equality    after the rows: build that index on the column
 *   query <n> <col> <op> <v> …    n comparisons ANDed (op: = <> < <= > >=, or isnull / isnotnull
 *                                 with v = -), as the TableFilterSet DuckDB would push
 * Each query runs through the seq_scan-shaped callbacks of cubit_scan.h (init_global with the
 * row id and every column projected, one local state, 2,048-row chunks) and prints
 *   result <count>
 *   <row id> <v0> <v1> …          ascending row id, values rendered as the spec writes them
 *
 * What it shows, type by type:
 *   FLOAT / DOUBLE   columns and constants as IEEE bit patterns (cubit_table_add_column);
 *   UBIGINT          the 64 bits, compared unsigned;
 *   VARCHAR          a cubit_dict over the column's strings, codes registered with
 *                    cubit_table_add_dict_column, constants as cubit_strings, chunk codes decoded
 *                    with cubit_dict_entry (the shim's CopyOut);
 *   HUGEINT/UHUGEINT the same over 16-byte order keys (cubit_key128; cubit_value128 back).
 */
#define _POSIX_C_SOURCE 200809L
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "cubit_gpu.h"
#include "cubit_scan.h"

#define CHECK(call)                                                                  \
    do {                                                                             \
        int rc_ = (call);                                                            \
        if (rc_ != CUBIT_OK) {                                                       \
            fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, cubit_last_error()); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)
#define CHECK_SCAN(call)                                                                  \
    do {                                                                                  \
        int rc_ = (call);                                                                 \
        if (rc_ != CUBIT_OK) {                                                            \
            fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, cubit_scan_last_error()); \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

enum { T_INTEGER, T_BIGINT, T_UBIGINT, T_FLOAT, T_DOUBLE, T_VARCHAR, T_HUGEINT, T_UHUGEINT };
static const char *TYPE_NAMES[] = {"integer", "bigint", "ubigint", "float", "double", "varchar", "hugeint", "uhugeint"};
#define MAX_COLS 8
#define MAX_TERMS 16

typedef struct {
    int type;
    uint64_t n;
    int64_t *values;    /* integer-backed and FP columns: the ABI's int64 form */
    char **bytes;       /* dictionary columns: each row's string / order key */
    uint64_t *lens;
    unsigned char *valid;
    cubit_dict *dict;
} column;

static column cols[MAX_COLS];
static int n_cols;
static uint64_t n_rows, cap_rows;

static void die(const char *what, const char *tok) {
    fprintf(stderr, "typed_scan: %s '%s'\n", what, tok ? tok : "");
    exit(2);
}

static int is_dict(int type) { return type == T_VARCHAR || type == T_HUGEINT || type == T_UHUGEINT; }

/* a decimal literal as a 128-bit two's-complement value */
static unsigned __int128 parse128(const char *s) {
    int neg = *s == '-';
    unsigned __int128 v = 0;
    for (const char *p = s + neg; *p; p++) {
        if (*p < '0' || *p > '9') die("bad integer", s);
        v = v * 10 + (unsigned)(*p - '0');
    }
    return neg ? (unsigned __int128)0 - v : v;
}

static void print128(unsigned __int128 u, int is_signed) {
    char buf[48];
    int i = 47, neg = is_signed && (u >> 127);
    buf[i] = 0;
    if (neg) u = (unsigned __int128)0 - u;
    do {
        buf[--i] = (char)('0' + (int)(u % 10));
        u /= 10;
    } while (u);
    if (neg) buf[--i] = '-';
    fputs(buf + i, stdout);
}

/* a literal in the ABI's int64 form (FP: bit pattern; UBIGINT: bits) */
static int64_t scalar_of(int type, const char *tok) {
    switch (type) {
    case T_FLOAT: {
        float f = strtof(tok, NULL);
        uint32_t u;
        memcpy(&u, &f, 4);
        return (int64_t)u;
    }
    case T_DOUBLE: {
        double d = strtod(tok, NULL);
        int64_t b;
        memcpy(&b, &d, 8);
        return b;
    }
    case T_UBIGINT: return (int64_t)strtoull(tok, NULL, 10);
    default: return strtoll(tok, NULL, 10);
    }
}

/* a dictionary column's literal as the bytes its dictionary holds: VARCHAR x<hex>, or the
 * 16-byte order key of a HUGEINT / UHUGEINT */
static char *bytes_of(int type, const char *tok, uint64_t *len) {
    if (type == T_VARCHAR) {
        if (tok[0] != 'x') die("VARCHAR literal is not x<hex>", tok);
        const size_t h = strlen(tok + 1);
        char *b = malloc(h / 2 + 1);
        for (size_t i = 0; i < h / 2; i++) {
            unsigned x;
            if (sscanf(tok + 1 + 2 * i, "%2x", &x) != 1) die("bad hex", tok);
            b[i] = (char)x;
        }
        *len = h / 2;
        return b;
    }
    const unsigned __int128 v = parse128(tok);
    char *k = malloc(16);
    cubit_key128(type == T_HUGEINT ? CUBIT_TYPE_INT128 : CUBIT_TYPE_UINT128, (uint64_t)v, (uint64_t)(v >> 64),
                 (unsigned char *)k);
    *len = 16;
    return k;
}

static void print_value(const column *c, int64_t v, int valid) {
    if (!valid) {
        fputs("NULL", stdout);
        return;
    }
    switch (c->type) {
    case T_FLOAT:
    case T_DOUBLE: {
        double d;
        if (c->type == T_FLOAT) {
            uint32_t u = (uint32_t)v;
            float f;
            memcpy(&f, &u, 4);
            d = f;
        } else {
            memcpy(&d, &v, 8);
        }
        if (d != d) fputs("nan", stdout);
        else if (d == 1.0 / 0.0) fputs("inf", stdout);
        else if (d == -1.0 / 0.0) fputs("-inf", stdout);
        else printf(c->type == T_FLOAT ? "%.9g" : "%.17g", d);
        return;
    }
    case T_UBIGINT: printf("%" PRIu64, (uint64_t)v); return;
    case T_VARCHAR:
    case T_HUGEINT:
    case T_UHUGEINT: {
        const char *p = NULL;
        uint64_t len = 0;
        CHECK(cubit_dict_entry(c->dict, (uint64_t)v, &p, &len));  /* the shim's CopyOut */
        if (c->type == T_VARCHAR) {
            putchar('x');
            for (uint64_t i = 0; i < len; i++) printf("%02x", (unsigned char)p[i]);
        } else {
            uint64_t lower, upper;
            cubit_value128(c->type == T_HUGEINT ? CUBIT_TYPE_INT128 : CUBIT_TYPE_UINT128, (const unsigned char *)p,
                           &lower, &upper);
            print128(((unsigned __int128)upper << 64) | lower, c->type == T_HUGEINT);
        }
        return;
    }
    default: printf("%" PRId64, v); return;
    }
}

/* every column on the GPU: dictionary columns through a cubit_dict over their valid values */
static void register_columns(cubit_table *t) {
    for (int j = 0; j < n_cols; j++) {
        column *c = &cols[j];
        uint64_t *words = calloc((n_rows + 63) / 64 + 1, 8);
        int all = 1;
        for (uint64_t r = 0; r < n_rows; r++) {
            if (c->valid[r]) words[r >> 6] |= 1ull << (r & 63);
            else all = 0;
        }
        if (is_dict(c->type)) {
            uint64_t total = 0;
            for (uint64_t r = 0; r < n_rows; r++) total += c->valid[r] ? c->lens[r] : 0;
            char *buf = malloc(total + 1);
            uint64_t *offs = malloc((n_rows + 1) * 8);
            offs[0] = 0;
            for (uint64_t r = 0; r < n_rows; r++) {
                const uint64_t l = c->valid[r] ? c->lens[r] : 0;
                if (l) memcpy(buf + offs[r], c->bytes[r], l);
                offs[r + 1] = offs[r] + l;
            }
            /* the dictionary over the valid values alone (NULL rows are empty slots of the encode) */
            char *vbuf = malloc(total + 1);
            uint64_t *voffs = malloc((n_rows + 1) * 8), nv = 0;
            voffs[0] = 0;
            for (uint64_t r = 0; r < n_rows; r++) {
                if (!c->valid[r]) continue;
                if (c->lens[r]) memcpy(vbuf + voffs[nv], c->bytes[r], c->lens[r]);
                voffs[nv + 1] = voffs[nv] + c->lens[r];
                nv++;
            }
            CHECK(cubit_dict_create(vbuf, voffs, nv, &c->dict));
            free(vbuf);
            free(voffs);
            int32_t *codes = malloc((n_rows + 1) * 4);
            CHECK(cubit_dict_encode(c->dict, buf, offs, n_rows, words, codes));
            CHECK(cubit_table_add_dict_column(t, j, c->dict, codes, all ? NULL : words, 0));
            free(codes);
            free(offs);
            free(buf);
        } else if (c->type == T_INTEGER || c->type == T_FLOAT) {
            int32_t *v = malloc((n_rows + 1) * 4);
            for (uint64_t r = 0; r < n_rows; r++) v[r] = (int32_t)(uint32_t)c->values[r];
            CHECK(cubit_table_add_column(t, j, c->type == T_FLOAT ? CUBIT_TYPE_FLOAT : CUBIT_TYPE_INT32, v,
                                         all ? NULL : words, 0));
            free(v);
        } else {
            const int type = c->type == T_DOUBLE ? CUBIT_TYPE_DOUBLE : c->type == T_UBIGINT ? CUBIT_TYPE_UINT64
                                                                                              : CUBIT_TYPE_INT64;
            CHECK(cubit_table_add_column(t, j, type, c->values, all ? NULL : words, 0));
        }
        free(words);
    }
}

typedef struct {
    int64_t rowid;
    int64_t v[MAX_COLS];
    unsigned char ok[MAX_COLS];
} out_row;

static int by_rowid(const void *a, const void *b) {
    const int64_t x = ((const out_row *)a)->rowid, y = ((const out_row *)b)->rowid;
    return x < y ? -1 : x > y;
}

static void run_query(cubit_table *t, char **tok, int n_terms) {
    cubit_filter_node nodes[1 + 2 * MAX_TERMS];
    cubit_string strs[MAX_TERMS];
    char *owned[MAX_TERMS];
    int n = 0, n_owned = 0;
    nodes[n++] = (cubit_filter_node){CUBIT_FILTER_AND, 0, -1, n_terms, 0};
    for (int k = 0; k < n_terms; k++) {
        const int col = atoi(tok[3 * k]);
        const char *op = tok[3 * k + 1], *lit = tok[3 * k + 2];
        if (col < 0 || col >= n_cols) die("bad column", tok[3 * k]);
        cubit_filter_node f = {CUBIT_FILTER_CONSTANT, 0, col, 0, 0};
        if (!strcmp(op, "isnull")) f.kind = CUBIT_FILTER_IS_NULL;
        else if (!strcmp(op, "isnotnull")) f.kind = CUBIT_FILTER_IS_NOT_NULL;
        else {
            f.cmp = !strcmp(op, "=") ? CUBIT_CMP_EQ : !strcmp(op, "<>") ? CUBIT_CMP_NE : !strcmp(op, "<") ? CUBIT_CMP_LT
                  : !strcmp(op, "<=") ? CUBIT_CMP_LE : !strcmp(op, ">") ? CUBIT_CMP_GT : !strcmp(op, ">=") ? CUBIT_CMP_GE
                  : -1;
            if (f.cmp < 0) die("bad comparison", op);
            if (is_dict(cols[col].type)) {  /* the constant as the address of a cubit_string */
                uint64_t len;
                owned[n_owned] = bytes_of(cols[col].type, lit, &len);
                strs[n_owned] = (cubit_string){owned[n_owned], len};
                f.constant = (int64_t)(intptr_t)&strs[n_owned];
                n_owned++;
            } else {
                f.constant = scalar_of(cols[col].type, lit);
            }
        }
        nodes[n++] = f;
    }
    uint64_t column_ids[MAX_COLS + 1], proj[MAX_COLS + 1];
    for (int j = 0; j < n_cols; j++) column_ids[j] = (uint64_t)j, proj[j + 1] = (uint64_t)j;
    column_ids[n_cols] = CUBIT_COLUMN_ROW_ID;
    proj[0] = (uint64_t)n_cols;
    const cubit_txn txn = {0, 0};
    cubit_scan *scan = NULL;
    cubit_scan_local *local = NULL;
    CHECK_SCAN(cubit_scan_init_global(t, column_ids, (uint32_t)n_cols + 1, proj, (uint32_t)n_cols + 1, nodes,
                                      (uint32_t)n, &txn, &scan));
    CHECK_SCAN(cubit_scan_init_local(scan, &local));
    int64_t *out[MAX_COLS + 1];
    uint64_t *valid[MAX_COLS + 1];
    for (int j = 0; j <= n_cols; j++) {
        out[j] = malloc(2048 * 8);
        valid[j] = malloc(32 * 8);
    }
    out_row *rows = malloc(sizeof(out_row) * (n_rows + 1));
    uint64_t total = 0;
    for (;;) {
        uint64_t cnt = 0;
        CHECK_SCAN(cubit_scan_function_validity(scan, local, out, valid, &cnt));
        if (!cnt) break;
        for (uint64_t i = 0; i < cnt; i++, total++) {
            rows[total].rowid = out[0][i];
            for (int j = 0; j < n_cols; j++) {
                rows[total].v[j] = out[j + 1][i];
                rows[total].ok[j] = (unsigned char)((valid[j + 1][i >> 6] >> (i & 63)) & 1);
            }
        }
    }
    qsort(rows, total, sizeof(out_row), by_rowid);
    printf("result %" PRIu64 "\n", total);
    for (uint64_t i = 0; i < total; i++) {
        printf("%" PRId64, rows[i].rowid);
        for (int j = 0; j < n_cols; j++) {
            putchar(' ');
            print_value(&cols[j], rows[i].v[j], rows[i].ok[j]);
        }
        putchar('\n');
    }
    fflush(stdout);
    CHECK_SCAN(cubit_scan_local_destroy(local));
    CHECK_SCAN(cubit_scan_destroy(scan));
    for (int j = 0; j <= n_cols; j++) {
        free(out[j]);
        free(valid[j]);
    }
    free(rows);
    for (int k = 0; k < n_owned; k++) free(owned[k]);
}

int main(void) {
    cubit_ctx *ctx = NULL;
    cubit_table *t = NULL;
    CHECK(cubit_ctx_create(0, &ctx));
    char line[1 << 16];
    while (fgets(line, sizeof line, stdin)) {
        char *tok[1 + 3 * MAX_TERMS + 2];
        int nt = 0;
        for (char *p = strtok(line, " \t\r\n"); p && nt < (int)(sizeof tok / sizeof tok[0]); p = strtok(NULL, " \t\r\n"))
            tok[nt++] = p;
        if (!nt) continue;
        if (!strcmp(tok[0], "column")) {
            if (t || n_cols == MAX_COLS || nt != 2) die("column", nt > 1 ? tok[1] : "");
            int type = -1;
            for (int k = 0; k < 8; k++)
                if (!strcmp(tok[1], TYPE_NAMES[k])) type = k;
            if (type < 0) die("unknown type", tok[1]);
            cols[n_cols++] = (column){.type = type};
        } else if (!strcmp(tok[0], "row")) {
            if (t || nt != 1 + n_cols) die("row before the columns or of the wrong width", tok[0]);
            if (n_rows == cap_rows) {
                cap_rows = cap_rows ? 2 * cap_rows : 64;
                for (int j = 0; j < n_cols; j++) {
                    cols[j].values = realloc(cols[j].values, cap_rows * 8);
                    cols[j].bytes = realloc(cols[j].bytes, cap_rows * sizeof(char *));
                    cols[j].lens = realloc(cols[j].lens, cap_rows * 8);
                    cols[j].valid = realloc(cols[j].valid, cap_rows);
                }
            }
            for (int j = 0; j < n_cols; j++) {
                column *c = &cols[j];
                const int ok = strcmp(tok[1 + j], "NULL") != 0;
                c->valid[n_rows] = (unsigned char)ok;
                c->values[n_rows] = 0;
                c->bytes[n_rows] = NULL;
                c->lens[n_rows] = 0;
                if (ok && is_dict(c->type)) c->bytes[n_rows] = bytes_of(c->type, tok[1 + j], &c->lens[n_rows]);
                else if (ok) c->values[n_rows] = scalar_of(c->type, tok[1 + j]);
            }
            n_rows++;
        } else if (!strcmp(tok[0], "index") || !strcmp(tok[0], "query")) {
            if (!t) {
                CHECK(cubit_table_create(ctx, n_rows, 0, &t));
                register_columns(t);
            }
            if (!strcmp(tok[0], "index")) {
                if (nt != 3) die("index <col> range|equality", tok[0]);
                const int enc = !strcmp(tok[2], "range") ? CUBIT_INDEX_RANGE : CUBIT_INDEX_EQUALITY;
                CHECK(cubit_table_build_index(t, atoi(tok[1]), enc, NULL, 0));
            } else {
                const int terms = nt > 1 ? atoi(tok[1]) : 0;
                if (terms < 1 || terms > MAX_TERMS || nt != 2 + 3 * terms) die("query <n> (<col> <op> <v>)*n", tok[0]);
                run_query(t, tok + 2, terms);
            }
        } else {
            die("unknown item", tok[0]);
        }
    }
    if (t) CHECK(cubit_table_destroy(t));
    for (int j = 0; j < n_cols; j++) {
        if (cols[j].dict) CHECK(cubit_dict_destroy(cols[j].dict));
        for (uint64_t r = 0; r < n_rows; r++) free(cols[j].bytes[r]);
        free(cols[j].values);
        free(cols[j].bytes);
        free(cols[j].lens);
        free(cols[j].valid);
    }
    CHECK(cubit_ctx_destroy(ctx));
    return 0;
}
