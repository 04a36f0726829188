/* ORACLE — test infrastructure only (see cpu_ref.c header). */
#ifndef CUBIT_ORACLE_CPU_REF_H
#define CUBIT_ORACLE_CPU_REF_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OMAX_COLS 16

/* FLOAT / DOUBLE: `data` holds the IEEE values; constants, update values and fetched values
 * carry their bit patterns (FLOAT: the 32-bit pattern, zero-extended) */
/* VARCHAR: `data` is an array of ostring; constants, update values and fetched values carry the
 * address of an ostring (string_t comparisons: unsigned bytes, then length — string_type.hpp:143-206) */
/* UINT64 (UBIGINT): the values' bits in `data`, constants and values as those bits, compared unsigned */
/* INT128 / UINT128 (HUGEINT / UHUGEINT): `data` is an array of ohuge (hugeint_t / uhugeint_t:
 * lower, upper — hugeint.hpp, uhugeint.hpp); constants, update values and fetched values carry the
 * address of an ohuge; compared as 128-bit integers, signed / unsigned */
enum { OTYPE_INT32 = 0, OTYPE_INT64 = 1, OTYPE_FLOAT = 2, OTYPE_DOUBLE = 3, OTYPE_VARCHAR = 4, OTYPE_UINT64 = 5,
       OTYPE_INT128 = 6, OTYPE_UINT128 = 7 };
typedef struct {
    const char *data;
    uint64_t size;
} ostring;
typedef struct {
    uint64_t lower;
    uint64_t upper; /* int64_t for HUGEINT */
} ohuge;
/* ExpressionType comparisons used by ConstantFilter (table_filter.hpp / constant_filter.cpp) */
enum { OCMP_EQ = 0, OCMP_NE = 1, OCMP_LT = 2, OCMP_LE = 3, OCMP_GT = 4, OCMP_GE = 5 };
/* TableFilterType (src/include/duckdb/planner/table_filter.hpp:20-27) */
enum { OF_CONST = 0, OF_IS_NULL = 1, OF_IS_NOT_NULL = 2, OF_OR = 3, OF_AND = 4 };
/* bitmap program opcodes (operands >= 0 are leaf indices) */
enum { OB_AND = -1, OB_OR = -2, OB_ANDNOT = -3, OB_NOT = -4 };

typedef struct {
    int32_t type;              /* OTYPE_* */
    int32_t pad;
    const void *data;          /* base values */
    const uint64_t *validity;  /* LSB-first words, NULL = all valid */
    uint64_t n_updates;        /* chronological update records */
    const int64_t *upd_rows;
    const int64_t *upd_values;
    const uint64_t *upd_version;
    const uint8_t *upd_valid;  /* per record: 0 = SET NULL (validity update chain), NULL = all values */
} ocol;

typedef struct {
    const uint64_t *inserted;  /* per-row insert ids, NULL = all 0 */
    const uint64_t *deleted;   /* per-row delete ids, NULL = none */
    uint64_t start_time;
    uint64_t transaction_id;
} omvcc;

typedef struct {
    int32_t kind;       /* OF_* */
    int32_t cmp;        /* OCMP_* for OF_CONST */
    int32_t column;     /* column (residual trees only) */
    int32_t n_children; /* OF_AND / OF_OR */
    int64_t constant;
} ofilter;

typedef struct {
    int32_t column;
    int32_t root; /* index of this column's filter subtree in nodes */
} opushed;

typedef struct {
    const ocol *cols;
    int32_t n_cols;
    int32_t n_pushed;
    const opushed *pushed;  /* TableFilterSet entries in evaluation order */
    const ofilter *nodes;
    int32_t residual_root;  /* -1 = none */
    int32_t canonical;      /* 1 = sort each vector's selection ascending */
    uint64_t n_rows;
    int64_t row_base;
    const omvcc *tx;        /* NULL = everything visible */
} oscan;

int64_t oracle_table_scan(const oscan *s, int64_t *out_rowids, uint64_t out_cap);
int64_t oracle_table_scan_mt(const oscan *s, int nthreads, uint64_t *sum_rowid);
int oracle_fetch(const ocol *c, const omvcc *tx, const int64_t *rowids, uint64_t n, int64_t row_base,
                 int64_t *out_vals, uint8_t *out_valid);
void oracle_sum_product(const int64_t *a, const int64_t *b, const int64_t *rowids, uint64_t n, int64_t row_base,
                        uint64_t *lo, int64_t *hi);
int64_t oracle_bitmap_eval(const uint64_t *const *leaves, const int32_t *prog, int n_prog, uint64_t n_rows,
                           int64_t row_base, int64_t *out, uint64_t out_cap, uint64_t *result_words);
void oracle_build_bitvector(const ocol *c, uint64_t n_rows, int cmp, int64_t constant, uint64_t *words);
uint64_t oracle_xor_hash(const int64_t *rowids, uint64_t n);

/* DuckDB BITPACKING restatement (bitpacking_ref.c). mode: 1 AUTO, 2 CONSTANT, 3 CONSTANT_DELTA,
 * 4 DELTA_FOR, 5 FOR (BitpackingMode). ttype: the value's byte size (1, 2, 4, 8) | 0x100 when
 * unsigned. compress: 0 ok, 1 not bitpackable, < 0 error. */
int oracle_bp_compress(const void *values, int ttype, const uint8_t *valid, uint64_t n, int mode, uint64_t block_size,
                       uint8_t *out, uint64_t out_cap, uint64_t *seg_off, uint64_t *seg_size, uint64_t *seg_count,
                       uint32_t max_segs, uint32_t *n_segs);
int oracle_bp_decode(const uint8_t *bytes, const uint64_t *seg_off, const uint64_t *seg_count, uint32_t n_segs,
                     int ttype, void *out_values);
int oracle_bp_group_modes(const uint8_t *bytes, const uint64_t *seg_off, const uint64_t *seg_count, uint32_t n_segs,
                          uint8_t *modes, uint64_t cap);

#ifdef __cplusplus
}
#endif
#endif
