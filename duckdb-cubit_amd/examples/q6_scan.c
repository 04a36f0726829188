/*
 * q6_scan — TPC-H Q6 through the C ABI alone (no Python, no PyTorch): what a C/C++ host such
 * as a DuckDB extension does with libcubitgpu.so and libcubit_scan.so.
 *
 *   q6_scan <sf> [threads] [--partitions N]      e.g. q6_scan 1, q6_scan 100 16, q6_scan 100 8 --partitions 8
 *
 * 1. generates lineitem's Q6 columns with libcubit_datagen (the repo's dbgen restatement);
 * 2. registers them on the GPU and builds the bitmap indexes (cubit_table_add_column /
 *    cubit_table_build_index);
 * 3. runs Q6's TableFilterSet three ways: cubit_table_scan (row ids in HBM), the fused
 *    cubit_table_sum_product (revenue), and the seq_scan-shaped callbacks of cubit_scan.h
 *    (init_global / init_local / function until an empty chunk);
 * 4. prints one line: rows, rows from the table function, Σ row ids, revenue.
 * tests/test_gpu_c_example.py checks that line against the reference's answer files.
 * 5. with [threads]: the whole query through the callbacks as a DuckDB pipeline runs it —
 *    init_global, then `threads` pipeline tasks (pthreads), each with its own local state,
 *    draining 2,048-row chunks of (l_extendedprice, l_discount) into a partial revenue —
 *    timed end to end (best of Q6_REPS runs, default 3; the median beside it) and checked against
 *    the fused revenue; one more line.
 * 6. with --partitions N: lineitem held as N row-range partitions, partition p on device
 *    p mod (devices visible), one context per device — one process driving every GPU of the node —
 *    and the same pipeline over all of them through one cursor (cubit_scan_init_global_multi:
 *    each partition decodes and probes on its own device, windows are copied from their own
 *    device, no device-to-device exchange); timed and checked the same way; one more line.
 */
#define _POSIX_C_SOURCE 200809L
#include <inttypes.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "cubit_gpu.h"
#include "cubit_scan.h"

/* libcubit_datagen.so */
int64_t cubit_tpch_orders(double sf);
int64_t cubit_tpch_lineitem_rows(double sf, int64_t order_begin, int64_t order_end, int nthreads);
int64_t cubit_tpch_lineitem_gen(double sf, int64_t order_begin, int64_t order_end, int32_t *shipdate,
                                int64_t *discount, int64_t *quantity, int64_t *extprice, int nthreads);

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

/* days since 1970-01-01 of y-m-1 (DuckDB DATE) */
static int32_t date_of(int y, int m) {
    static const int cum[12] = {0, 31, 59, 90, 120, 151, 181, 212, 243, 273, 304, 334};
    int32_t days = 0;
    for (int yy = 1970; yy < y; ++yy) days += (yy % 4 == 0 && (yy % 100 != 0 || yy % 400 == 0)) ? 366 : 365;
    days += cum[m - 1];
    if (m > 2 && (y % 4 == 0 && (y % 100 != 0 || y % 400 == 0))) days += 1;
    return days;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* one pipeline task: TableScanInitLocal, then TableScanFunc until an empty chunk, aggregating
 * sum(l_extendedprice * l_discount) of its chunks (DuckDB's PhysicalUngroupedAggregate sink) */
typedef struct {
    cubit_scan *scan;
    uint64_t rows;
    __int128 revenue;
    int rc;
    double scan_s, consume_s; /* time inside cubit_scan_function / in the aggregate */
} task_t;

static void *pipeline_task(void *arg) {
    task_t *tk = (task_t *)arg;
    cubit_scan_local *local;
    tk->rc = cubit_scan_init_local(tk->scan, &local);
    if (tk->rc != CUBIT_OK) return NULL;
    int64_t *cols[2] = {malloc(2048 * 8), malloc(2048 * 8)};
    uint64_t got = 0;
    double t = now_s();
    do {
        tk->rc = cubit_scan_function(tk->scan, local, cols, &got);
        const double t1 = now_s();
        tk->scan_s += t1 - t;
        if (tk->rc != CUBIT_OK) break;
        __int128 s = 0;
        for (uint64_t i = 0; i < got; ++i) s += (__int128)cols[0][i] * cols[1][i];
        tk->revenue += s;
        tk->rows += got;
        t = now_s();
        tk->consume_s += t - t1;
    } while (got);
    cubit_scan_local_destroy(local);
    free(cols[0]);
    free(cols[1]);
    return NULL;
}

/* `threads` pipeline tasks over one init_global (best of Q6_REPS end to end); returns the best
 * time, the median in *median_ms */
static double run_pipeline(cubit_table *const *parts, uint32_t n_parts, const cubit_filter_node *q6, uint32_t nn,
                           int threads, uint64_t want_rows, __int128 want_rev, double *init_ms, double split_ms[2],
                           double *median_ms) {
    const uint64_t proj_ids[] = {3, 1};
    double best = 1e30;
    task_t *tasks = calloc((size_t)threads, sizeof(task_t));
    pthread_t *th = calloc((size_t)threads, sizeof(pthread_t));
    const char *reps_env = getenv("Q6_REPS");
    const int reps = reps_env && atoi(reps_env) > 0 ? atoi(reps_env) : 3;
    double *times = calloc((size_t)reps, sizeof(double));
    for (int rep = 0; rep < reps; ++rep) {
        const double t0 = now_s();
        cubit_scan *ps;
        CHECK_SCAN(cubit_scan_init_global_multi(parts, n_parts, proj_ids, 2, NULL, 0, q6, nn, NULL, &ps));
        const double t1 = now_s();
        for (int i = 0; i < threads; ++i) {
            tasks[i] = (task_t){ps, 0, 0, 0, 0, 0};
            if (pthread_create(&th[i], NULL, pipeline_task, &tasks[i]) != 0) exit(1);
        }
        uint64_t rows_p = 0;
        __int128 rev_p = 0;
        double scan_s = 0, consume_s = 0;
        for (int i = 0; i < threads; ++i) {
            pthread_join(th[i], NULL);
            CHECK_SCAN(tasks[i].rc);
            rows_p += tasks[i].rows;
            rev_p += tasks[i].revenue;
            scan_s += tasks[i].scan_s;
            consume_s += tasks[i].consume_s;
        }
        const double t2 = now_s();
        CHECK_SCAN(cubit_scan_destroy(ps));
        times[rep] = t2 - t0;
        if (t2 - t0 < best) {
            best = t2 - t0;
            *init_ms = (t1 - t0) * 1e3;
            split_ms[0] = scan_s * 1e3 / threads; /* per task: inside the callbacks */
            split_ms[1] = consume_s * 1e3 / threads; /* per task: the aggregate's own work */
        }
        if (rows_p != want_rows || rev_p != want_rev) {
            fprintf(stderr, "pipeline: %" PRIu64 " rows, revenue differs from the fused sum\n", rows_p);
            exit(1);
        }
    }
    for (int i = 1; i < reps; ++i) /* insertion sort: the median */
        for (int j = i; j > 0 && times[j] < times[j - 1]; --j) {
            const double x = times[j];
            times[j] = times[j - 1];
            times[j - 1] = x;
        }
    *median_ms = times[reps / 2] * 1e3;
    free(times);
    free(tasks);
    free(th);
    return best;
}

int main(int argc, char **argv) {
    int n_partitions = 0;
    for (int i = 1; i + 1 < argc; ++i)
        if (!strcmp(argv[i], "--partitions")) {
            n_partitions = atoi(argv[i + 1]);
            for (int j = i; j + 2 < argc; ++j) argv[j] = argv[j + 2];  /* drop the option */
            argc -= 2;
            break;
        }
    const double sf = argc > 1 ? atof(argv[1]) : 1.0;
    const int64_t orders = cubit_tpch_orders(sf);
    const int64_t n = cubit_tpch_lineitem_rows(sf, 0, orders, 0);
    int32_t *shipdate = malloc(n * sizeof(int32_t));
    int64_t *discount = malloc(n * sizeof(int64_t)), *quantity = malloc(n * sizeof(int64_t));
    int64_t *extprice = malloc(n * sizeof(int64_t));
    if (!shipdate || !discount || !quantity || !extprice) return 1;
    if (cubit_tpch_lineitem_gen(sf, 0, orders, shipdate, discount, quantity, extprice, 0) != n) return 1;

    cubit_ctx *ctx;
    cubit_table *t;
    CHECK(cubit_ctx_create(0, &ctx));
    CHECK(cubit_table_create(ctx, (uint64_t)n, 0, &t));
    CHECK(cubit_table_add_column(t, 0, CUBIT_TYPE_INT32, shipdate, NULL, 0));
    CHECK(cubit_table_add_column(t, 1, CUBIT_TYPE_INT64, discount, NULL, 0));
    CHECK(cubit_table_add_column(t, 2, CUBIT_TYPE_INT64, quantity, NULL, 0));
    CHECK(cubit_table_add_column(t, 3, CUBIT_TYPE_INT64, extprice, NULL, 0));
    int64_t edges[85];
    int ne = 0;
    for (int y = 1992; y <= 1998; ++y)
        for (int m = 1; m <= 12; ++m) edges[ne++] = date_of(y, m);
    edges[ne++] = date_of(1999, 1);
    CHECK(cubit_table_build_index(t, 0, CUBIT_INDEX_RANGE, edges, (uint32_t)ne));
    CHECK(cubit_table_build_index(t, 1, CUBIT_INDEX_RANGE, NULL, 0));
    CHECK(cubit_table_build_index(t, 2, CUBIT_INDEX_RANGE, NULL, 0));

    /* the TableFilterSet DuckDB pushes for Q6 (AND root over the per-column filters) */
    const cubit_filter_node q6[] = {
        {CUBIT_FILTER_AND, 0, 0, 3, 0},
        {CUBIT_FILTER_AND, 0, 0, 3, 0},
        {CUBIT_FILTER_CONSTANT, CUBIT_CMP_GE, 0, 0, date_of(1994, 1)},
        {CUBIT_FILTER_CONSTANT, CUBIT_CMP_LT, 0, 0, date_of(1995, 1)},
        {CUBIT_FILTER_IS_NOT_NULL, 0, 0, 0, 0},
        {CUBIT_FILTER_AND, 0, 1, 3, 0},
        {CUBIT_FILTER_CONSTANT, CUBIT_CMP_GE, 1, 0, 5},
        {CUBIT_FILTER_CONSTANT, CUBIT_CMP_LE, 1, 0, 7},
        {CUBIT_FILTER_IS_NOT_NULL, 0, 1, 0, 0},
        {CUBIT_FILTER_AND, 0, 2, 2, 0},
        {CUBIT_FILTER_CONSTANT, CUBIT_CMP_LT, 2, 0, 2400},
        {CUBIT_FILTER_IS_NOT_NULL, 0, 2, 0, 0},
    };
    const uint32_t nn = sizeof(q6) / sizeof(q6[0]);

    /* 1. row ids in HBM (ascending with CUBIT_SCAN_ORDERED) */
    void *d_ids, *d_cnt, *d_sum;
    CHECK(cubit_dev_alloc(ctx, (uint64_t)n * 8, &d_ids));
    CHECK(cubit_dev_alloc(ctx, 16, &d_cnt));
    CHECK(cubit_dev_alloc(ctx, 16, &d_sum));
    CHECK(cubit_table_scan(t, q6, nn, NULL, d_ids, (uint64_t)n, d_cnt, CUBIT_SCAN_ORDERED));
    CHECK(cubit_sync(ctx));
    uint64_t q = 0;
    CHECK(cubit_memcpy_d2h(ctx, &q, d_cnt, 8));
    int64_t *ids = malloc((q ? q : 1) * sizeof(int64_t));
    CHECK(cubit_memcpy_d2h(ctx, ids, d_ids, q * 8));
    uint64_t sum_ids = 0;
    for (uint64_t i = 0; i < q; ++i) {
        if (i && ids[i] <= ids[i - 1]) {
            fprintf(stderr, "row ids not ascending at %" PRIu64 "\n", i);
            return 1;
        }
        sum_ids += (uint64_t)ids[i];
    }

    /* 2. fused sum(l_extendedprice * l_discount) */
    CHECK(cubit_table_sum_product(t, q6, nn, NULL, 3, 1, d_sum, NULL, 0));
    CHECK(cubit_sync(ctx));
    int64_t s[2];
    CHECK(cubit_memcpy_d2h(ctx, s, d_sum, 16));
    const __int128 rev = ((__int128)s[1] << 64) | (unsigned __int128)(uint64_t)s[0];
    const int64_t whole = (int64_t)(rev / 10000), frac = (int64_t)(rev % 10000);

    /* 3. the seq_scan callbacks: project l_extendedprice and the row id, drain every chunk */
    const uint64_t column_ids[] = {3, CUBIT_COLUMN_ROW_ID};
    cubit_scan *scan;
    cubit_scan_local *local;
    CHECK_SCAN(cubit_scan_init_global(t, column_ids, 2, NULL, 0, q6, nn, NULL, &scan));
    CHECK_SCAN(cubit_scan_init_local(scan, &local));
    int64_t *cols[2] = {malloc(2048 * 8), malloc(2048 * 8)};
    uint64_t rows_tf = 0, sum_tf = 0, got = 0;
    do {
        CHECK_SCAN(cubit_scan_function(scan, local, cols, &got));
        for (uint64_t i = 0; i < got; ++i) {
            if (cols[0][i] != extprice[cols[1][i]]) {
                fprintf(stderr, "probe mismatch at row %" PRId64 "\n", cols[1][i]);
                return 1;
            }
            sum_tf += (uint64_t)cols[1][i];
        }
        rows_tf += got;
    } while (got);
    CHECK_SCAN(cubit_scan_local_destroy(local));
    CHECK_SCAN(cubit_scan_destroy(scan));

    printf("rows %" PRIu64 " table_function_rows %" PRIu64 " sum_rowid %" PRIu64 " table_function_sum_rowid %" PRIu64
           " revenue %" PRId64 ".%04" PRId64 "\n",
           q, rows_tf, sum_ids, sum_tf, whole, frac);

    /* 5. the query as a pipeline of `threads` tasks over the callbacks */
    const int threads = argc > 2 ? atoi(argv[2]) : 0;
    if (threads > 0) {
        double init_ms = 0, split[2] = {0, 0}, median_ms = 0;
        const double best = run_pipeline(&t, 1, q6, nn, threads, q, rev, &init_ms, split, &median_ms);
        printf("pipeline threads %d init_global_ms %.3f total_ms %.3f rows %" PRIu64 " rows_per_s %.4e revenue_match 1"
               " task_scan_ms %.3f task_aggregate_ms %.3f median_ms %.3f\n",
               threads, init_ms, best * 1e3, q, q / best, split[0], split[1], median_ms);
        /* the link's own device-to-host rate into page-locked memory (one 64 MiB copy, best of 3):
         * the floor the pipeline's window copies share */
        const uint64_t link_bytes = (uint64_t)n * 8 < (64ull << 20) ? (uint64_t)n * 8 : (64ull << 20);
        void *h_link;
        CHECK(cubit_host_alloc(ctx, link_bytes, &h_link));
        double link_best = 1e30;
        for (int rep = 0; rep < 3; ++rep) {
            const double l0 = now_s();
            CHECK(cubit_memcpy_d2h(ctx, h_link, d_ids, link_bytes));
            const double l1 = now_s();
            if (l1 - l0 < link_best) link_best = l1 - l0;
        }
        CHECK(cubit_host_free(ctx, h_link));
        printf("link_d2h bytes %" PRIu64 " ms %.3f gb_per_s %.2f\n", link_bytes, link_best * 1e3, link_bytes / link_best / 1e9);
    }

    /* 5b. Q6_AB=1: staged and per-window copies alternated run by run in this process (paired
     * comparison: the box's other tenants load both alike), best and median of each */
    if (threads > 0 && getenv("Q6_AB") && atoi(getenv("Q6_AB")) == 1) {
        const char *reps_env = getenv("Q6_REPS");
        const int reps = reps_env && atoi(reps_env) > 0 ? atoi(reps_env) : 3;
        double ab[2][64];
        int k = 0;
        for (; k < reps && k < 64; ++k)
            for (int mode = 0; mode < 2; ++mode) {
                setenv("CUBIT_SCAN_STAGE_MB", mode ? "0" : "1024", 1);
                setenv("Q6_REPS", "1", 1);
                double init_ms = 0, split[2] = {0, 0}, median_ms = 0;
                ab[mode][k] = run_pipeline(&t, 1, q6, nn, threads, q, rev, &init_ms, split, &median_ms) * 1e3;
            }
        if (reps_env) setenv("Q6_REPS", reps_env, 1);
        unsetenv("CUBIT_SCAN_STAGE_MB");
        for (int mode = 0; mode < 2; ++mode) {
            for (int i = 1; i < k; ++i)
                for (int j = i; j > 0 && ab[mode][j] < ab[mode][j - 1]; --j) {
                    const double x = ab[mode][j];
                    ab[mode][j] = ab[mode][j - 1];
                    ab[mode][j - 1] = x;
                }
            printf("pipeline_ab %s threads %d runs %d best_ms %.3f median_ms %.3f\n", mode ? "per_window" : "staged",
                   threads, k, ab[mode][0], ab[mode][k / 2]);
        }
    }

    /* 6. the same pipeline over N row-range partitions, one context each, spread over the devices */
    if (threads > 0 && n_partitions > 0) {
        int n_dev = 1;
        CHECK(cubit_device_count(&n_dev));
        const int n_ctx = n_dev < n_partitions ? n_dev : n_partitions;
        cubit_ctx **pctx = calloc((size_t)n_ctx, sizeof(cubit_ctx *));
        cubit_table **pt = calloc((size_t)n_partitions, sizeof(cubit_table *));
        for (int d = 0; d < n_ctx; ++d) CHECK(cubit_ctx_create(d, &pctx[d]));
        for (int p = 0; p < n_partitions; ++p) {
            const int64_t b = n * p / n_partitions, e = n * (p + 1) / n_partitions;
            CHECK(cubit_table_create(pctx[p % n_ctx], (uint64_t)(e - b), b, &pt[p]));
            CHECK(cubit_table_add_column(pt[p], 0, CUBIT_TYPE_INT32, shipdate + b, NULL, 0));
            CHECK(cubit_table_add_column(pt[p], 1, CUBIT_TYPE_INT64, discount + b, NULL, 0));
            CHECK(cubit_table_add_column(pt[p], 2, CUBIT_TYPE_INT64, quantity + b, NULL, 0));
            CHECK(cubit_table_add_column(pt[p], 3, CUBIT_TYPE_INT64, extprice + b, NULL, 0));
            CHECK(cubit_table_build_index(pt[p], 0, CUBIT_INDEX_RANGE, edges, (uint32_t)ne));
            CHECK(cubit_table_build_index(pt[p], 1, CUBIT_INDEX_RANGE, NULL, 0));
            CHECK(cubit_table_build_index(pt[p], 2, CUBIT_INDEX_RANGE, NULL, 0));
        }
        for (int d = 0; d < n_ctx; ++d) CHECK(cubit_sync(pctx[d]));
        double init_ms = 0, split[2] = {0, 0}, median_ms = 0;
        const double best = run_pipeline(pt, (uint32_t)n_partitions, q6, nn, threads, q, rev, &init_ms, split, &median_ms);
        printf("partitioned_pipeline partitions %d devices %d threads %d init_global_ms %.3f total_ms %.3f rows %" PRIu64
               " rows_per_s %.4e revenue_match 1 task_scan_ms %.3f task_aggregate_ms %.3f median_ms %.3f\n",
               n_partitions, n_ctx, threads, init_ms, best * 1e3, q, q / best, split[0], split[1], median_ms);
        CHECK_SCAN(cubit_scan_release_cached(NULL, NULL));
        for (int p = 0; p < n_partitions; ++p) CHECK(cubit_table_destroy(pt[p]));
        for (int d = 0; d < n_ctx; ++d) CHECK(cubit_ctx_destroy(pctx[d]));
        free(pt);
        free(pctx);
    }
    CHECK(cubit_dev_free(ctx, d_ids));
    CHECK(cubit_dev_free(ctx, d_cnt));
    CHECK(cubit_dev_free(ctx, d_sum));
    CHECK(cubit_table_destroy(t));
    CHECK(cubit_ctx_destroy(ctx));
    free(cols[0]);
    free(cols[1]);
    free(ids);
    free(shipdate);
    free(discount);
    free(quantity);
    free(extprice);
    return 0;
}
