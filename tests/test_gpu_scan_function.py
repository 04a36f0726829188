"""The TableFunction mirror (include/cubit_scan.h) driven the way DuckDB's pipeline drives
seq_scan: N tasks with their own local state call `function` until it returns an empty
chunk (PhysicalTableScan::GetData, physical_table_scan.cpp:82-103); an order-preserving sink
sorts chunks by batch index (table_scan.cpp:179-189).

Every test runs twice: with the partition's rows staged to the host by init_global on one copy
stream in groups (the default), and with CUBIT_SCAN_STAGE_MB=0, where each task copies the window it
claims."""
import os
import threading

import numpy as np
import pytest

from conftest import lineitem, revenue_from_answer
from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.scan_function import ROW_ID, CubitScanFunction
from cubit_amd.table import Context, CubitTable
from oracle import oracle as O

pytestmark = pytest.mark.gpu

TXN_START = 4611686018427388000


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


@pytest.fixture(autouse=True, params=["staged", "per_window"])
def staging(request):
    old = os.environ.get("CUBIT_SCAN_STAGE_MB")
    if request.param == "per_window":
        os.environ["CUBIT_SCAN_STAGE_MB"] = "0"
    else:
        os.environ.pop("CUBIT_SCAN_STAGE_MB", None)
    yield request.param
    if old is None:
        os.environ.pop("CUBIT_SCAN_STAGE_MB", None)
    else:
        os.environ["CUBIT_SCAN_STAGE_MB"] = old


def q6_table(ctx, li):
    t = CubitTable(ctx, li.n_rows, li.row_base)
    for c, arr in enumerate((li.l_shipdate, li.l_discount, li.l_quantity, li.l_extendedprice)):
        t.add_column(c, arr)
    months = [F.date(y, m, 1) for y in range(1992, 1999) for m in range(1, 13)] + [F.date(1999, 1, 1)]
    t.build_index(0, L.INDEX_RANGE, months)
    t.build_index(1, L.INDEX_RANGE)
    t.build_index(2, L.INDEX_RANGE)
    return t


def drain(fn, n_tasks, validity=False):
    """Run n_tasks pipeline tasks; returns [(batch_index, chunk columns)] — with validity=True
    each column's bool mask follows the value columns (cubit_scan_function_validity)."""
    out, lock = [], threading.Lock()

    def task():
        local = fn.init_local()
        while True:
            if validity:
                vals, masks = fn.function_validity(local)
                cols = vals + masks
            else:
                cols = fn.function(local)
            if len(cols[0]) == 0:
                return
            assert len(cols[0]) <= 2048
            b = fn.get_batch_index(local)
            with lock:
                out.append((b, cols))

    th = [threading.Thread(target=task) for _ in range(n_tasks)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    return out


def assert_window_batches(chunks, tile_of):
    """Batch index = the first tile of the chunk's window (one batch per window, a morsel): every
    chunk's rows lie in tiles >= its batch index and below the next batch index present, and
    chunks are full — at most one chunk per batch holds fewer than 2,048 rows."""
    bs = sorted({b for b, _ in chunks})
    nxt = {b: (bs[i + 1] if i + 1 < len(bs) else np.iinfo(np.int64).max) for i, b in enumerate(bs)}
    short = {}
    for b, cols in chunks:
        t = tile_of(cols[0])
        assert np.all(t >= b) and np.all(t < nxt[b]), b
        short[b] = short.get(b, 0) + (len(cols[0]) < 2048)
    assert max(short.values(), default=0) <= 1


def ordered(chunks, col):
    chunks = sorted(chunks, key=lambda bc: (bc[0], bc[1][0][0] if len(bc[1][0]) else 0))
    return np.concatenate([c[col] for _, c in chunks]) if chunks else np.empty(0, np.int64)


@pytest.mark.parametrize("tasks", [1, 4])
def test_q6_through_table_function(ctx, golden, tasks):
    li = lineitem(0.1)
    t = q6_table(ctx, li)
    # SELECT rowid, l_extendedprice, l_discount ... WHERE <Q6>: column_ids include the filter
    # columns, projection_ids drop them (filter_prune)
    column_ids = [0, 1, 2, 3, ROW_ID]
    projection_ids = [4, 3, 1]
    fn = CubitScanFunction(t, column_ids, projection_ids, F.q6_filter_set(0, 1, 2))
    assert fn.max_threads() >= 1
    chunks = drain(fn, tasks)
    rows = ordered(chunks, 0)
    ref = O.table_scan([O.Column(li.l_shipdate), O.Column(li.l_discount), O.Column(li.l_quantity)],
                       F.serialize(F.q6_filter_set()), li.n_rows)
    assert np.array_equal(rows, ref)
    assert np.array_equal(ordered(chunks, 1), li.l_extendedprice[ref])
    assert np.array_equal(ordered(chunks, 2), li.l_discount[ref])
    rev = int((ordered(chunks, 1).astype(object) * ordered(chunks, 2).astype(object)).sum())
    assert rev == revenue_from_answer(golden["tpch"]["q6_revenue"]["0.1"]["revenue"])
    assert fn.progress() == pytest.approx(100.0)
    assert_window_batches(chunks, lambda ids: ids // 131072)


@pytest.mark.parametrize("tasks", [1, 4])
def test_non_selective_filter_decodes_once(ctx, tasks):
    """init_global sizes its row-id buffer from the planner's estimate
    (cubit_table_estimate_rows), so a filter keeping half the rows decodes once instead of
    overflowing the old n/8 guess and decoding again; rows and probed values equal the oracle's.
    A filter the estimate gets wrong (three copies of one column: independence predicts 1/8,
    the filter keeps 1/2) still returns the oracle's rows, by the second pass."""
    rng = np.random.default_rng(17)
    n = 1_000_003
    a = rng.integers(0, 1000, n).astype(np.int64)
    b = rng.integers(-50, 50, n).astype(np.int32)
    t = CubitTable(ctx, n, row_base=11)
    t.add_column(0, a)
    t.add_column(1, b)
    t.add_column(2, a.copy())
    t.build_index(0, L.INDEX_RANGE, [250, 500, 750])
    fs = F.TableFilterSet({0: F.ConstantFilter("<", 500)})
    est = t.estimate_rows(fs)
    assert abs(est - n // 2) < n // 20
    fn = CubitScanFunction(t, [0, 1, ROW_ID], [2, 1], fs)
    chunks = drain(fn, tasks)
    assert fn.decodes() == 1
    ref = O.table_scan([O.Column(a), O.Column(b)], F.serialize(fs), n, row_base=11)
    assert len(ref) > n // 3
    assert np.array_equal(ordered(chunks, 0), ref)
    assert np.array_equal(ordered(chunks, 1), b[ref - 11])
    # correlated columns: three copies of a, each < 500, keep 1/2 while independence predicts
    # 1/8 — the capacity (max(n/8, 2 · n/8)) falls short and the second pass returns the rows
    t.add_column(3, a.copy())
    fs3 = F.TableFilterSet({0: F.ConstantFilter("<", 500), 2: F.ConstantFilter("<", 500),
                            3: F.ConstantFilter("<", 500)})
    fn3 = CubitScanFunction(t, [0, 2, 3, ROW_ID], [3], fs3)
    rows3 = ordered(drain(fn3, tasks), 0)
    assert fn3.decodes() == 2
    ref3 = np.flatnonzero(a < 500) + 11
    assert np.array_equal(rows3, ref3)
    fn.close()
    fn3.close()
    t.close()


def test_estimate_rows_shapes(ctx):
    """cubit_table_estimate_rows over the filter shapes the scan takes: constants on one column
    folded into one interval, OR, IS NULL / IS NOT NULL, an empty interval, no filter."""
    from cubit_amd.datagen import validity_from_mask

    n = 262_144 * 4
    v = np.arange(n, dtype=np.int64) % 1000
    ok = np.ones(n, dtype=bool)
    ok[: 131_072] = np.arange(131_072) % 2 == 0  # NULLs in the first zone only
    t = CubitTable(ctx, n)
    t.add_column(0, v, validity_from_mask(ok))
    near = lambda got, want: abs(got - want) <= 0.02 * n  # noqa: E731
    assert t.estimate_rows(None) == n
    assert near(t.estimate_rows(F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", 100),
                                                                                 F.ConstantFilter("<", 300)])})),
                n * 0.2)
    assert t.estimate_rows(F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", 300),
                                                                          F.ConstantFilter("<", 100)])})) == 0
    assert near(t.estimate_rows(F.TableFilterSet({0: F.ConjunctionOrFilter([F.ConstantFilter("<", 100),
                                                                             F.ConstantFilter(">=", 900)])})),
                n * 0.19)
    assert near(t.estimate_rows(F.TableFilterSet({0: F.ConstantFilter("!=", 5)})), n)
    assert t.estimate_rows(F.TableFilterSet({0: F.IsNullFilter()})) == 131_072  # the zones holding a NULL
    assert t.estimate_rows(F.TableFilterSet({0: F.IsNotNullFilter()})) == n
    with pytest.raises(L.CubitError):
        t.estimate_rows(F.TableFilterSet({5: F.ConstantFilter("<", 1)}))
    t.close()


def test_no_filter_full_scan_and_empty_result(ctx):
    n = 300_000
    a = np.arange(n, dtype=np.int64) % 1000
    t = CubitTable(ctx, n, row_base=7)
    t.add_column(0, a)
    fn = CubitScanFunction(t, [ROW_ID, 0])
    chunks = drain(fn, 3)
    assert np.array_equal(ordered(chunks, 0), np.arange(n) + 7)
    assert np.array_equal(ordered(chunks, 1), a)
    fn2 = CubitScanFunction(t, [0], None, F.TableFilterSet({0: F.ConstantFilter(">", 5000)}))
    local = fn2.init_local()
    assert len(fn2.function(local)[0]) == 0
    assert fn2.progress() == 100.0


def test_mvcc_views_through_table_function(ctx, golden):
    li = lineitem(0.01)
    t = q6_table(ctx, li)
    n = li.n_rows
    writer = TXN_START + 1
    t.set_deletes(np.arange(0, n, 11), np.full(len(range(0, n, 11)), writer, dtype=np.uint64))
    upd = np.arange(0, n, 7)
    t.set_updates(2, upd, np.full(len(upd), 100), np.full(len(upd), writer, dtype=np.uint64))
    fp = golden["tpch"]["fingerprints"]["sf001_mvcc"]
    for txn, want in ((L.Txn(2, writer), fp["writer_view"]), (L.Txn(2, TXN_START + 2), fp["reader_view"])):
        fn = CubitScanFunction(t, [0, 1, 2, ROW_ID], [3, 2], F.q6_filter_set(), txn=txn)
        chunks = drain(fn, 2)
        assert len(ordered(chunks, 0)) == want
        # the probed l_quantity is the version the transaction sees
        q = ordered(chunks, 1)
        rows = ordered(chunks, 0)
        exp = li.l_quantity[rows].copy()
        if txn.transaction_id == writer:
            exp[rows % 7 == 0] = 100
        assert np.array_equal(q, exp)


def test_cardinality_and_statistics_callbacks(ctx):
    """seq_scan's bind-time callbacks: TableScanCardinality (table_scan.cpp:201-208) and
    TableScanStatistics (table_scan.cpp:108-117 → DataTable::GetStatistics): min / max of the
    valid values widened by update records, has_null / has_no_null, none for the row id."""
    from cubit_amd import scan_function as S
    from cubit_amd.datagen import validity_from_mask

    rng = np.random.default_rng(8)
    n = 700_001
    a = rng.integers(-1000, 1000, n).astype(np.int32)
    b = rng.integers(0, 2 ** 40, n).astype(np.int64)
    valid_b = rng.random(n) > 0.2
    c = np.zeros(n, dtype=np.int64)
    t = CubitTable(ctx, n, row_base=5)
    t.add_column(0, a)
    t.add_column(1, b, validity_from_mask(valid_b))
    t.add_column(2, c, validity_from_mask(np.zeros(n, dtype=bool)))  # every row NULL
    assert S.cardinality(t) == (n, n)
    assert S.statistics(t, S.ROW_ID) is None
    assert S.statistics(t, 0) == (int(a.min()), int(a.max()), False, True)
    assert S.statistics(t, 1) == (int(b[valid_b].min()), int(b[valid_b].max()), True, True)
    assert S.statistics(t, 2) == (0, 0, True, False)
    assert t.column_statistics(0) == S.statistics(t, 0)
    # update records widen the bounds (any version, as UpdateSegment merges its statistics)
    t.set_updates(0, np.array([3, 9], dtype=np.int64), np.array([-5000, 7000], dtype=np.int64),
                  np.array([2, TXN_START + 1], dtype=np.uint64))
    assert S.statistics(t, 0) == (-5000, 7000, False, True)
    # appends change the statistics (the cached zone statistics are dropped)
    t.append({0: np.array([-9999], dtype=np.int32), 1: np.array([1], dtype=np.int64),
              2: np.array([42], dtype=np.int64)}, validity={2: np.array([1], dtype=np.uint64)})
    assert S.statistics(t, 0) == (-9999, 7000, False, True)
    assert S.statistics(t, 2) == (42, 42, True, True)
    assert S.cardinality(t) == (n + 1, n + 1)
    t.close()
    empty = CubitTable(ctx, 0)
    empty.add_column(0, np.empty(0, dtype=np.int64))
    assert S.statistics(empty, 0) == (0, 0, False, False)
    assert S.cardinality(empty) == (0, 0)
    empty.close()


def test_windows_stream_in_batch_order_per_task(ctx):
    """A result of several copy windows (262,144 rows each) drained by 4 tasks: every task's
    batch indexes never decrease (PipelineExecutor::NextBatch refuses a lower one,
    pipeline_executor.cpp:132-136), every chunk's rows lie in its batch's window, and the rows
    equal numpy's predicate. The filter keeps half the rows: init_global's estimate sizes the
    decode for them (one pass)."""
    from cubit_amd import scan_function as S

    n = 3_000_017
    rng = np.random.default_rng(21)
    a = rng.integers(0, 1000, n).astype(np.int64)
    b = rng.integers(-50, 50, n).astype(np.int32)
    t = CubitTable(ctx, n, row_base=1_000)
    t.add_column(0, a)
    t.add_column(1, b)
    t.build_index(0, L.INDEX_RANGE)
    fs = F.TableFilterSet({0: F.ConstantFilter("<", 500)})
    fn = CubitScanFunction(t, [1, 0, ROW_ID], [2, 0], fs)
    assert fn.max_threads() >= 4
    per_task, lock = {}, threading.Lock()

    def task(k):
        local = fn.init_local()
        seen = []
        while True:
            cols = fn.function(local)
            if len(cols[0]) == 0:
                break
            seen.append((fn.get_batch_index(local), cols))
        with lock:
            per_task[k] = seen

    th = [threading.Thread(target=task, args=(k,)) for k in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    chunks = []
    for k, seen in per_task.items():
        idx = [bi for bi, _ in seen]
        assert idx == sorted(idx), k
        chunks += seen
    assert_window_batches(chunks, lambda ids: (ids - 1_000) // 131072)
    assert fn.decodes() == 1
    want = np.flatnonzero(a < 500)
    assert np.array_equal(ordered(chunks, 0), want + 1_000)
    assert np.array_equal(ordered(chunks, 1), b[want])
    assert fn.progress() == pytest.approx(100.0)
    fn.close()
    pinned, device = C_release()
    assert pinned > 0 and device > 0  # the finished scan's buffers were cached, now freed
    assert C_release() == (0, 0)
    t.close()


def C_release():
    import ctypes as C

    p, d = C.c_uint64(), C.c_uint64()
    L.check_scan(L.scan_lib().cubit_scan_release_cached(C.byref(p), C.byref(d)))
    return int(p.value), int(d.value)


def test_pinned_windows_are_reused_across_scans(ctx):
    """page-locked windows are filed under no context, and a later scan must find
    them there — two identical scans in a row leave as many pinned bytes cached as one scan
    (a pool that never hits pins fresh memory for the second scan and caches both)."""
    n = 2_000_003
    a = np.random.default_rng(5).integers(0, 1000, n).astype(np.int64)
    t = CubitTable(ctx, n)
    t.add_column(0, a)
    t.build_index(0, L.INDEX_RANGE)
    fs = F.TableFilterSet({0: F.ConstantFilter("<", 300)})

    def drain():
        fn = CubitScanFunction(t, [0, ROW_ID], [], fs)
        local = fn.init_local()
        rows = 0
        while True:
            cols = fn.function(local)
            if len(cols[0]) == 0:
                break
            rows += len(cols[0])
        fn.close()
        assert rows == int((a < 300).sum())

    C_release()
    drain()
    one, _ = C_release()
    drain()
    drain()
    two, _ = C_release()
    assert two == one > 0
    t.close()


def test_window_transfer_compaction_round_trips(ctx):
    """Windows cross PCIe as int32 (value - offset) where a column's statistics allow it
    (cubit_narrow_i32) and as int64 otherwise; either way the chunks carry the exact values:
    row ids of a partition based at 2^40, a DATE-like int32 column, a DECIMAL-like int64 column
    inside int32 range with negatives, one far outside it, and a column with NULL rows (probed with
    its validity: every row's value and NULL-ness equal the oracle's fetch, NULL rows as 0)."""
    from cubit_amd.datagen import validity_from_mask

    n = 1_500_007
    base = 1 << 40
    rng = np.random.default_rng(31)
    key = rng.integers(0, 100, n).astype(np.int32)
    small = rng.integers(-2_000_000, 2_000_000, n).astype(np.int64)
    big = rng.integers(-(1 << 50), 1 << 50, n).astype(np.int64)
    date = (8035 + rng.integers(0, 2526, n)).astype(np.int32)
    nulls = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
    valid = rng.random(n) > 0.05
    t = CubitTable(ctx, n, row_base=base)
    t.add_column(0, key)
    t.add_column(1, small)
    t.add_column(2, big)
    t.add_column(3, date)
    t.add_column(4, nulls, validity_from_mask(valid))
    t.build_index(0, L.INDEX_RANGE)
    fs = F.TableFilterSet({0: F.ConstantFilter("<", 30)})
    fn = CubitScanFunction(t, [ROW_ID, 1, 2, 3, 4, 0], [0, 1, 2, 3, 4], fs)
    chunks = drain(fn, 3, validity=True)
    fn.close()
    keep = np.flatnonzero(key < 30)
    assert np.array_equal(ordered(chunks, 0), keep.astype(np.int64) + base)
    assert np.array_equal(ordered(chunks, 1), small[keep])
    assert np.array_equal(ordered(chunks, 2), big[keep])
    assert np.array_equal(ordered(chunks, 3), date[keep].astype(np.int64))
    for c in range(4):
        assert ordered(chunks, 5 + c).all()  # columns without NULLs: every row valid
    ref_vals, ref_valid = O.fetch(O.Column(nulls, validity_from_mask(valid)), keep, with_valid=True)
    assert np.array_equal(ordered(chunks, 9), ref_valid)
    assert np.array_equal(ordered(chunks, 4), ref_vals)
    t.close()


@pytest.mark.parametrize("tasks", [1, 4])
def test_float_and_double_columns_through_table_function(ctx, tasks):
    """FLOAT / DOUBLE filter and projection columns (DuckDB's floating-point comparisons: NaN
    greatest and equal to NaN, -0.0 == +0.0): the filter on a DOUBLE column and on a FLOAT one
    equals the oracle's scan, and every projected row hands back the stored bit pattern (FLOAT
    crossing as 4 bytes, DOUBLE as 8; -0.0 and NaN payloads intact) with its NULL-ness."""
    from cubit_amd.datagen import validity_from_mask

    n = 900_001
    rng = np.random.default_rng(41)
    special = [0.0, -0.0, np.inf, -np.inf, np.nan, 1.5, -1.5]
    d = (rng.standard_normal(n) * 100).astype(np.float64)
    d[rng.integers(0, n, 5000)] = np.array(special)[rng.integers(0, len(special), 5000)]
    d[7] = np.array([0xFFF8000000000123], dtype=np.uint64).view(np.float64)[0]  # a negative NaN with payload
    f = (rng.standard_normal(n) * 10).astype(np.float32)
    f[rng.integers(0, n, 5000)] = np.array(special, dtype=np.float32)[rng.integers(0, len(special), 5000)]
    fvalid = rng.random(n) > 0.03
    t = CubitTable(ctx, n)
    t.add_column(0, d)
    t.add_column(1, f, validity_from_mask(fvalid))
    t.build_index(1, L.INDEX_RANGE, np.array([-10.0, -1.0, 0.0, 1.0, 10.0], dtype=np.float32))
    cols = [O.Column(d), O.Column(f, validity_from_mask(fvalid))]
    for fs in [F.TableFilterSet({0: F.ConstantFilter(">=", 150.0)}),
               F.TableFilterSet({0: F.ConstantFilter("=", np.nan)}),
               F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">", -5.0), F.ConstantFilter("<=", 5.0)]),
                                 1: F.ConstantFilter("!=", np.float32(-0.0))}),
               F.TableFilterSet({1: F.ConjunctionOrFilter([F.ConstantFilter("<", np.float32(-9.5)),
                                                           F.ConstantFilter("=", np.float32(0.0))])})]:
        keep = O.table_scan(cols, F.serialize(fs), n)
        fn = CubitScanFunction(t, [ROW_ID, 0, 1], [0, 1, 2], fs)
        chunks = drain(fn, tasks, validity=True)
        fn.close()
        assert np.array_equal(ordered(chunks, 0), keep)
        assert np.array_equal(ordered(chunks, 1), O.fetch(cols[0], keep))
        fv, fok = O.fetch(cols[1], keep, with_valid=True)
        assert np.array_equal(ordered(chunks, 2), fv)
        assert np.array_equal(ordered(chunks, 5), fok)
    t.close()


def test_compaction_overflow_falls_back_to_8_byte_values(ctx, monkeypatch):
    """The device checks the compaction bound as it narrows: with every compacted column's offset
    moved one above its minimum (CUBIT_SCAN_TEST_SHIFT_OFFSET), the groups (staged) or the
    partition (per window) holding a minimum are flagged and their windows cross as 8-byte values —
    the chunks still carry the exact values, row ids included."""
    from cubit_amd.datagen import validity_from_mask

    n = 2_000_003
    rng = np.random.default_rng(5)
    key = rng.integers(0, 100, n).astype(np.int32)
    price = rng.integers(90_000, 10_000_000, n).astype(np.int64)
    disc = rng.integers(0, 11, n).astype(np.int64)
    nul = rng.integers(-5, 5, n).astype(np.int64)
    ok = rng.random(n) > 0.1
    t = CubitTable(ctx, n, row_base=3)
    t.add_column(0, key)
    t.add_column(1, price)
    t.add_column(2, disc)
    t.add_column(3, nul, validity_from_mask(ok))
    t.build_index(0, L.INDEX_RANGE)
    monkeypatch.setenv("CUBIT_SCAN_TEST_SHIFT_OFFSET", "1")
    fs = F.TableFilterSet({0: F.ConstantFilter("<", 60)})
    fn = CubitScanFunction(t, [0, 1, 2, 3, ROW_ID], [4, 1, 2, 3], fs)  # row ids first: ordered() sorts by them
    chunks = drain(fn, 4, validity=True)
    fn.close()
    keep = np.flatnonzero(key < 60)
    assert np.array_equal(ordered(chunks, 0), keep.astype(np.int64) + 3)
    assert np.array_equal(ordered(chunks, 1), price[keep])
    assert np.array_equal(ordered(chunks, 2), disc[keep])
    ref_vals, ref_valid = O.fetch(O.Column(nul, validity_from_mask(ok)), keep, with_valid=True)
    assert np.array_equal(ordered(chunks, 7), ref_valid)
    assert np.array_equal(ordered(chunks, 3), ref_vals)
    t.close()


@pytest.mark.parametrize("tasks", [1, 4])
def test_nullable_projection_and_unpruned_is_null_filter(ctx, tasks):
    """SELECT b, c, rowid … WHERE a < k AND c IS NULL with c not pruned (DuckDB keeps a filter
    column that is also projected): b and c carry their validity through the chunks — c is NULL on
    every row, b on its own NULL rows, including rows whose NULL-ness an update record changed for
    this transaction (ColumnData::FilterScan + Slice, column_data.cpp:305-309)."""
    from cubit_amd.datagen import validity_from_mask

    n = 1_000_003
    rng = np.random.default_rng(77)
    a = rng.integers(0, 100, n).astype(np.int32)
    b = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
    bv = rng.random(n) > 0.3
    c = rng.integers(0, 5, n).astype(np.int32)
    cv = rng.random(n) > 0.5
    t = CubitTable(ctx, n, row_base=11)
    t.add_column(0, a)
    t.add_column(1, b, validity_from_mask(bv))
    t.add_column(2, c, validity_from_mask(cv))
    t.build_index(0, L.INDEX_RANGE)
    me = TXN_START + 3
    urows = np.sort(rng.choice(n, 4000, replace=False)).astype(np.int64)
    uvals = rng.integers(0, 1000, len(urows)).astype(np.int64)
    uok = rng.random(len(urows)) > 0.5
    t.set_updates(1, urows, uvals, np.full(len(urows), me, np.uint64), valid=uok)
    txn = L.Txn(2, me)
    fs = F.TableFilterSet({0: F.ConstantFilter("<", 40), 2: F.IsNullFilter()})
    fn = CubitScanFunction(t, [0, 1, 2, ROW_ID], [3, 1, 2], fs, txn=txn)
    chunks = drain(fn, tasks, validity=True)  # rowid, b, c, then their masks
    fn.close()
    keep = np.flatnonzero((a < 40) & ~cv)
    assert np.array_equal(ordered(chunks, 0), keep + 11)
    assert ordered(chunks, 3).all()
    tx = O.Mvcc(2, me)
    ocol_b = O.Column(b, validity_from_mask(bv), (urows, uvals, np.full(len(urows), me, np.uint64), uok))
    rv, rvalid = O.fetch(ocol_b, keep, tx=tx, with_valid=True)
    assert np.array_equal(ordered(chunks, 4), rvalid) and np.array_equal(ordered(chunks, 1), rv)
    assert not ordered(chunks, 5).any() and not ordered(chunks, 2).any()  # c IS NULL on every row
    assert (~rvalid).any() and rvalid.any() and len(keep) > 100_000
    t.close()


def test_scan_tiles_returns_this_scans_directory(ctx):
    """cubit_table_scan_tiles: the directory copied within the scan call equals the one
    cubit_ctx_last_tiles describes right after it, survives a later scan on the context, and a
    directory buffer too small is refused with CUBIT_ERR_CAPACITY."""
    import ctypes as C

    from cubit_amd.filters import serialize, to_ctypes

    rng = np.random.default_rng(5)
    n = 1_000_003
    v = rng.integers(0, 100, n, dtype=np.int32)
    t = CubitTable(ctx, n, row_base=4)
    t.add_column(0, v)
    t.build_index(0, L.INDEX_RANGE)

    def scan_tiles(lt, dir_cap):
        nodes = to_ctypes(serialize(F.TableFilterSet({0: F.ConstantFilter("<", lt)})).nodes)
        ids, cnt = ctx.alloc(n * 8), ctx.alloc(16)
        d = ctx.alloc(max(dir_cap, 1) * 16)
        nt, rpt = C.c_uint32(), C.c_uint64()
        rc = ctx.lib.cubit_table_scan_tiles(t.handle, nodes, len(nodes), None, C.c_void_p(ids.addr), n,
                                            C.c_void_p(cnt.addr), L.SCAN_ORDERED, C.c_void_p(d.addr), dir_cap,
                                            C.byref(nt), C.byref(rpt))
        return rc, ids, cnt, d, nt.value, rpt.value

    tiles = (n + 131071) // 131072
    rc, ids, cnt, d, nt, rpt = scan_tiles(7, tiles)
    assert rc == 0 and nt == tiles and rpt == 131072
    mine = d.download(np.uint64, 2 * nt).reshape(-1, 2)
    last, _ = ctx.last_tiles()
    assert np.array_equal(mine, np.asarray(last, dtype=np.uint64).reshape(-1, 2))
    k = int(cnt.download(np.uint64, 1)[0])
    ref = np.flatnonzero(v < 7).astype(np.int64) + 4
    assert np.array_equal(ids.download(np.int64, k), ref)
    assert int(mine[:, 1].sum()) == k
    scan_tiles(50, tiles)  # another scan on the context leaves the first copy alone
    assert np.array_equal(d.download(np.uint64, 2 * nt).reshape(-1, 2), mine)
    rc, *_ = scan_tiles(7, tiles - 1)
    assert rc == L.ERR_CAPACITY
    t.close()


def test_q6_over_an_empty_lineitem(ctx):
    """test/sql/tpch/tpch_sf0.test runs every TPC-H query over dbgen(sf=0): Q6's filter over an
    empty lineitem (indexes built on no rows) gives no rows through the scan, the count, the fused
    sum and the table function (one partition, and an empty partition beside a non-empty one)."""
    from cubit_amd import scan_function as S

    def q6_empty():
        t = CubitTable(ctx, 0)
        t.add_column(0, np.empty(0, np.int32))
        for c in (1, 2, 3):
            t.add_column(c, np.empty(0, np.int64))
        months = [F.date(y, m, 1) for y in range(1992, 1999) for m in range(1, 13)] + [F.date(1999, 1, 1)]
        t.build_index(0, L.INDEX_RANGE, months)
        t.build_index(1, L.INDEX_RANGE)
        t.build_index(2, L.INDEX_RANGE)
        return t

    t = q6_empty()
    fs = F.q6_filter_set()
    assert t.scan(fs).tolist() == [] and t.count(fs) == 0
    assert t.sum_product(3, 1, fs) == (0, 0)
    assert S.cardinality(t) == (0, 0)
    fn = CubitScanFunction(t, [0, 1, 2, 3, ROW_ID], [4, 3, 1], F.q6_filter_set(0, 1, 2))
    assert len(fn.function(fn.init_local())[0]) == 0
    assert fn.progress() == 100.0
    fn.close()
    # an empty partition in front of the SF0.01 lineitem: the cursor steps over it
    li = lineitem(0.01)
    full = CubitTable(ctx, li.n_rows, 0)
    for c, arr in enumerate((li.l_shipdate, li.l_discount, li.l_quantity, li.l_extendedprice)):
        full.add_column(c, arr)
    fn = CubitScanFunction([t, full], [0, 1, 2, 3, ROW_ID], [4], F.q6_filter_set(0, 1, 2))
    rows = ordered(drain(fn, 2), 0)
    fn.close()
    ref = O.table_scan([O.Column(li.l_shipdate), O.Column(li.l_discount), O.Column(li.l_quantity)],
                       F.serialize(F.q6_filter_set()), li.n_rows)
    assert np.array_equal(rows, ref) and len(rows) == 1191
    full.close()
    t.close()
