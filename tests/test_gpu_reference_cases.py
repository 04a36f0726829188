"""The reference's own SQL test cases (tests/golden/reference_cases.json, each citing its
.test file) through the C ABI on the GPU, with and without bitmap indexes."""
import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from cubit_amd.scan_function import ROW_ID, CubitScanFunction
from cubit_amd.table import Context, CubitTable
from test_oracle_tpch import (art_appended_cases, art_scan_cases, block_boundary_states, filter_cache_filters, filter_cache_table,
                              filter_pushdown_tables, many_updaters_reads, multi_version_views,
                              obsolete_filter_columns, obsolete_filter_sets, residual_from_json, timestamp_filter_sets,
                              timestamp_table, update_case_views, zonemap_table)

pytestmark = pytest.mark.gpu

TXN_START = 4611686018427388000


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_zonemap_segment(ctx, golden, encoding):
    c = golden["cases"]["zonemap_segment"]
    data = np.repeat(np.array(c["values"], dtype=np.int32), c["block_rows"])
    t = CubitTable(ctx, len(data))
    t.add_column(0, data)
    if encoding is not None:
        t.build_index(0, encoding)
    for k, want in c["expected_sum_eq"].items():
        rows = t.scan(F.TableFilterSet({0: F.ConstantFilter("=", int(k))}))
        got = int(data[rows].astype(np.int64).sum()) if len(rows) else None
        assert got == want, k


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_timestamp_date_pushdown(ctx, golden, encoding):
    """timestamp_to_date_pushdown.test: a TIMESTAMP column (int64 microseconds) filtered by the
    day range DuckDB pushes for ts::date = d, beside a bound on i; the file's counts, with the
    timestamp column unindexed, range- or equality-indexed."""
    c = golden["cases"]["timestamp_date_pushdown"]
    ts, i, us = timestamp_table(c)
    t = CubitTable(ctx, len(ts))
    t.add_column(0, ts)
    t.add_column(1, i)
    if encoding is not None:
        t.build_index(0, encoding)
    for fs, want in timestamp_filter_sets(c, us):
        assert len(t.scan(fs)) == want and t.count(fs) == want
    t.close()


def test_interleaved_versions(ctx, golden):
    data = np.array([1, 2], dtype=np.int32)
    t1, t2 = TXN_START + 10, TXN_START + 11
    t = CubitTable(ctx, 2)
    t.add_column(0, data)
    exp = golden["cases"]["interleaved_versions"]["steps"]

    def s(start, tid):
        r = t.scan(F.TableFilterSet(), txn=L.Txn(start, tid))
        return int(data[r].sum()) if len(r) else None

    t.set_deletes(np.array([0, 1]), np.array([t1, t2], dtype=np.uint64))
    assert s(5, t1) == exp[0]["expect"]["con1"]
    assert s(5, t2) == exp[0]["expect"]["con2"]
    assert s(5, TXN_START + 12) == exp[0]["expect"]["con3"]
    t.set_deletes(np.array([0, 1]), np.array([6, t2], dtype=np.uint64))  # con1 committed at 6
    assert s(5, t2) == exp[1]["expect"]["con2"]
    assert s(7, TXN_START + 13) == 2


@pytest.mark.parametrize("index", [False, True])
def test_table_or_pushdown(ctx, golden, index):
    c = golden["cases"]["table_or_pushdown"]
    data = np.array(c["rows"], dtype=np.int32)
    t = CubitTable(ctx, len(data))
    t.add_column(0, data)
    t.add_column(1, data.copy())
    if index:
        t.build_index(0, L.INDEX_RANGE)
        t.build_index(1, L.INDEX_EQUALITY)
    for q in c["queries"]:
        rows = t.scan(None, residual_from_json(q["tree"]))
        assert data[rows].tolist() == q["expect"], q["sql"]


def select_all(t, fs, txn, col=0):
    """SELECT col FROM t WHERE … through the cubit_scan table-function callbacks."""
    fn = CubitScanFunction(t, [col], None, fs, txn=txn)
    local = fn.init_local()
    out = []
    while True:
        chunk = fn.function(local)[0]
        if len(chunk) == 0:
            return out
        out += chunk.tolist()


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_update(ctx, golden, encoding):
    """test/sql/update/test_update.test through the table function; after the rollback the
    committed update is merged into the base and the index, and every view stays the same."""
    data = np.array(golden["cases"]["update"]["rows"], dtype=np.int32)
    t = CubitTable(ctx, len(data))
    t.add_column(0, data)
    if encoding is not None:
        t.build_index(0, encoding)
    for step, upd, conns in update_case_views(golden):
        t.set_updates(0, *upd)
        for merged in ([False, True] if step is golden["cases"]["update"]["steps"][-1] else [False]):
            if merged:
                assert t.merge_updates(0, 8) == 1
            for con, eq, expect in step["checks"]:
                fs = F.TableFilterSet({0: F.ConstantFilter("=", eq)}) if eq is not None else F.TableFilterSet()
                assert select_all(t, fs, L.Txn(*conns[con])) == expect, (step["do"], con, eq, merged)
    t.close()


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE])
def test_multi_version(ctx, golden, encoding):
    """test/sql/transactions/test_multi_version.test through the table function: con1's
    update, second update, delete and insert (rows appended with its transaction id) are seen
    by con1 alone until COMMIT re-stamps them with commit id 6; con2's later snapshot sees all."""
    t = CubitTable(ctx, 3)
    t.add_column(0, np.array([1, 2, 3], dtype=np.int32))
    if encoding is not None:
        t.build_index(0, encoding)
    appended = False
    for step, upd, deleted, (ins, ins_id), conns in multi_version_views(golden):
        t.set_updates(0, *upd)
        drows = [r for r, d in enumerate(deleted) if d != 2 ** 64 - 2]
        t.set_deletes(np.array(drows, np.int64), np.array([deleted[r] for r in drows], np.uint64))
        if ins and not appended:
            t.append({0: np.array(ins, dtype=np.int32)}, insert_id=ins_id)
            appended = True
        elif ins:
            t.set_inserts(np.array([3]), np.array([3 + len(ins)]), np.array([ins_id], np.uint64))
        for con, want in step["expect"].items():
            got = select_all(t, F.TableFilterSet(), L.Txn(*conns[con]))
            assert sum(got) == want, (step["do"], con, got)
    t.close()


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_many_updaters(ctx, golden, encoding):
    """test/sql/update/test_update_many_updaters.test through the table function: all 26
    views (SELECT * ORDER BY a) of four snapshots, the writer and the committed state, and the
    same views under a pushed filter a >= 4 (the patched index leaves when indexed)."""
    c = golden["cases"]["many_updaters"]
    t = CubitTable(ctx, 3)
    t.add_column(0, np.array(c["rows"], dtype=np.int32))
    if encoding is not None:
        t.build_index(0, encoding)
    ge4 = F.TableFilterSet({0: F.ConstantFilter(">=", 4)})
    reads = list(many_updaters_reads(golden))
    assert [r[0] for r in reads] == [v[0] for v in c["views"]]
    for (con, snap, upd), (_, want) in zip(reads, c["views"]):
        t.set_updates(0, *upd)
        txn = L.Txn(*snap)
        assert sorted(select_all(t, F.TableFilterSet(), txn)) == want, (con, snap)
        assert sorted(select_all(t, ge4, txn)) == [v for v in want if v >= 4], (con, snap)
    t.close()


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_art_scans(ctx, golden, encoding):
    """The reference's ART scan tests (test_art_negative_range_scan, test_art_many_matches) on
    the index variant: the bitmap index in place of the ART (or no index), sums through the
    table function and counts through the count kernel equal the files'."""
    for v, queries in art_scan_cases(golden):
        t = CubitTable(ctx, len(v))
        t.add_column(0, v)
        if encoding is not None:
            t.build_index(0, encoding)
        for fs, kind, want in queries:
            if kind == "sum":
                assert sum(select_all(t, fs, None)) == want, (encoding, want)
            else:
                assert t.count(fs) == want and len(t.scan(fs)) == want, (encoding, want)
        t.close()


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_obsolete_filters(ctx, golden, encoding):
    """test/sql/filter/test_obsolete_filters.test's 33 integer queries through the table
    function: AND chains on nullable a (redundant, subsumed, contradictory) return the file's
    (a, b) rows, with a unindexed or indexed."""
    (a, av), (b, bv) = obsolete_filter_columns(golden)
    t = CubitTable(ctx, len(a))
    t.add_column(0, a, validity=validity_from_mask(av))
    t.add_column(1, b, validity=validity_from_mask(bv))
    if encoding is not None:
        t.build_index(0, encoding)
    for where, fs, want in obsolete_filter_sets(golden):
        rows = t.scan(fs)
        got = sorted((int(a[r]) if av[r] else None, int(b[r]) if bv[r] else None) for r in rows)
        assert got == want, (where, encoding)
        fn = CubitScanFunction(t, [0, 1], None, fs)
        local = fn.init_local()
        seen = []
        while True:
            chunk = fn.function(local)
            if len(chunk[0]) == 0:
                break
            seen += list(zip(chunk[0].tolist(), chunk[1].tolist()))
        assert len(seen) == len(want), (where, encoding)
    t.close()


@pytest.mark.parametrize("a_index", [False, True])
def test_zonemap_or_trees(ctx, golden, a_index):
    """test/sql/filter/test_zonemap.test_slow on the GPU at its full 1e8 rows: count(*) of the
    cross-column OR trees (residual filters) equals the file's counts — with a unindexed (K0 over
    the BIGINT column) or range-indexed at the trees' constants, b range-indexed; the row ids of
    the selective trees equal numpy's."""
    c = golden["cases"]["zonemap_or_trees"]
    a, b = zonemap_table(c["rows"])
    t = CubitTable(ctx, c["rows"])
    t.add_column(0, a)
    t.add_column(1, b)
    t.build_index(1, L.INDEX_RANGE)
    if a_index:
        t.build_index(0, L.INDEX_RANGE, [301, 401, 501, 601, 701, 7001])
    for q in c["queries"]:
        res = residual_from_json(q["tree"])
        assert t.count(None, res) == q["count"], (q["sql"], a_index)
        if q["count"] < 1000:
            mask = np.zeros(len(a), bool)
            if q["count"] == 499:
                mask = ((a > 500) & (b == 3)) | ((a > 7000) & (b == 2))
            else:
                mask = ((a > 500) & (b == 1)) | (b < 2)
            assert np.array_equal(t.scan(None, res, capacity=1024), np.flatnonzero(mask)), q["sql"]
    t.close()


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_filter_cache(ctx, golden, encoding):
    """test/sql/filter/filter_cache.test: the nested subqueries' filters as one scan (comparisons
    pushed, the OR of ranges as a residual) — count(*) equals the file's, through the count
    kernel and the table function, and the rows equal numpy's."""
    a = filter_cache_table(golden)
    t = CubitTable(ctx, len(a))
    t.add_column(0, a)
    if encoding is not None:
        t.build_index(0, encoding)
    for q in golden["cases"]["filter_cache"]["queries"]:
        fs, res = filter_cache_filters(q)
        assert t.count(fs, res) == q["count"], (q["sql"], encoding)
        fn = CubitScanFunction(t, [0, ROW_ID], None, fs, res)
        local = fn.init_local()
        got = []
        while True:
            cols = fn.function(local)
            if len(cols[0]) == 0:
                break
            got += cols[1].tolist()
        fn.close()
        mask = a < 5
        if q["tree"]:
            mask &= ((a > 1) & (a < 10) | (a > 9995)) if q["count"] == 30 else ((a != 3) & (a < 50) | (a > 9995)) & (a > 1) & (a < 20)
        assert sorted(got) == np.flatnonzero(mask).tolist(), (q["sql"], encoding)
    t.close()


@pytest.mark.parametrize("encoding", [L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_art_scans_over_appended_rows(ctx, golden, encoding):
    """test_art_range_scan.test's integer parts: an indexed USMALLINT key column created empty (the
    PRIMARY KEY's index exists before any row), rows appended (cubit_table_append maintains the
    index: new keys, values above the old range), each query's rows as the file has them; and
    test_art_adaptive_scan.test: 2,050 rows of 42 and 5,000 others, indexed after, COUNT = 2050."""
    for source, dtype, steps in art_appended_cases(golden):
        t = CubitTable(ctx, 0)
        t.add_column(0, np.empty(0, np.dtype(dtype)))
        if "adaptive" not in source:
            t.build_index(0, encoding)  # the index exists before the rows
        v = np.zeros(0, np.int64)
        for add, fs, count, rows in steps:
            t.append({0: add.astype(np.int32)})
            v = np.concatenate([v, add])
            if "adaptive" in source:
                t.build_index(0, encoding)  # CREATE INDEX after the inserts
            got = t.scan(fs)
            assert np.array_equal(got, np.flatnonzero(fs_mask(fs, v))), (source, encoding)
            if count is not None:
                assert t.count(fs) == count, (source, encoding)
            else:
                assert v[got].tolist() == rows, (source, encoding)
        t.close()


def fs_mask(fs, v):
    (flt,) = fs.filters.values()
    return {">": v > flt.constant, "=": v == flt.constant}[flt.comparison]


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE])
def test_block_boundary_update(ctx, golden, encoding):
    """block_boundary_update.test_slow through the table function: COUNT(i), SUM(i) after
    whole-table updates (every vector and row-group boundary of 50,000 / 100,000 rows) and an
    INSERT … SELECT of the table into itself (appended with its commit id), then the same after
    the update chains are merged into the base and the index; a filter i < 1000 on the
    (patched) index counts the rows the reference's values give."""
    c = golden["cases"]["block_boundary_update"]
    t = CubitTable(ctx, c["rows"])
    t.add_column(0, np.arange(c["rows"], dtype=np.int64))
    if encoding is not None:
        t.build_index(0, encoding)
    lt = F.TableFilterSet({0: F.ConstantFilter("<", 1000)})
    cur = np.arange(c["rows"], dtype=np.int64)
    for st, appended, upd, ins, start, want in block_boundary_states(golden):
        if appended is not None:
            t.append({0: appended}, insert_id=start - 1)
            cur = np.concatenate([cur, cur])
        elif st == "update":
            cur = cur + 1
        t.set_updates(0, *upd)
        txn = L.Txn(start, 4611686018427388000 + 60)
        got = select_all(t, F.TableFilterSet(), txn)
        assert (len(got), sum(got)) == want, st
        assert t.count(lt, txn=txn) == int((cur < 1000).sum()), st
    assert t.merge_updates(0, 2 ** 62) == len(cur)
    got = select_all(t, F.TableFilterSet(), L.Txn(100, 4611686018427388000 + 61))
    assert (len(got), sum(got)) == tuple(c["count_sum"][-1])
    assert t.count(lt) == int((cur < 1000).sum())
    t.close()


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE])
def test_concurrent_reads_while_updating(ctx, golden, encoding):
    """concurrent_reads_while_updating.test_slow on one context: one thread commits the 20
    UPDATE i=i+1 (each adds 10,000 update records stamped with its commit id) while 19 threads
    take snapshots and read — SELECT i through the table function, and count(*) WHERE i < 5000
    through the (patched) index. Every snapshot is whole: after k commits it sees 10,000 rows
    summing to 49,995,000 + 10,000·k and 5,000 - k rows below 5,000 — never a torn state. Then
    the update chains are merged and the final 10,000 / 50,195,000 read back."""
    import threading

    c = golden["cases"]["concurrent_reads_while_updating"]
    n, n_upd, lo, hi = c["rows"], c["updates"], c["reader_sum_range"][0], c["reader_sum_range"][1]
    t = CubitTable(ctx, n)
    t.add_column(0, np.arange(n, dtype=np.int32))
    if encoding is not None:
        t.build_index(0, encoding)
    lock = threading.Lock()
    state = {"k": 0}
    errors, seen = [], set()
    lt5000 = F.TableFilterSet({0: F.ConstantFilter("<", 5000)})

    def updater():
        try:
            for k in range(1, n_upd + 1):
                rows = np.tile(np.arange(n, dtype=np.int64), k)
                vals = np.concatenate([np.arange(n, dtype=np.int64) + j for j in range(1, k + 1)])
                vers = np.repeat(np.arange(1, k + 1, dtype=np.uint64) * 10, n)
                o = np.argsort(rows, kind="stable")  # each row's records in commit order
                t.set_updates(0, rows[o], vals[o], vers[o])
                with lock:
                    state["k"] = k  # committed: snapshots from now on start after 10·k
        except Exception as e:
            errors.append(repr(e))

    def reader(tid):
        try:
            for _ in range(10):
                with lock:
                    k = state["k"]
                txn = L.Txn(10 * k + 1, 4611686018427388000 + 1000 + tid)
                got = select_all(t, F.TableFilterSet(), txn)
                total = sum(got)
                if len(got) != c["reader_count"] or not lo <= total <= hi or total != lo + n * k:
                    errors.append(f"reader {tid}: k={k} rows={len(got)} sum={total}")
                cnt = t.count(lt5000, txn=txn)
                if cnt != 5000 - k:
                    errors.append(f"reader {tid}: k={k} count(i<5000)={cnt}")
                seen.add(k)
        except Exception as e:
            errors.append(repr(e))

    th = [threading.Thread(target=updater)] + [threading.Thread(target=reader, args=(i,))
                                               for i in range(1, c["threads"])]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:3]
    assert t.merge_updates(0, 10 * n_upd + 1) == n
    final = select_all(t, F.TableFilterSet(), L.Txn(10 * n_upd + 2, 4611686018427388000 + 5000))
    assert (len(final), sum(final)) == (c["final"]["count"], c["final"]["sum"])
    assert t.count(lt5000) == 5000 - n_upd
    t.close()


@pytest.mark.parametrize("index", [False, True])
def test_table_filter_pushdown(ctx, golden, index):
    """test/optimizer/pushdown/table_filter_pushdown.test: the filters it expects pushed into
    the scan, over every integer-backed type the shim attaches, with NULLs."""
    for name, cols, queries in filter_pushdown_tables(golden):
        n = len(cols[0][0])
        t = CubitTable(ctx, n)
        for j, (v, m) in enumerate(cols):
            t.add_column(j, v, validity_from_mask(m) if m is not None else None)
            if index:
                t.build_index(j, L.INDEX_RANGE)
        for fs, out_col, expect in queries:
            rows = t.scan(fs)
            if out_col is None:
                assert len(rows) == expect, name
                assert t.count(fs) == expect, name
            else:
                assert cols[out_col][0][rows].tolist() == expect, name
        t.close()


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_transitive_filters_through_table_function(ctx, golden, encoding):
    """test_transitive_filters.test's 40 one-table queries: the constant comparison on i pushed
    into cubit_scan (plain, range- or equality-indexed i), i and j probed through the table
    function, and the j-to-i comparison DuckDB evaluates above the scan applied to the chunks:
    the file's rows in its order."""
    from test_oracle_filters import transitive_filter_cases

    i, j, cases = transitive_filter_cases(golden)
    t = CubitTable(ctx, len(i))
    t.add_column(0, i)
    t.add_column(1, j)
    if encoding is not None:
        t.build_index(0, encoding)
    for fs, residual, want, where in cases:
        fn = CubitScanFunction(t, [0, 1, 2 ** 64 - 1], None, fs)
        local = fn.init_local()
        got = []
        while True:
            cols = fn.function(local)
            if len(cols[0]) == 0:
                break
            got += [[int(a), int(b), int(r)] for a, b, r in zip(*cols)]
        fn.close()
        got.sort(key=lambda x: x[2])  # batch order = row order
        assert [[a, b] for a, b, _ in got if residual(b, a)] == want, (where, encoding)
    t.close()
