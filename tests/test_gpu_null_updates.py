"""NULL-ness through MVCC updates on the GPU: the reference's NULL-update tests
(tests/null_updates.py replays test_null_update.test, null_update_merge.test,
null_update_merge_transaction.test, test_update_many_updaters_nulls.test, update_null_integers.test)
answered through cubit_table_set_updates_nullable, the table function with validity
(cubit_scan_function_validity), pushed IS [NOT] NULL / comparison filters on patched leaves,
cubit_table_probe_validity and cubit_table_merge_updates — each against the file's rows and the
oracle (UpdateMergeValidity / FetchRowValidity restated in cpu_ref.c)."""
import numpy as np
import pytest

import null_updates as NU
from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from cubit_amd.scan_function import CubitScanFunction
from cubit_amd.table import Context, CubitTable
from oracle import oracle as O
from test_oracle_null_updates import CASES, oracle_columns, predicates

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def gpu_table(ctx, q: NU.Query, encoding):
    n = len(q.base[q.columns[0]])
    t = CubitTable(ctx, n)
    for j, c in enumerate(q.columns):
        base = q.base[c]
        data = np.array([0 if v is None else v for v in base], dtype=np.int32)
        valid = np.array([v is not None for v in base], dtype=bool)
        t.add_column(j, data, validity_from_mask(valid) if not valid.all() else None)
        if encoding == "bins":  # an every-value range index plus binned bitvectors beside it
            t.build_index(j, L.INDEX_RANGE)
            t.build_index(j, L.INDEX_BINS, [0, 2, 4, 8, 17, 100])
        elif encoding is not None:
            t.build_index(j, encoding)
    return t


def set_records(t, q: NU.Query, since=0):
    for j, c in enumerate(q.columns):
        rows, vals, vers, ok = q.update_arrays(c)
        keep = vers >= since
        t.set_updates(j, rows[keep], vals[keep], vers[keep], valid=ok[keep])


def table_function_view(t, q: NU.Query, txn, tasks_cols=None):
    """SELECT * through the table-function callbacks: every column's values and NULL-ness."""
    k = len(q.columns)
    fn = CubitScanFunction(t, list(range(k)) + [2 ** 64 - 1], None, F.TableFilterSet(), txn=txn)
    local = fn.init_local()
    rows = {}
    while True:
        cols, valid = fn.function_validity(local)
        if len(cols[0]) == 0:
            break
        assert valid[k].all()  # the row id is never NULL
        for i, r in enumerate(cols[k].tolist()):
            rows[r] = {c: (int(cols[j][i]) if valid[j][i] else None) for j, c in enumerate(q.columns)}
            for j in range(k):
                assert valid[j][i] or cols[j][i] == 0
    fn.close()
    return [rows[r] for r in sorted(rows)]


def check_query(t, q: NU.Query, nulls_first, label):
    txn = L.Txn(q.start, q.tid)
    view = table_function_view(t, q, txn)
    assert NU.answer(q, view, nulls_first) == q.rows, (label, q.con, q.sql)
    assert view == q.view, label
    n = len(view)
    ids = np.arange(n, dtype=np.int64)
    tx = O.Mvcc(q.start, q.tid)
    for j, c in enumerate(q.columns):
        vals, valid = t.fetch(j, ids, txn)
        rv, rvalid = O.fetch(oracle_columns(q)[j], ids, tx=tx, with_valid=True)
        assert np.array_equal(valid, rvalid) and np.array_equal(vals, rv), (label, c)
        for flt, pred in predicates(q, c):
            fs = F.TableFilterSet({j: flt})
            want = [r for r in range(n) if pred(view[r][c])]
            assert t.scan(fs, txn=txn).tolist() == want, (label, q.sql, c, flt)
            assert t.count(fs, txn=txn) == len(want), (label, q.sql, c, flt)


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE, L.INDEX_EQUALITY, "bins"])
@pytest.mark.parametrize("name", CASES)
def test_null_update_scripts_on_gpu(ctx, golden, name, encoding):
    case = NU.cases(golden)[name]
    qs = NU.queries(case)
    t = gpu_table(ctx, qs[0], encoding)
    for q in qs:
        set_records(t, q)
        check_query(t, q, case["nulls_first"], (name, encoding))
    # checkpoint: the records below the last snapshot's start merge into the base values, the
    # validity and every index leaf; the rest stay records, and the view is unchanged
    last = qs[-1]
    for j in range(len(last.columns)):
        t.merge_updates(j, last.start)
    check_query(t, last, case["nulls_first"], (name, encoding, "merged"))
    t.close()


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE, L.INDEX_EQUALITY, "bins"])
def test_null_update_merge_checkpoints_every_statement(ctx, golden, encoding):
    """null_update_merge.test with a checkpoint after every statement: each query's committed
    records are merged as soon as it has read them (NULL → value and value → NULL flips of the
    validity and of every range / equality leaf), and the next query sees only its new records."""
    case = NU.cases(golden)["null_update_merge"]
    qs = NU.queries(case)
    t = gpu_table(ctx, qs[0], encoding)
    merged = 0
    for q in qs:
        set_records(t, q, since=merged)
        check_query(t, q, case["nulls_first"], ("merge-each", encoding))
        for j in range(len(q.columns)):
            t.merge_updates(j, q.start)
        merged = q.start
        set_records(t, q, since=merged)
        check_query(t, q, case["nulls_first"], ("merge-each", encoding, "after"))
        assert t.column_statistics(1)[2] == any(v is None for v in (r["a"] for r in q.view))
    t.close()


def test_set_null_on_a_column_without_validity(ctx):
    """A column registered without NULLs gets a validity bitvector on its first SET NULL record:
    IS NULL finds the row for the writer only; statistics report has_null; the sum_product MVCC
    fallback skips the NULL row; a merge makes the NULL part of the base."""
    n = 200_003
    rng = np.random.default_rng(3)
    a = rng.integers(0, 100, n).astype(np.int64)
    b = rng.integers(1, 10, n).astype(np.int64)
    t = CubitTable(ctx, n)
    t.add_column(0, a)
    t.add_column(1, b)
    t.build_index(0, L.INDEX_RANGE)
    writer = NU.TXN_START + 5
    rows = np.array([7, 100_000, 150_001], np.int64)
    t.set_updates(0, rows, np.array([0, 55, 0], np.int64), np.array([writer, 3, writer], np.uint64),
                  valid=np.array([False, True, False]))
    w, r = L.Txn(4, writer), L.Txn(4, NU.TXN_START + 6)
    isnull = F.TableFilterSet({0: F.IsNullFilter()})
    assert t.scan(isnull, txn=w).tolist() == [7, 150_001]
    assert t.scan(isnull, txn=r).tolist() == []
    assert t.column_statistics(0)[2] is True
    lt50 = F.TableFilterSet({0: F.ConstantFilter("<", 50)})
    exp_a = a.copy()
    exp_a[100_000] = 55
    want_w = [i for i in np.flatnonzero(exp_a < 50).tolist() if i not in (7, 150_001)]
    assert t.scan(lt50, txn=w).tolist() == want_w
    s, cnt = t.sum_product(0, 1, lt50, txn=w)
    assert cnt == len(want_w) and s == int((exp_a[want_w] * b[want_w]).sum())
    vals, valid = t.fetch(0, rows, w)
    assert valid.tolist() == [False, True, False] and vals.tolist() == [0, 55, 0]
    # commit the writer at 5, merge everything below 6
    t.set_updates(0, rows, np.array([0, 55, 0], np.int64), np.array([5, 3, 5], np.uint64),
                  valid=np.array([False, True, False]))
    assert t.merge_updates(0, 6) == 3
    fresh = L.Txn(7, NU.TXN_START + 7)
    assert t.scan(isnull, txn=fresh).tolist() == [7, 150_001]
    assert t.scan(lt50).tolist() == want_w
    vals, valid = t.fetch(0, rows)
    assert valid.tolist() == [False, True, False] and vals.tolist() == [0, 55, 0]
    t.close()

