"""The reference's MVCC sqllogictests on the GPU: NULL updates and inserts /
deletes / updates under concurrent transactions (the files tests/sql_replay.py lists), each query
answered through the table function with validity (cubit_scan_function_validity) under the query's
snapshot, with the WHERE pushed as a TableFilterSet, and compared with the file's rows, the replay's
view and the oracle.

The device table follows the script as DuckDB's storage does: rows are appended as the script
inserts them (cubit_table_append, every index maintained), insert and delete stamps are re-declared
per query (cubit_table_set_inserts / cubit_table_set_deletes — a COMMIT re-stamps them), update
records with their validity (cubit_table_set_updates_nullable); the last snapshot's committed
records are merged at the end (cubit_table_merge_updates, the checkpoint) and the last query asked
again."""
import numpy as np
import pytest

import sql_replay as R
from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from cubit_amd.scan_function import CubitScanFunction
from cubit_amd.table import Context, CubitTable
from oracle import oracle as O
from test_oracle_mvcc_scripts import ALL, oracle_columns, predicates, pushed_filters, script

pytestmark = pytest.mark.gpu

ENCODINGS = [None, L.INDEX_RANGE, L.INDEX_EQUALITY, "bins"]
SMALL_BINS = [0, 2, 4, 8, 17, 100]
# columns with more distinct values than an every-value index should hold: chosen edges / keys
LARGE_KEYS = [0, 1, 2, 1000, 2000, 5000, 500000, 1000000]


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def add_index(t, j, vals, encoding):
    if encoding is None:
        return
    small = len(np.unique(vals)) <= 4096
    if encoding == "bins":  # a range index plus binned bitvectors beside it
        t.build_index(j, L.INDEX_RANGE, None if small else LARGE_KEYS)
        t.build_index(j, L.INDEX_BINS, SMALL_BINS if small else LARGE_KEYS)
    else:
        t.build_index(j, encoding, None if small else LARGE_KEYS)


class DeviceScript:
    """The device table of one script, kept in step with the replay's state query by query."""

    def __init__(self, ctx, encoding):
        self.ctx, self.encoding, self.t = ctx, encoding, None

    def sync(self, q: R.Query, since=0):
        n = q.n_rows
        if self.t is None:
            self.t = CubitTable(self.ctx, n)
            for j, c in enumerate(q.columns):
                data, valid = q.base[c]
                self.t.add_column(j, data.astype(np.int32), None if valid.all() else validity_from_mask(valid))
                add_index(self.t, j, data[valid], self.encoding)
        elif n > self.t.n_rows:
            old = self.t.n_rows
            cols, vmask = {}, {}
            for j, c in enumerate(q.columns):
                data, valid = q.base[c]
                cols[j] = data[old:n].astype(np.int32)
                if not valid[old:n].all():
                    vmask[j] = validity_from_mask(valid[old:n])
            self.t.append(cols, vmask or None)
        self.t.set_inserts(*q.insert_ranges())
        self.t.set_deletes(*q.delete_arrays())
        for j, c in enumerate(q.columns):
            rows, vals, vers, ok = q.update_arrays(c)
            keep = vers >= since
            self.t.set_updates(j, rows[keep], vals[keep], vers[keep], valid=ok[keep])

    def close(self):
        if self.t is not None:
            self.t.close()


def table_function_frame(t, q: R.Query, txn, fs=None) -> R.Frame:
    """SELECT <every column>, rowid through the table-function callbacks: values and NULL-ness."""
    k = len(q.columns)
    fn = CubitScanFunction(t, list(range(k)) + [2 ** 64 - 1], None, fs or F.TableFilterSet(), txn=txn)
    local = fn.init_local()
    parts = []
    while True:
        cols, valid = fn.function_validity(local)
        if len(cols[0]) == 0:
            break
        assert valid[k].all()  # the row id is never NULL
        for j in range(k):
            assert (cols[j][~valid[j]] == 0).all()
        parts.append((cols, valid))
    fn.close()
    if parts:
        ids = np.concatenate([p[0][k] for p in parts]).astype(np.int64)
        o = np.argsort(ids, kind="stable")
        f = {c: (np.concatenate([p[0][j] for p in parts]).astype(np.int64)[o], np.concatenate([p[1][j] for p in parts])[o])
             for j, c in enumerate(q.columns)}
        f["rowid"] = (ids[o], np.ones(len(ids), bool))
        return f
    empty = (np.zeros(0, np.int64), np.zeros(0, bool))
    return {**{c: empty for c in q.columns}, "rowid": empty}


def check_query(t, q: R.Query, nulls_first, label, exhaustive):
    txn = L.Txn(q.start, q.tid)
    view = table_function_frame(t, q, txn)
    assert R.frame_equal(view, q.view), (label, q.con, q.sql)
    assert R.answer(q, view, nulls_first) == q.rows, (label, q.con, q.sql)
    _, where, _ = R.split_query(q.sql)
    fs = pushed_filters(q, where)
    if where and fs is not None:
        got = table_function_frame(t, q, txn, fs)
        assert R.answer(q, got, nulls_first, filtered=True) == q.rows, (label, q.sql, "pushed")
        assert t.count(fs, txn=txn) == len(got["rowid"][0]), (label, q.sql)
    ids = view["rowid"][0]
    tx = O.Mvcc(q.start, q.tid, inserted=q.inserted, deleted=q.deleted)
    ocols = oracle_columns(q)
    for j, c in enumerate(q.columns):
        vals, valid = t.fetch(j, ids, txn)
        rv, rvalid = O.fetch(ocols[j], ids, tx=tx, with_valid=True)
        assert np.array_equal(valid, rvalid) and np.array_equal(vals, rv), (label, c)
        if not exhaustive:
            continue
        v, ok = view[c]
        for flt, pred in predicates(q, c):
            fsj = F.TableFilterSet({j: flt})
            want = ids[pred(v, ok)].tolist()
            assert t.scan(fsj, txn=txn).tolist() == want, (label, q.sql, c, flt)
            assert t.count(fsj, txn=txn) == len(want), (label, q.sql, c, flt)


@pytest.mark.parametrize("encoding", ENCODINGS)
@pytest.mark.parametrize("group,name", ALL)
def test_scripts_on_gpu(ctx, golden, group, name, encoding):
    case = script(golden, group, name)
    qs = R.queries(case)
    dev = DeviceScript(ctx, encoding)
    for q in qs:
        dev.sync(q)
        check_query(dev.t, q, case["nulls_first"], (name, encoding), exhaustive=q.n_rows <= 4096)
    # checkpoint: the records below the last snapshot's start merge into the base values, the
    # validity and every index leaf; the rest stay records, and the last view is unchanged
    last = qs[-1]
    for j in range(len(last.columns)):
        dev.t.merge_updates(j, last.start)
    check_query(dev.t, last, case["nulls_first"], (name, encoding, "merged"), exhaustive=last.n_rows <= 4096)
    dev.close()


@pytest.mark.parametrize("encoding", [None, "bins"])
@pytest.mark.parametrize("group,name", ALL)
def test_scripts_with_a_checkpoint_after_every_query(ctx, golden, group, name, encoding):
    """Every script with a checkpoint after each query: the committed records below the oldest
    open snapshot merge into the base values, the validity and the index leaves, and the next query
    hands over only the records at or above that horizon — every later query still reads the
    file's rows."""
    case = script(golden, group, name)
    dev = DeviceScript(ctx, encoding)
    merged = 0
    for q in R.queries(case):
        dev.sync(q, since=merged)
        check_query(dev.t, q, case["nulls_first"], (name, encoding, "merge-each"), exhaustive=False)
        horizon = max(merged, q.horizon)
        for j in range(len(q.columns)):
            dev.t.merge_updates(j, horizon)
        merged = horizon
    dev.close()


@pytest.mark.parametrize("encoding", ENCODINGS)
def test_null_update_merge_checkpoints_every_statement(ctx, golden, encoding):
    """null_update_merge.test with a checkpoint after every statement: each query's committed
    records are merged as soon as it has read them (NULL → value and value → NULL flips of the
    validity and of every range / equality leaf), and the next query sees only its new records."""
    case = script(golden, "null_updates", "null_update_merge")
    qs = R.queries(case)
    dev = DeviceScript(ctx, encoding)
    merged = 0
    for q in qs:
        dev.sync(q, since=merged)
        check_query(dev.t, q, case["nulls_first"], ("merge-each", encoding), exhaustive=True)
        for j in range(len(q.columns)):
            dev.t.merge_updates(j, q.start)
        merged = q.start
        dev.sync(q, since=merged)
        check_query(dev.t, q, case["nulls_first"], ("merge-each", encoding, "after"), exhaustive=True)
        assert dev.t.column_statistics(1)[2] == (~q.view["a"][1]).any()
    dev.close()


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
    writer = R.TXN_START + 5
    rows = np.array([7, 100_000, 150_001], np.int64)
    t.set_updates(0, rows, np.array([0, 55, 0], np.int64), np.array([writer, 3, writer], np.uint64),
                  valid=np.array([False, True, False]))
    w, r = L.Txn(4, writer), L.Txn(4, R.TXN_START + 6)
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
    fresh = L.Txn(7, R.TXN_START + 7)
    assert t.scan(isnull, txn=fresh).tolist() == [7, 150_001]
    assert t.scan(lt50).tolist() == want_w
    vals, valid = t.fetch(0, rows)
    assert valid.tolist() == [False, True, False] and vals.tolist() == [0, 55, 0]
    t.close()
