"""Regression tests for the round-1 review findings, all through the C ABI:

* a filter folded to FALSE (or a count) after a non-empty scan on the same context leaves no
  tile directory behind for the table function to hand out (CubitScanInitGlobal);
* the fused sum with b decoded from its range index keeps b in full int64 (values past 2^31,
  staged and dense tiles alike);
* CUBIT_SCAN_CHECK_CAPACITY reports an overflowing buffer as CUBIT_ERR_CAPACITY;
* switching the context's stream keeps results exact (the old stream is drained first).
"""
import ctypes as C

import numpy as np
import pytest
import torch

from conftest import lineitem
from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.scan_function import ROW_ID, CubitScanFunction
from cubit_amd.table import Context, CubitTable, to_ctypes
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def q6_table(ctx, li):
    t = CubitTable(ctx, li.n_rows, li.row_base)
    for c, arr in enumerate((li.l_shipdate, li.l_discount, li.l_quantity, li.l_extendedprice)):
        t.add_column(c, arr)
    months = [F.date(y, m, 1) for y in range(1992, 1999) for m in range(1, 13)] + [F.date(1999, 1, 1)]
    t.build_index(0, L.INDEX_RANGE, months)
    t.build_index(1, L.INDEX_RANGE)
    t.build_index(2, L.INDEX_RANGE)
    return t


def drain_all(fn):
    local = fn.init_local()
    out = []
    while True:
        cols = fn.function(local)
        if len(cols[0]) == 0:
            return out
        out.append(cols)


def test_false_fold_after_nonempty_scan_leaves_no_directory(ctx):
    li = lineitem(0.1)
    t = q6_table(ctx, li)
    first = CubitScanFunction(t, [0, 1, 2, ROW_ID], [3], F.q6_filter_set())
    assert sum(len(c[0]) for c in drain_all(first)) > 0
    assert ctx.last_tiles()[0].shape[0] > 0
    # l_quantity > 10,000 lies past the index's vmax: the planner folds it to FALSE
    off = F.TableFilterSet({2: F.ConstantFilter(">", 10_000 * 100)})
    fn = CubitScanFunction(t, [2, ROW_ID], [1], off)
    assert drain_all(fn) == []
    assert fn.progress() == 100.0
    assert ctx.last_tiles()[0].shape[0] == 0
    # the same after a count(*) and after a fused sum (neither writes row ids)
    t.scan(F.q6_filter_set())
    t.count(F.q6_filter_set())
    assert ctx.last_tiles()[0].shape[0] == 0
    t.scan(F.q6_filter_set())
    t.sum_product(3, 1, F.q6_filter_set())
    assert ctx.last_tiles()[0].shape[0] == 0
    fn = CubitScanFunction(t, [2, ROW_ID], [1], off)
    assert drain_all(fn) == []


@pytest.mark.parametrize("base", [2 ** 33 - 3, -(2 ** 40) + 11, 2 ** 62])
def test_fused_sum_decoded_b_beyond_int32(ctx, base):
    """b pinned by the filter to 4 stored values far outside int32 (BIGINT / scaled DECIMAL
    storage): decoded from its range index, the 128-bit sum equals the exact one on sparse
    (staged) and dense (direct) tiles."""
    n = 700_000
    rng = np.random.default_rng(base & 0xFFFF)
    # a narrow spread far from zero: the all-distinct-values range index builds (presence
    # bitmap over [vmin, vmax]), and every value is outside int32
    steps = np.array([0, 7, 19, 20, 1000, 40_000], dtype=np.int64)
    vals = np.int64(base) + steps
    b = vals[rng.integers(0, len(vals), n)]
    a = rng.integers(-(10 ** 9), 10 ** 9, n).astype(np.int64)
    # c: sparse tiles (2 % pass) in the first half, every row passes in the second (dense tiles)
    c = rng.integers(0, 1000, n).astype(np.int32)
    c[n // 2:] = 0
    t = CubitTable(ctx, n)
    t.add_column(0, a)
    t.add_column(1, b)
    t.add_column(2, c)
    t.build_index(1, L.INDEX_RANGE)
    t.build_index(2, L.INDEX_RANGE)
    lo, hi = int(vals[1]), int(vals[4])
    fs = F.TableFilterSet({1: F.ConjunctionAndFilter([F.ConstantFilter(">=", lo), F.ConstantFilter("<=", hi)]),
                           2: F.ConstantFilter("<", 20)})
    keep = np.nonzero((b >= lo) & (b <= hi) & (c < 20))[0]
    want = int((a[keep].astype(object) * b[keep].astype(object)).sum())
    got, cnt = t.sum_product(0, 1, fs)
    assert t.last_sum_decode() == 4  # decoded, not gathered
    assert cnt == len(keep)
    assert got == want
    got2, _ = t.sum_product(0, 1, fs, gather_b=True)
    assert got2 == want


def test_check_capacity_flag(ctx):
    n = 400_000
    v = (np.arange(n, dtype=np.int64) * 7919) % 1000
    t = CubitTable(ctx, n)
    t.add_column(0, v)
    t.build_index(0, L.INDEX_RANGE)
    fs = F.TableFilterSet({0: F.ConstantFilter("<", 100)})
    plan = F.serialize(fs)
    arr = to_ctypes(plan.nodes)
    want = int((v < 100).sum())
    cap = want // 2
    out = ctx.alloc(cap * 8)
    cnt = ctx.alloc(16)
    for flags in (0, L.SCAN_ORDERED):
        # without the flag: OK, the count still reports every qualifying row
        rc = ctx.lib.cubit_table_scan(t.handle, arr, len(plan.nodes), None, C.c_void_p(out.addr), cap,
                                      C.c_void_p(cnt.addr), flags)
        assert rc == L.OK
        ctx.check()
        assert int(cnt.download(np.uint64, 1)[0]) == want
        rc = ctx.lib.cubit_table_scan(t.handle, arr, len(plan.nodes), None, C.c_void_p(out.addr), cap,
                                      C.c_void_p(cnt.addr), flags | L.SCAN_CHECK_CAPACITY)
        assert rc == L.ERR_CAPACITY
        assert b"capacity" in ctx.lib.cubit_last_error()
    big = ctx.alloc(want * 8)
    rc = ctx.lib.cubit_table_scan(t.handle, arr, len(plan.nodes), None, C.c_void_p(big.addr), want,
                                  C.c_void_p(cnt.addr), L.SCAN_ORDERED | L.SCAN_CHECK_CAPACITY)
    assert rc == L.OK
    assert np.array_equal(big.download(np.int64, want), np.nonzero(v < 100)[0])


def test_stream_switch_between_scans(ctx):
    li = lineitem(0.1)
    ref = O.table_scan([O.Column(li.l_shipdate), O.Column(li.l_discount), O.Column(li.l_quantity)],
                       F.serialize(F.q6_filter_set()), li.n_rows)
    c2 = Context(0)
    t = q6_table(c2, li)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    plan = F.serialize(F.q6_filter_set())
    outs = [c2.alloc(li.n_rows * 8) for _ in range(4)]
    cnts = [c2.alloc(16) for _ in range(4)]
    for i in range(4):
        # launch on one stream, switch to the other without waiting: the ticket / directory
        # reuse must stay in order
        c2.set_stream((s1 if i % 2 == 0 else s2).cuda_stream)
        t.scan_into(plan.nodes, outs[i].addr, li.n_rows, cnts[i].addr, ordered=True)
    c2.sync()
    for i in range(4):
        n = int(cnts[i].download(np.uint64, 1)[0])
        assert np.array_equal(outs[i].download(np.int64, n), ref)
    c2.set_stream(None)
    t.close()
    c2.close()


def test_updates_outside_index_statistics(ctx):
    """Round 2: the planner folded constants against the index's base statistics (vmin / vmax,
    every-distinct-value exactness) alone, so a visible update to a value outside them was
    dropped (e.g. `v < -3` folded to FALSE while an update set a row to -7). The statistics are
    now widened with the update values, as DuckDB's zonemaps consult update statistics
    (standard_column_data.cpp:50-57)."""
    rng = np.random.default_rng(12)
    n = 70_001
    t = CubitTable(ctx, n)
    cols = []
    for c, enc in enumerate((L.INDEX_RANGE, L.INDEX_EQUALITY, L.INDEX_RANGE)):
        d = rng.integers(0, 50, n).astype(np.int64)
        t.add_column(c, d)
        t.build_index(c, enc, [10, 20, 30, 40] if c == 2 else None)
        if c == 2:
            t.build_index(c, L.INDEX_BINS, [0, 10, 20, 30, 40, 50])
        rows = np.array([5, 77, 1000, 5000, 60_000], dtype=np.int64)
        vals = np.array([-7, 80, 23, 55, -1], dtype=np.int64)  # 23: inside, the rest outside [0, 50)
        vers = np.array([1, 1, 1, 1, 9], dtype=np.uint64)
        t.set_updates(c, rows, vals, vers)
        cols.append(O.Column(d, updates=(rows, vals, vers)))
    for start in (2, 10):
        tx = L.Txn(start, TXN_START_REG + start)
        for c in range(3):
            for cmp, k in (("<", -3), ("<", 0), ("<=", -7), ("=", -7), ("=", 80), (">", 60), (">=", 50),
                           ("!=", 23), ("=", -1), ("<", 51), (">", -8)):
                fs = F.TableFilterSet({c: F.ConstantFilter(cmp, k)})
                ref = O.table_scan(cols, F.serialize(fs), n, tx=O.Mvcc(start, TXN_START_REG + start))
                got = t.scan(fs, txn=tx)
                assert np.array_equal(got, ref), (start, c, cmp, k)
            fs = F.TableFilterSet({c: F.ConjunctionAndFilter([F.ConstantFilter(">=", 50), F.ConstantFilter("<", 90)])})
            ref = O.table_scan(cols, F.serialize(fs), n, tx=O.Mvcc(start, TXN_START_REG + start))
            assert np.array_equal(t.scan(fs, txn=tx), ref), (start, c, "interval")
    t.close()


TXN_START_REG = 4611686018427388000


def test_exact_index_over_a_wide_span(ctx):
    """TIMESTAMP-like INT64 columns: few distinct values spread over more than 2^32. The
    all-distinct-values index used to refuse them (the shim builds that index on attach);
    now the distinct values are sorted on the host. Appends bring new wide values."""
    rng = np.random.default_rng(5)
    keys = np.array([-(1 << 50), 0, 1 << 40, (1 << 62) + 3], dtype=np.int64)
    n = 70_001
    a = keys[rng.integers(0, len(keys), n)]
    valid = rng.random(n) > 0.05
    from cubit_amd.datagen import validity_from_mask

    t = CubitTable(ctx, n)
    t.add_column(0, a, validity_from_mask(valid))
    t.build_index(0, L.INDEX_RANGE)
    extra = np.array([1 << 45, -(1 << 50), 7], dtype=np.int64)[rng.integers(0, 3, 5000)]
    ev = rng.random(5000) > 0.05
    for step in range(2):
        data = a if step == 0 else np.concatenate([a, extra])
        vm = valid if step == 0 else np.concatenate([valid, ev])
        col = O.Column(data, validity_from_mask(vm))
        for cmp in ("=", "<", ">=", "!="):
            for k in list(keys) + [1 << 45, 7, 5]:
                fs = F.TableFilterSet({0: F.ConstantFilter(cmp, int(k))})
                ref = O.table_scan([col], F.serialize(fs), len(data))
                assert np.array_equal(t.scan(fs), ref), (step, cmp, k)
        if step == 0:
            t.append({0: extra}, {0: validity_from_mask(ev)})
    t.close()


def test_equality_at_int64_max_on_a_binned_column(ctx):
    """Round 6: an AND over a column with a BINS index folds its constants into one half-open
    interval; `v = INT64_MAX` has no representable end, and was folded to FALSE. It is [INT64_MAX,
    ∞) = {INT64_MAX} (UBIGINT's 2^64 - 1 has that key). Every comparison at both ends of int64
    against numpy, with and without the bins."""
    n = 200_003
    rng = np.random.default_rng(3)
    v = rng.integers(-1000, 1000, n).astype(np.int64)
    v[::7] = np.iinfo(np.int64).max
    v[::11] = np.iinfo(np.int64).min
    for bins in (False, True):
        t = CubitTable(ctx, n)
        t.add_column(0, v)
        t.build_index(0, L.INDEX_RANGE)
        if bins:
            t.build_index(0, L.INDEX_BINS, [-(2 ** 63), -10, 0, 10, 2 ** 63 - 1])
        for c in (2 ** 63 - 1, -(2 ** 63), 0):
            for cmp, op in (("=", np.equal), ("<", np.less), ("<=", np.less_equal), (">", np.greater),
                            (">=", np.greater_equal), ("!=", np.not_equal)):
                fs = F.TableFilterSet({0: F.ConstantFilter(cmp, c)})
                assert np.array_equal(t.scan(fs), np.flatnonzero(op(v, c))), (bins, cmp, c)
        t.close()
