"""Selection narrowing of unindexed comparisons: RowGroup::TemplatedScan reads each filter
column after the first only at the rows the earlier filters kept (ColumnData::Select over the
shared SelectionVector, src/storage/table/row_group.cpp:537-550). Here a constant comparison on a
column the index cannot answer (K0), inside a conjunction whose other literals keep at most one
row in 32, reads its column only at those rows (masked_compare_kernel). It must never change a
result: every scan is compared with the oracle, with narrowing on and off, for every comparison,
INT32 / INT64 columns with NULLs, constants past the column type, masks of every density, under
deletes and under updates (which build the leaves in full)."""
import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from oracle import oracle as O

pytestmark = pytest.mark.gpu

BASE = 7
TXN_START = 4611686018427388000
CMPS = ["=", "!=", "<", "<=", ">", ">="]
N = 2_000_003


@pytest.fixture(scope="module")
def ctx():
    from cubit_amd.table import Context
    c = Context(0)
    yield c
    c.close()


def make(ctx, n=N, seed=1):
    from cubit_amd.table import CubitTable
    rng = np.random.default_rng(seed)
    c0 = rng.integers(0, 1000, n).astype(np.int32)                   # equality index: 0.1 % per key
    c1 = rng.integers(-1_000_000, 1_000_000, n).astype(np.int32)     # unindexed INT32, NULLs
    c1[:50] = [np.iinfo(np.int32).min, np.iinfo(np.int32).max] * 25
    c2 = rng.integers(-2 ** 62, 2 ** 62, n).astype(np.int64)         # unindexed INT64
    c2[50:60] = [np.iinfo(np.int64).min, np.iinfo(np.int64).max] * 5
    c3 = rng.integers(0, 100, n).astype(np.int32)                    # range index
    valid1 = rng.random(n) >= 0.05
    vw = validity_from_mask(valid1)
    cols = [c0, c1, c2, c3]
    t = CubitTable(ctx, n, row_base=BASE)
    for c, a in enumerate(cols):
        t.add_column(c, a, vw if c == 1 else None)
    t.build_index(0, L.INDEX_EQUALITY)
    t.build_index(3, L.INDEX_RANGE)
    return t, cols, vw


def ocols(cols, vw, updates=None):
    updates = updates or {}
    return [O.Column(a, vw if c == 1 else None, updates=updates.get(c)) for c, a in enumerate(cols)]


def check(t, oc, fs, residual=None, txn=None, tx=None, what=""):
    ref = O.table_scan(oc, F.serialize(fs, residual), t.n_rows, row_base=BASE, tx=tx)
    t.use_narrowing(True)
    got = t.scan(fs, residual, txn=txn)
    narrowed = t.last_narrowed()
    assert np.array_equal(got, ref), ("narrowing on", what, fs, residual)
    assert t.count(fs, residual, txn=txn) == len(ref)
    t.use_narrowing(False)
    got_off = t.scan(fs, residual, txn=txn)
    assert t.last_narrowed() == 0
    t.use_narrowing(True)
    assert np.array_equal(got_off, ref), ("narrowing off", what, fs, residual)
    return ref, narrowed


def test_every_comparison_after_an_index_leaf(ctx):
    t, cols, vw = make(ctx)
    oc = ocols(cols, vw)
    i32, i64 = np.iinfo(np.int32), np.iinfo(np.int64)
    consts = {1: [0, 123_456, -999_999, i32.min, i32.max, 2 ** 40, -2 ** 40],
              2: [0, 2 ** 61, -2 ** 61, i64.min, i64.max]}
    for col, cs in consts.items():
        for c in cs:
            for op in CMPS:
                fs = F.TableFilterSet({0: F.ConstantFilter("=", 17), col: F.ConstantFilter(op, int(c))})
                ref, narrowed = check(t, oc, fs, what=(col, op, c))
                # the equality leaf keeps 0.1 % of the rows: the comparison is narrowed
                # (unless the planner folded it away as always true / false)
                assert narrowed <= 1
    # two unindexed comparisons behind the index leaf, both narrowed, one after the other
    fs = F.TableFilterSet({0: F.ConstantFilter("=", 5), 1: F.ConstantFilter(">", 0), 2: F.ConstantFilter("<", 0)})
    ref, narrowed = check(t, oc, fs)
    assert narrowed == 2 and len(ref) > 0
    t.close()


def test_mask_density_decides(ctx):
    t, cols, vw = make(ctx)
    oc = ocols(cols, vw)
    # a dense mask (half the rows): the comparison reads the whole column
    fs = F.TableFilterSet({3: F.ConstantFilter("<", 50), 1: F.ConstantFilter("<", 0)})
    _, narrowed = check(t, oc, fs)
    assert narrowed == 0
    # a 2 % mask (the range index): narrowed
    fs = F.TableFilterSet({3: F.ConstantFilter("<", 2), 1: F.ConstantFilter("<", 0)})
    _, narrowed = check(t, oc, fs)
    assert narrowed == 1
    # only unindexed comparisons: the first in full, the ones after it through its rows
    fs = F.TableFilterSet({1: F.ConstantFilter("<", -980_000), 2: F.ConstantFilter("<", -2 ** 62 + 2 ** 57)})
    ref, narrowed = check(t, oc, fs)
    assert narrowed == 1 and len(ref) > 0
    fs = F.TableFilterSet({1: F.ConstantFilter(">", -500_000), 2: F.ConstantFilter(">", -2 ** 61)})
    _, narrowed = check(t, oc, fs)
    assert narrowed == 0  # the first keeps 3/4 of the rows
    # a mask with no row at all, and a residual conjunction of several index leaves
    fs = F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter("=", 3), F.ConstantFilter("=", 4)]),
                           1: F.ConstantFilter("!=", 0)})
    ref, _ = check(t, oc, fs)
    assert len(ref) == 0
    res = F.And(F.And(F.Cmp(0, ">=", 10), F.Cmp(0, "<", 20)), F.And(F.Cmp(3, "=", 7), F.Cmp(2, ">=", 0)))
    _, narrowed = check(t, oc, None, res)
    assert narrowed >= 1  # column 2 through the mask of [10, 20) (a union of the equality index's leaves) and 3 = 7
    # an OR keeps the comparison whole (no conjunction to narrow by)
    res = F.Or(F.Cmp(0, "=", 3), F.Cmp(1, "<", 0))
    _, narrowed = check(t, oc, None, res)
    assert narrowed == 0
    # IS NULL / IS NOT NULL beside the comparison
    fs = F.TableFilterSet({0: F.ConstantFilter("=", 9),
                           1: F.ConjunctionAndFilter([F.IsNotNullFilter(), F.ConstantFilter(">=", -5)])})
    check(t, oc, fs)
    t.close()


def test_sum_product_and_deletes(ctx):
    t, cols, vw = make(ctx)
    n = t.n_rows
    valid1 = np.unpackbits(vw.view(np.uint8), bitorder="little")[:n].astype(bool)
    fs = F.TableFilterSet({0: F.ConstantFilter("=", 42), 1: F.ConstantFilter(">", 0)})
    mask = (cols[0] == 42) & (cols[1] > 0) & valid1
    want = int((cols[3][mask].astype(object) * cols[0][mask].astype(object)).sum())
    t.add_column(4, cols[3].astype(np.int64))  # DECIMAL storage for the fused sum
    t.add_column(5, cols[0].astype(np.int64))
    for on in (True, False):
        t.use_narrowing(on)
        s, cnt = t.sum_product(4, 5, fs)
        assert (s, cnt) == (want, int(mask.sum())), on
        assert t.last_narrowed() == (1 if on else 0)
    t.use_narrowing(True)
    # deletes from two transactions: the visibility leaf joins the mask
    rng = np.random.default_rng(4)
    rows = np.sort(rng.choice(n, size=40_000, replace=False)).astype(np.int64)
    writer = TXN_START + 3
    ids = np.where(rng.random(len(rows)) < 0.5, np.uint64(4), np.uint64(writer)).astype(np.uint64)
    t.set_deletes(rows, ids)
    deleted = np.full(n, np.uint64(2 ** 64 - 2), dtype=np.uint64)
    deleted[rows] = ids
    oc = ocols(cols, vw)
    for start, tid in ((2, writer), (10, TXN_START + 5)):
        tx = O.Mvcc(start, tid, deleted=deleted)
        for op in CMPS:
            fs = F.TableFilterSet({0: F.ConstantFilter("=", 77), 2: F.ConstantFilter(op, 0)})
            check(t, oc, fs, txn=L.Txn(start, tid), tx=tx, what=(start, op))
    t.close()


def test_updates_build_full_leaves(ctx):
    t, cols, vw = make(ctx)
    n = t.n_rows
    rng = np.random.default_rng(8)
    writer = TXN_START + 7
    upd = {}
    for c, (lo, hi) in ((1, (-1_000_000, 1_000_000)), (0, (0, 1000))):
        rows = np.sort(rng.choice(n, size=20_000, replace=False)).astype(np.int64)
        vals = rng.integers(lo, hi, len(rows)).astype(np.int64)
        vers = np.where(rng.random(len(rows)) < 0.5, np.uint64(3), np.uint64(writer)).astype(np.uint64)
        t.set_updates(c, rows, vals, vers)
        upd[c] = (rows, vals, vers)
    oc = ocols(cols, vw, upd)
    for start, tid in ((2, writer), (10, TXN_START + 8), (1, TXN_START + 9)):
        tx = O.Mvcc(start, tid)
        for op in ("<", "=", "!="):
            fs = F.TableFilterSet({0: F.ConstantFilter("=", 11), 1: F.ConstantFilter(op, 0)})
            _, narrowed = check(t, oc, fs, txn=L.Txn(start, tid), tx=tx, what=(start, tid, op))
            if start == 1 and tid != writer:
                assert narrowed == 1  # no update visible: narrowed as usual
            else:
                assert narrowed == 0
    t.close()


def test_random_conjunctions(ctx):
    t, cols, vw = make(ctx, 1_000_033, seed=3)
    oc = ocols(cols, vw)
    rng = np.random.default_rng(13)
    lims = {0: (-1, 1001), 1: (-1_000_100, 1_000_100), 2: (-2 ** 62, 2 ** 62), 3: (-1, 101)}
    narrowed_total = 0
    for i in range(60):
        filters = {}
        for c in rng.choice(4, size=rng.integers(2, 5), replace=False):
            c = int(c)
            lo, hi = lims[c]
            f = F.ConstantFilter(CMPS[rng.integers(0, 6)], int(rng.integers(lo, hi)))
            if c == 1 and rng.random() < 0.2:
                f = F.ConjunctionAndFilter([f, F.IsNotNullFilter()])
            filters[c] = f
        fs = F.TableFilterSet(filters)
        residual = None
        if rng.random() < 0.3:
            residual = F.And(F.Cmp(0, CMPS[rng.integers(0, 6)], int(rng.integers(0, 1000))),
                             F.Cmp(2, CMPS[rng.integers(0, 6)], int(rng.integers(-2 ** 62, 2 ** 62))))
        _, narrowed = check(t, oc, fs, residual, what=i)
        narrowed_total += narrowed
    assert narrowed_total >= 5, narrowed_total
    t.close()


def test_order_by_estimated_selectivity(ctx):
    """Two unindexed comparisons in both textual orders (and behind an index leaf): the plan
    builds the most selective one first — full-column, as the mask — and reads the other only at
    its rows, whatever the order the filters came in (the reference's AdaptiveFilter reorders
    its filters by measured cost, adaptive_filter.cpp:21-88); rows equal the oracle either way.
    The estimate comes from per-zone min / max, so no count is read back while planning."""
    t, cols, vw = make(ctx)
    oc = ocols(cols, vw)
    sel1 = F.ConstantFilter("<", -990_000)        # col 1: ≈ 0.5 % (the more selective)
    sel2 = F.ConstantFilter("<", -2 ** 62 + 2 ** 59)  # col 2: ≈ 6 %
    orders = []
    for fs in (F.TableFilterSet({1: sel1, 2: sel2}), F.TableFilterSet({2: sel2, 1: sel1})):
        ref, narrowed = check(t, oc, fs)
        assert len(ref) > 0 and narrowed == 1
        t.scan(fs)
        orders.append(t.last_k0_order())
    assert orders[0] == orders[1] == [1, 2], orders
    # behind an index leaf keeping 2 % (the mask), both chained, most selective first
    for fs in (F.TableFilterSet({0: F.ConstantFilter("<", 20), 1: sel1, 2: sel2}),
               F.TableFilterSet({2: sel2, 0: F.ConstantFilter("<", 20), 1: sel1})):
        t.build_index(0, L.INDEX_RANGE)
        ref, narrowed = check(t, oc, fs)
        assert narrowed == 2
        t.scan(fs)
        assert t.last_k0_order() == [1, 2]
    t.close()


def test_caller_owned_column_changed(ctx):
    """A caller-owned device column rewritten in place: after cubit_table_column_changed the
    zonemaps and statistics follow the new values (stale per-zone bounds would skip zones that
    now qualify)."""
    import torch

    from cubit_amd.table import CubitTable

    n = 1_000_003
    a = torch.arange(n, dtype=torch.int64, device="cuda")  # ascending: zones with disjoint bounds
    t = CubitTable(ctx, n)
    t.add_device_column(0, a.data_ptr(), L.TYPE_INT64)
    fs = F.TableFilterSet({0: F.ConstantFilter("<", 1000)})
    assert t.count(fs) == 1000
    assert t.last_zones()[0] < t.last_zones()[1]  # the zonemap skipped zones
    a.copy_(torch.flip(a, [0]))  # now the small values sit in the last zone
    torch.cuda.synchronize()
    t.column_changed(0)
    assert t.count(fs) == 1000
    assert t.scan(fs)[0] == n - 1000
    assert t.column_statistics(0)[:2] == (0, n - 1)
    t.close()
