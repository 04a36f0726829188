"""Zonemaps: RowGroup::CheckZonemap / CheckZonemapSegments
(src/storage/table/row_group.cpp:361-371, 407-445) skip row groups whose min/max statistics
prove a filter false. Here every index and validity bitvector carries per-zone classes (no row
/ every row of a 131,072-row zone set), the planner evaluates the filter over them and the
kernels skip the zones it is false on. Skipping must never change a result: every scan here is
compared with the oracle, with the skip on and off, on clustered data where it prunes (a
date-like ascending column, a column with whole NULL zones) beside unclustered columns where
it cannot, then again after appends, merges and under MVCC updates that move rows between
zones."""
import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from cubit_amd.scan_function import ROW_ID, CubitScanFunction
from cubit_amd.table import Context, CubitTable, runs_in_row_order
from oracle import oracle as O

pytestmark = pytest.mark.gpu

ZONE = 131072
BASE = 1_000_000_007
TXN_START = 4611686018427388000
CMPS = ["=", "!=", "<", "<=", ">", ">="]


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def clustered(n, seed, start=0):
    """Column data for rows [start, start + n) of the clustered table."""
    rng = np.random.default_rng(seed)
    i = np.arange(start, start + n, dtype=np.int64)
    c0 = ((i * 2500) // 6_000_011 + rng.integers(0, 8, n)).astype(np.int32)  # date-like, ascending + jitter
    c1 = (i // 20_000).astype(np.int64)                                      # sorted, NULL zones below
    valid1 = ~((i >= 1_000_000) & (i < 1_400_000)) & ~((i >= 4_000_000) & (rng.random(n) < 0.01))
    c2 = rng.integers(0, 50, n).astype(np.int32)                             # unclustered
    c3 = (i // 7).astype(np.int64)                                           # sorted, no index (K0)
    return [c0, c1, c2, c3], valid1


def make_table(ctx, n=6_000_011):
    cols, valid1 = clustered(n, 5)
    t = CubitTable(ctx, n, row_base=BASE)
    vw = validity_from_mask(valid1)
    for c, a in enumerate(cols):
        t.add_column(c, a, vw if c == 1 else None)
    t.build_index(0, L.INDEX_RANGE, list(range(0, 2600, 25)))
    t.build_index(0, L.INDEX_BINS, list(range(0, 2700, 100)))
    t.build_index(1, L.INDEX_RANGE)
    t.build_index(2, L.INDEX_EQUALITY)
    return t, cols, vw


def oracle_cols(cols, vw, updates=None):
    updates = updates or {}
    return [O.Column(a, vw if c == 1 else None, updates=updates.get(c)) for c, a in enumerate(cols)]


def rand_filter(rng, col, depth=0):
    lo, hi = {0: (-10, 2620), 1: (-2, 305), 2: (-1, 51), 3: (-5, 900_000)}[col]
    r = rng.random()
    if depth < 1 and r < 0.3:
        kids = [rand_filter(rng, col, depth + 1) for _ in range(2)]
        return F.ConjunctionAndFilter(kids) if rng.random() < 0.7 else F.ConjunctionOrFilter(kids)
    if col == 1 and r < 0.4:
        return F.IsNullFilter() if rng.random() < 0.5 else F.IsNotNullFilter()
    return F.ConstantFilter(CMPS[rng.integers(0, 6)], int(rng.integers(lo, hi)))


def rand_residual(rng, depth=0):
    if depth < 2 and rng.random() < 0.5:
        kids = [rand_residual(rng, depth + 1) for _ in range(2)]
        return F.And(*kids) if rng.random() < 0.5 else F.Or(*kids)
    c = int(rng.integers(0, 3))
    lo, hi = {0: (-10, 2620), 1: (-2, 305), 2: (-1, 51)}[c]
    return F.Cmp(c, CMPS[rng.integers(0, 6)], int(rng.integers(lo, hi)))


def check_scan(t, ocols, fs, residual=None, txn=None, tx=None, what=""):
    ref = O.table_scan(ocols, F.serialize(fs, residual), t.n_rows, row_base=BASE, tx=tx)
    got = t.scan(fs, residual, txn=txn)
    assert np.array_equal(got, ref), ("zonemap on", what, fs, residual)
    live, zones = t.last_zones()
    got_off = t.scan(fs, residual, txn=txn, zonemap=False)
    assert np.array_equal(got_off, ref), ("zonemap off", what, fs, residual)
    return ref, live, zones


def test_clustered_range_skips_zones(ctx):
    t, cols, vw = make_table(ctx)
    ocols = oracle_cols(cols, vw)
    nz = (t.n_rows + ZONE - 1) // ZONE
    # a ten-day window of the date-like column: one or two zones of 46
    fs = F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", 1000), F.ConstantFilter("<", 1010)])})
    ref, live, zones = check_scan(t, ocols, fs)
    assert zones == nz and 1 <= live <= 3, (live, zones)
    assert len(ref) > 0
    # tile-run order through the directory: skipped tiles have empty entries
    got = t.scan(fs, ordered=False)
    d, _ = ctx.last_tiles()
    assert int(d[:, 1].sum()) == len(ref)
    assert np.array_equal(runs_in_row_order(got, d), ref)
    assert t.count(fs) == len(ref)
    assert t.last_zones()[0] == live
    assert t.count(fs, zonemap=False) == len(ref)
    assert t.last_zones()[0] == nz
    # the unclustered column alone prunes nothing
    fs2 = F.TableFilterSet({2: F.ConstantFilter("=", 7)})
    _, live2, _ = check_scan(t, ocols, fs2)
    assert live2 == nz
    # IS NULL: only the zones holding NULLs (rows 1.0-1.4 M, and the sparse NULLs past 4 M)
    fs3 = F.TableFilterSet({1: F.IsNullFilter()})
    ref3, live3, _ = check_scan(t, ocols, fs3)
    assert live3 < nz and len(ref3) > 400_000
    # two clustered ranges that never meet: every zone is ruled out, no launch
    fs4 = F.TableFilterSet({0: F.ConstantFilter("<", 100), 1: F.ConstantFilter(">=", 250)})
    ref4, live4, _ = check_scan(t, ocols, fs4)
    assert len(ref4) == 0 and live4 == 0
    # a range OR an unclustered equality: the OR keeps every zone
    res = F.Or(F.Cmp(0, ">=", 2400), F.Cmp(2, "=", 3))
    _, live_or, _ = check_scan(t, ocols, None, res)
    assert live_or == nz
    # ... while an AND with the range keeps the range's zones only
    res = F.And(F.Cmp(0, ">=", 2400), F.Cmp(2, "=", 3))
    _, live5, _ = check_scan(t, ocols, None, res)
    assert live5 <= nz // 20 + 2
    # NOT of a range (v < c complemented): the zones past c
    _, live6, _ = check_scan(t, ocols, F.TableFilterSet({0: F.ConstantFilter(">=", 2450)}))
    assert live6 <= 3
    # a column without an index (K0 leaf): classes from the column's per-zone min / max, as the
    # reference's CheckZonemap does for every column
    _, live7, _ = check_scan(t, ocols, F.TableFilterSet({3: F.ConstantFilter("<", 20_000)}))
    assert live7 <= 2
    # a constant between index keys (candidate-check leaf): the same statistics
    _, live8, _ = check_scan(t, ocols, F.TableFilterSet({0: F.ConstantFilter("=", 1234)}))
    assert live8 <= 3
    t.close()


def test_fused_sum_and_table_function_with_skipped_zones(ctx):
    t, cols, vw = make_table(ctx)
    valid1 = np.unpackbits(vw.view(np.uint8), bitorder="little")[: t.n_rows].astype(bool)
    fs = F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", 2000), F.ConstantFilter("<", 2100)]),
                           2: F.ConstantFilter("<", 25)})
    mask = (cols[0] >= 2000) & (cols[0] < 2100) & (cols[2] < 25)
    want = int((cols[3][mask & valid1].astype(object) * cols[1][mask & valid1].astype(object)).sum())
    for zm in (True, False):
        s, n = t.sum_product(3, 1, fs, zonemap=zm)
        assert n == int(mask.sum()) and s == want, (zm, n, s)
        live, nz = t.last_zones()
        assert (live < nz // 4) if zm else (live == nz)
    # the TableFunction mirror hands out only the evaluated tiles, rows in batch order
    fn = CubitScanFunction(t, [0, 2, 3, ROW_ID], [3, 2], fs)
    local = fn.init_local()
    rows, c3 = [], []
    while True:
        chunk = fn.function(local)
        if len(chunk[0]) == 0:
            break
        rows.append(chunk[0])
        c3.append(chunk[1])
    rows = np.concatenate(rows)
    order = np.argsort(rows, kind="stable")
    ref = np.flatnonzero(mask) + BASE
    assert np.array_equal(rows[order], ref)
    assert np.array_equal(np.concatenate(c3)[order], cols[3][ref - BASE])
    t.close()


def test_random_filters_on_clustered_data(ctx):
    t, cols, vw = make_table(ctx)
    ocols = oracle_cols(cols, vw)
    rng = np.random.default_rng(11)
    skipped = 0
    for i in range(90):
        filters = {int(c): rand_filter(rng, int(c)) for c in rng.choice(4, size=rng.integers(1, 4), replace=False)}
        fs = F.TableFilterSet(filters)
        residual = rand_residual(rng) if rng.random() < 0.4 else None
        _, live, nz = check_scan(t, ocols, fs, residual, what=i)
        skipped += live < nz
        if i % 5 == 0:
            ref = O.table_scan(ocols, F.serialize(fs, residual), t.n_rows, row_base=BASE)
            assert t.count(fs, residual) == len(ref)
    assert skipped >= 10, skipped
    t.close()


def test_random_filters_on_clustered_data_with_mvcc(ctx):
    """The same fuzz under an MVCC delta that moves rows across zones: committed and writer
    updates on the clustered columns (values far from the zone's neighbours), deletes from two
    transactions and a hidden insert range. A patched leaf keeps its base leaf's zone classes
    except in the zones holding an update record; the visibility leaf has none — the skip stays
    exact for every view."""
    t, cols, vw = make_table(ctx, 3_000_017)
    n = t.n_rows
    rng = np.random.default_rng(29)
    writer = TXN_START + 21
    upd = {}
    # updates of the clustered columns sit in a few zones (the rest keep their classes)
    for c, (lo, hi), (r0, r1) in ((0, (0, 2600), (0, 400_000)), (1, (0, 160), (1_000_000, 1_300_000)),
                                  (2, (0, 50), (0, n))):
        rows = np.sort(r0 + rng.choice(r1 - r0, size=4_000, replace=False)).astype(np.int64)
        vals = rng.integers(lo, hi, len(rows)).astype(np.int64)
        vers = np.where(rng.random(len(rows)) < 0.5, np.uint64(3), np.uint64(writer)).astype(np.uint64)
        t.set_updates(c, rows, vals, vers)
        upd[c] = (rows, vals, vers)
    ocols = oracle_cols(cols, vw, upd)
    del_rows = np.sort(rng.choice(n, size=30_000, replace=False)).astype(np.int64)
    del_ids = np.where(rng.random(len(del_rows)) < 0.5, np.uint64(4), np.uint64(writer)).astype(np.uint64)
    t.set_deletes(del_rows, del_ids)
    deleted = np.full(n, np.uint64(2 ** 64 - 2), dtype=np.uint64)
    deleted[del_rows] = del_ids
    inserted = np.zeros(n, dtype=np.uint64)
    inserted[2_500_000:2_700_000] = 8  # an insert range committed at 8
    t.set_inserts(np.array([2_500_000]), np.array([2_700_000]), np.array([8], dtype=np.uint64))
    views = [(2, writer), (5, TXN_START + 22), (10, TXN_START + 23)]
    skipped = 0
    for i in range(45):
        filters = {int(c): rand_filter(rng, int(c)) for c in rng.choice(3, size=rng.integers(1, 3), replace=False)}
        fs = F.TableFilterSet(filters)
        residual = rand_residual(rng) if rng.random() < 0.3 else None
        start, tid = views[i % 3]
        tx = O.Mvcc(start, tid, inserted=inserted, deleted=deleted)
        _, live, nz = check_scan(t, ocols, fs, residual, txn=L.Txn(start, tid), tx=tx, what=(i, start, tid))
        skipped += live < nz
    assert skipped >= 3, skipped
    t.close()


def test_zones_follow_appends_merges_and_updates(ctx):
    n0 = 6_000_011
    t, cols, vw = make_table(ctx, n0)
    valid1 = np.unpackbits(vw.view(np.uint8), bitorder="little")[:n0].astype(bool)
    rng = np.random.default_rng(3)
    late = F.TableFilterSet({0: F.ConstantFilter(">=", 2500)})
    # warm the zone maps, then append rows that continue the clustering (and new keys)
    t.scan(late)
    for k, n_new in enumerate((1, 70_000, 400_003)):
        start = t.n_rows
        add, addv = clustered(n_new, 100 + k, start=start)
        add[0] = (add[0] + 20).astype(np.int32)  # values past the old maximum
        t.append({c: a for c, a in enumerate(add)}, validity={1: validity_from_mask(addv)})
        cols = [np.concatenate([a, b]) for a, b in zip(cols, add)]
        valid1 = np.concatenate([valid1, addv])
        vw = validity_from_mask(valid1)
        ocols = oracle_cols(cols, vw)
        ref, live, nz = check_scan(t, ocols, late, what=("append", n_new))
        assert len(ref) == int((cols[0] >= 2500).sum())
        assert live < nz
        check_scan(t, ocols, F.TableFilterSet({1: F.IsNullFilter()}), what=("append null", n_new))
    n = t.n_rows
    # updates move early rows of column 1 to the last values: a writer sees them, a reader not
    rows = np.sort(rng.choice(500_000, size=2_000, replace=False)).astype(np.int64)
    vals = np.full(len(rows), 400, dtype=np.int64)  # past every base value (max 324)
    writer = TXN_START + 9
    vers = np.where(np.arange(len(rows)) % 2 == 0, np.uint64(3), np.uint64(writer)).astype(np.uint64)
    t.set_updates(1, rows, vals, vers)
    ocols = oracle_cols(cols, vw, {1: (rows, vals, vers)})
    hi = F.TableFilterSet({1: F.ConstantFilter(">=", 350)})
    for start, tid in ((2, writer), (10, TXN_START + 10), (2, TXN_START + 11)):
        tx = O.Mvcc(start, tid)
        ref, _, _ = check_scan(t, ocols, hi, txn=L.Txn(start, tid), tx=tx, what=("update view", start, tid))
        expect = (start > 3) * (len(rows) // 2) + (tid == writer) * (len(rows) // 2)
        assert len(ref) == expect
    # merge the committed half: the base now holds 400 in early zones, which must be evaluated
    assert t.merge_updates(1, 5) == len(rows) // 2
    merged = cols[1].copy()
    merged[rows[vers == 3]] = 400
    valid_m = valid1.copy()
    valid_m[rows[vers == 3]] = True
    cols_m = [cols[0], merged, cols[2], cols[3]]
    keep = vers != 3
    ocols = oracle_cols(cols_m, validity_from_mask(valid_m), {1: (rows[keep], vals[keep], vers[keep])})
    ref, live, nz = check_scan(t, ocols, hi, txn=L.Txn(10, TXN_START + 12), tx=O.Mvcc(10, TXN_START + 12),
                               what="merged")
    assert len(ref) == len(rows) // 2 and live < nz
    # no transaction: the merged base alone (the writer's records are not applied)
    ref, _, _ = check_scan(t, oracle_cols(cols_m, validity_from_mask(valid_m)), hi, what="merged, no txn")
    assert len(ref) == len(rows) // 2
    assert n == t.n_rows
    t.close()
