"""HIP path vs the oracle on identical inputs — bit-exact row-id sets (and probe values).

Every test here calls libcubitgpu.so through the C ABI on the MI355X.
"""
import numpy as np
import pytest

from conftest import lineitem, revenue_from_answer
from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import uniform_i32, validity_from_mask
from cubit_amd.table import Context, CubitTable, padded_words, runs_in_row_order
from oracle import oracle as O

pytestmark = pytest.mark.gpu

TXN_START = 4611686018427388000


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def q6_table(ctx, li, index=True, encoding=L.INDEX_RANGE):
    t = CubitTable(ctx, li.n_rows, li.row_base)
    t.add_column(0, li.l_shipdate)
    t.add_column(1, li.l_discount)
    t.add_column(2, li.l_quantity)
    t.add_column(3, li.l_extendedprice)
    if index:
        # shipdate binned at month starts (Q6's year bounds are month starts: exact);
        # discount / quantity: every distinct value
        months = [F.date(y, m, 1) for y in range(1992, 1999) for m in range(1, 13)] + [F.date(1999, 1, 1)]
        t.build_index(0, L.INDEX_RANGE, months)
        t.build_index(1, encoding)
        t.build_index(2, encoding)
    return t


def oracle_q6(li):
    cols = [O.Column(li.l_shipdate), O.Column(li.l_discount), O.Column(li.l_quantity)]
    return O.table_scan(cols, F.serialize(F.q6_filter_set()), li.n_rows, li.row_base)


@pytest.mark.parametrize("sf", [0.01, 0.1])
@pytest.mark.parametrize("index", [True, False])
def test_q6_rowids_bit_exact(ctx, sf, index):
    li = lineitem(sf)
    t = q6_table(ctx, li, index=index)
    got = t.scan(F.q6_filter_set())
    assert np.array_equal(got, oracle_q6(li))
    if index:
        k, passes = t.last_plan()
        assert k == 5 and passes == 1  # range-encoded Q6 = 5 bitvectors, one fused pass


def test_q6_sf1_fingerprint_and_revenue(ctx, golden):
    li = lineitem(1)
    t = q6_table(ctx, li)
    fp = golden["tpch"]["fingerprints"]["sf1_q6"]
    rows = t.scan(F.q6_filter_set())
    assert len(rows) == fp["count"] and int(rows.sum()) == fp["sum_rowid"]
    assert O.xor_hash(rows) == fp["xor_hash"]
    assert np.array_equal(rows, oracle_q6(li))
    # K3: probe + fused sum on the device
    d_rows = ctx.upload(rows)
    d_cnt = ctx.upload(np.array([len(rows)], dtype=np.uint64))
    out = ctx.alloc(16)
    ep = ctx.upload(li.l_extendedprice)
    di = ctx.upload(li.l_discount)
    L.check(ctx.lib.cubit_gather_sum_product(ctx.handle, ep.ptr, di.ptr, d_rows.ptr, d_cnt.ptr, len(rows), 0,
                                             out.ptr))
    lo, hi = out.download(np.int64, 2)
    rev = (int(hi) << 64) + (int(lo) & (2 ** 64 - 1))
    assert rev == revenue_from_answer(golden["tpch"]["q6_revenue"]["1"]["revenue"])
    probe = ctx.alloc(len(rows) * 8)
    t.probe(3, d_rows.addr, d_cnt.addr, len(rows), probe.addr)
    assert np.array_equal(probe.download(np.int64, len(rows)), li.l_extendedprice[rows])


def test_sf1_equality_encoded_shipdate(ctx, golden):
    li = lineitem(1)
    t = CubitTable(ctx, li.n_rows)
    t.add_column(0, li.l_shipdate)
    t.build_index(0, L.INDEX_EQUALITY)
    nbv, nbytes = t.index_info(0)
    assert nbv == 2526
    fp = golden["tpch"]["fingerprints"]["sf1_shipdate_eq_1995_03_15"]
    fs = F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter("=", F.date(1995, 3, 15)),
                                                      F.IsNotNullFilter()])})
    rows = t.scan(fs)
    assert len(rows) == fp["count"] and int(rows.sum()) == fp["sum_rowid"]
    assert O.xor_hash(rows) == fp["xor_hash"]
    assert t.last_plan()[0] == 1


def test_synthetic_range_config2_small(ctx):
    n = 10_000_003
    v = uniform_i32(42, n, 1_000_000)
    t = CubitTable(ctx, n)
    t.add_column(0, v)
    t.build_index(0, L.INDEX_RANGE, [10_000])
    fs = F.TableFilterSet({0: F.ConstantFilter("<", 10_000)})
    got = t.scan(fs)
    assert np.array_equal(got, np.nonzero(v < 10_000)[0])
    assert t.last_plan() == (1, 1)


def test_or_tree_config4_small(ctx):
    n = 3_000_017
    cols = [uniform_i32(s, n, 1_000_000) for s in (1, 2, 3, 4)]
    t = CubitTable(ctx, n)
    for i, c in enumerate(cols):
        t.add_column(i, c)
        t.build_index(i, L.INDEX_RANGE, [100_000])
    tree = F.Or(F.And(F.Cmp(0, "<", 100_000), F.Cmp(1, "<", 100_000)),
                F.And(F.Cmp(2, "<", 100_000), F.Cmp(3, "<", 100_000)))
    got = t.scan(None, tree)
    ref = O.table_scan([O.Column(c) for c in cols], F.serialize(None, tree), n)
    assert np.array_equal(got, ref)
    assert t.last_plan() == (4, 1)


@pytest.mark.parametrize("n", [1, 63, 64, 65, 4095, 65535, 65536, 65537, 131_071, 131_072, 131_073, 200_001, 262_145])
def test_tails_and_dense_tiles(ctx, n):
    """Tail words, tile boundaries and a dense result (> LDS stage capacity per tile)."""
    rng = np.random.default_rng(n)
    a = rng.integers(0, 10, n).astype(np.int64)
    t = CubitTable(ctx, n, row_base=1000)
    t.add_column(0, a)
    t.build_index(0, L.INDEX_RANGE)
    for cmp, c in [("<", 9), (">=", 1), ("!=", 3), ("=", 0), (">", 100), ("<=", 9)]:
        fs = F.TableFilterSet({0: F.ConstantFilter(cmp, c)})
        ref = O.table_scan([O.Column(a)], F.serialize(fs), n, row_base=1000)
        assert np.array_equal(t.scan(fs), ref), (cmp, c)


def test_nulls_comparisons_and_null_filters(ctx):
    n = 300_000
    rng = np.random.default_rng(5)
    a = rng.integers(-50, 50, n).astype(np.int32)
    valid = rng.random(n) > 0.2
    vw = validity_from_mask(valid)
    t = CubitTable(ctx, n)
    t.add_column(0, a, vw)
    t.add_column(1, a)  # no index, no nulls: K0 path
    t.build_index(0, L.INDEX_RANGE)
    oc = [O.Column(a, vw), O.Column(a)]
    cases = [F.ConstantFilter("<", 0), F.ConstantFilter(">=", 10), F.ConstantFilter("!=", 3),
             F.ConstantFilter("=", -50), F.IsNullFilter(), F.IsNotNullFilter(),
             F.ConjunctionOrFilter([F.ConstantFilter("<", -40), F.IsNullFilter()]),
             F.ConjunctionAndFilter([F.ConstantFilter(">", -10), F.ConstantFilter("<=", 10), F.IsNotNullFilter()])]
    for f in cases:
        for col in (0, 1):
            fs = F.TableFilterSet({col: f})
            ref = O.table_scan(oc, F.serialize(fs), n)
            assert np.array_equal(t.scan(fs), ref), (f, col)


def test_equality_index_ranges_and_wide_or(ctx):
    n = 500_000
    rng = np.random.default_rng(9)
    a = rng.integers(0, 40, n).astype(np.int64)
    t = CubitTable(ctx, n)
    t.add_column(0, a)
    t.build_index(0, L.INDEX_EQUALITY)
    for f in [F.ConstantFilter("<", 5), F.ConstantFilter(">=", 30), F.ConstantFilter("<", 30),
              F.ConjunctionOrFilter([F.ConstantFilter("=", k) for k in range(0, 40, 3)])]:
        fs = F.TableFilterSet({0: f})
        ref = O.table_scan([O.Column(a)], F.serialize(fs), n)
        assert np.array_equal(t.scan(fs), ref), f


def test_k0_compare_bitvector_matches_oracle(ctx):
    n = 100_003
    rng = np.random.default_rng(2)
    for dt in (np.int32, np.int64):
        a = rng.integers(-1000, 1000, n).astype(dt)
        valid = rng.random(n) > 0.1
        vw = validity_from_mask(valid)
        da = ctx.upload(a)
        dv = ctx.upload(np.concatenate([vw, np.zeros(padded_words(n) - len(vw), dtype=np.uint64)]))
        out = ctx.alloc(padded_words(n) * 8)
        for cmp in range(6):
            L.check(ctx.lib.cubit_build_bitvector(ctx.handle, da.ptr, 0 if dt == np.int32 else 1, dv.ptr, n, cmp, 17,
                                                  out.ptr))
            got = out.download(np.uint64, padded_words(n))
            ref = O.build_bitvector(O.Column(a, vw), n, cmp, 17)
            assert np.array_equal(got[: len(ref)], ref)
            assert not got[len(ref):].any()


def test_low_level_eval_random_programs(ctx):
    """cubit_bitvector_eval vs the oracle bitmap evaluator on random programs / negations."""
    rng = np.random.default_rng(123)
    n = 777_777
    pw = padded_words(n)
    nw = (n + 63) // 64
    leaves = []
    dleaves = []
    for k in range(8):
        dens = rng.choice([0.02, 0.3, 0.9])
        w = validity_from_mask(rng.random(n) < dens)
        leaves.append(w)
        dleaves.append(ctx.upload(np.concatenate([w, np.zeros(pw - nw, dtype=np.uint64)])))
    import ctypes as C

    ptrs = (C.c_void_p * 8)(*[d.ptr.value for d in dleaves])
    out = ctx.alloc(n * 8)
    cnt = ctx.alloc(16)
    words = ctx.alloc(pw * 8)
    ops = [L.OP_AND, L.OP_OR, L.OP_ANDNOT]
    for trial in range(40):
        k = int(rng.integers(1, 9))
        neg = int(rng.integers(0, 1 << k))
        # random postfix over leaves 0..k-1
        prog, depth = [], 0
        leaf_i = 0
        while leaf_i < k or depth > 1:
            if leaf_i < k and (depth < 2 or rng.random() < 0.5):
                prog.append(leaf_i)
                leaf_i += 1
                depth += 1
            else:
                prog.append(int(rng.choice(ops)))
                depth -= 1
        p = (C.c_int32 * len(prog))(*prog)
        rc = ctx.lib.cubit_bitvector_eval(ctx.handle, ptrs, k, neg, p, len(prog), n, 5, out.ptr, n, cnt.ptr,
                                          words.ptr, L.SCAN_ORDERED if trial % 2 else 0)
        if rc == L.ERR_UNSUPPORTED:
            continue  # stack deeper than 4
        L.check(rc)
        ctx.check()
        c = int(cnt.download(np.uint64, 1)[0])
        ol = [(~leaves[i] if (neg >> i) & 1 else leaves[i]) for i in range(k)]
        ref_rows, ref_words = O.bitmap_eval(ol, prog, n, 5)
        assert c == len(ref_rows)
        got = out.download(np.int64, c)
        if trial % 2 == 0:
            d, _ = ctx.last_tiles()
            got = runs_in_row_order(got, d)
        assert np.array_equal(got, ref_rows)
        assert np.array_equal(words.download(np.uint64, nw), ref_words)


def test_tile_run_output_and_directory(ctx):
    """Default output order: ascending runs per 131,072-row tile, directory restores row
    order; the run multiset equals the oracle's row-id set (DuckDB parallel-scan semantics)."""
    li = lineitem(0.1)
    t = q6_table(ctx, li)
    raw = t.scan(F.q6_filter_set(), ordered=False)
    d, rows_per_tile = ctx.last_tiles()
    ref = oracle_q6(li)
    assert rows_per_tile == 131072
    assert len(d) * rows_per_tile >= li.n_rows
    assert int(d[:, 1].sum()) == len(raw) == len(ref)
    for i, (start, n) in enumerate(d):
        run = raw[int(start): int(start) + int(n)]
        assert np.all(np.diff(run) > 0)
        if n:
            assert run[0] >= i * rows_per_tile and run[-1] < (i + 1) * rows_per_tile
    assert np.array_equal(runs_in_row_order(raw, d), ref)
    assert np.array_equal(np.sort(raw), ref)


def test_capacity_is_respected_and_count_reported(ctx):
    n = 100_000
    a = np.arange(n, dtype=np.int64)
    t = CubitTable(ctx, n)
    t.add_column(0, a)
    with pytest.raises(L.CubitError):
        t.scan(F.TableFilterSet({0: F.ConstantFilter("<", 50_000)}), capacity=1000)
    assert t.count(F.TableFilterSet({0: F.ConstantFilter("<", 50_000)})) == 50_000


def test_mvcc_writer_reader_views_sf001(ctx, golden):
    """SURVEY §3-E scenario on the GPU: visibility bitvector (deletes) + patched quantity
    leaves (updates) → 1267 rows for the writer, 1191 for the concurrent reader."""
    li = lineitem(0.01)
    fp = golden["tpch"]["fingerprints"]["sf001_mvcc"]
    n = li.n_rows
    writer = TXN_START + 1
    upd_rows = np.arange(0, n, 7, dtype=np.int64)
    del_rows = np.arange(0, n, 11, dtype=np.int64)
    for index in (True, False):
        t = q6_table(ctx, li, index=index)
        t.set_deletes(del_rows, np.full(len(del_rows), writer, dtype=np.uint64))
        t.set_updates(2, upd_rows, np.full(len(upd_rows), 100), np.full(len(upd_rows), writer, dtype=np.uint64))
        w = t.scan(F.q6_filter_set(), txn=L.Txn(2, writer))
        r = t.scan(F.q6_filter_set(), txn=L.Txn(2, TXN_START + 2))
        assert len(w) == fp["writer_view"] and len(r) == fp["reader_view"]
        # exact sets vs the oracle
        deleted = np.full(n, np.uint64(2 ** 64 - 2), dtype=np.uint64)
        deleted[del_rows] = writer
        qty = O.Column(li.l_quantity, updates=(upd_rows, np.full(len(upd_rows), 100, dtype=np.int64),
                                               np.full(len(upd_rows), writer, dtype=np.uint64)))
        cols = [O.Column(li.l_shipdate), O.Column(li.l_discount), qty]
        plan = F.serialize(F.q6_filter_set())
        assert np.array_equal(w, O.table_scan(cols, plan, n, tx=O.Mvcc(2, writer, deleted=deleted)))
        assert np.array_equal(r, O.table_scan(cols, plan, n, tx=O.Mvcc(2, TXN_START + 2, deleted=deleted)))
        # probe sees the writer's value
        d_rows = ctx.upload(w)
        d_cnt = ctx.upload(np.array([len(w)], dtype=np.uint64))
        pr = ctx.alloc(len(w) * 8)
        t.probe(2, d_rows.addr, d_cnt.addr, len(w), pr.addr, txn=L.Txn(2, writer))
        assert np.array_equal(pr.download(np.int64, len(w)), O.fetch(qty, w, tx=O.Mvcc(2, writer)))


def test_visibility_bitvector_cache_across_snapshots(ctx):
    """Committed deletes at ids 5 / 20 / 40 and one uncommitted (writer) delete set; a
    sequence of snapshots that reuses, rebuilds and bypasses the cached visibility bitvector
    must match the oracle at every step (chunk_info.cpp:11-19 visibility rule)."""
    n = 400_000
    a = uniform_i32(7, n, 1000)
    t = CubitTable(ctx, n)
    t.add_column(0, a)
    t.build_index(0, L.INDEX_RANGE, [100, 500])
    rng = np.random.default_rng(3)
    rows = rng.choice(n, size=40_000, replace=False).astype(np.int64)
    writer = TXN_START + 9
    ids = np.array([5, 20, 40, writer], dtype=np.uint64)[rng.integers(0, 4, len(rows))]
    fs = F.TableFilterSet({0: F.ConstantFilter("<", 500)})
    plan = F.serialize(fs)

    def check(start, tid):
        got = t.scan(fs, txn=L.Txn(start, tid))
        deleted = np.full(n, np.uint64(2 ** 64 - 2), dtype=np.uint64)
        deleted[rows] = ids
        ref = O.table_scan([O.Column(a)], plan, n, tx=O.Mvcc(start, tid, deleted=deleted))
        assert np.array_equal(got, ref), (start, tid)

    t.set_deletes(rows, ids)
    for start, tid in ((10, TXN_START + 1), (10, TXN_START + 2), (30, TXN_START + 3), (3, TXN_START + 4),
                       (50, writer), (50, TXN_START + 5), (10, TXN_START + 6)):
        check(start, tid)
    # replacing the delete list invalidates the cached bitvector
    ids = np.full(len(rows), 5, dtype=np.uint64)
    t.set_deletes(rows, ids)
    check(10, TXN_START + 7)


def test_insert_versions_and_deletes_across_snapshots(ctx):
    """Appended row ranges carry insert ids (ChunkConstantInfo::insert_id / ChunkVectorInfo::
    inserted): committed before the reader (3), after it (20, 45) and uncommitted (writer).
    With deletes beside them, every snapshot — other readers, the inserting writer, later
    readers — sees exactly the oracle's rows (UseInsertedVersion, chunk_info.cpp:11-19), and
    the cached visibility bitvector follows the snapshots."""
    li = lineitem(0.1)
    n = li.n_rows
    t = q6_table(ctx, li)
    writer = TXN_START + 5
    cuts = [n - 60_000, n - 45_001, n - 30_000, n - 12_345, n]
    b = np.array(cuts[:-1], dtype=np.int64)
    e = np.array(cuts[1:], dtype=np.int64)
    ins_ids = np.array([3, 20, writer, 45], dtype=np.uint64)
    rng = np.random.default_rng(12)
    del_rows = rng.choice(n, size=5_000, replace=False).astype(np.int64)
    del_ids = np.array([4, 25, writer], dtype=np.uint64)[rng.integers(0, 3, len(del_rows))]
    inserted = np.zeros(n, dtype=np.uint64)
    for lo, hi, i in zip(b, e, ins_ids):
        inserted[lo:hi] = i
    deleted = np.full(n, np.uint64(2 ** 64 - 2), dtype=np.uint64)
    cols = [O.Column(li.l_shipdate), O.Column(li.l_discount), O.Column(li.l_quantity)]
    plan = F.serialize(F.q6_filter_set())

    def check(start, tid, with_deletes):
        got = t.scan(F.q6_filter_set(), txn=L.Txn(start, tid))
        ref = O.table_scan(cols, plan, n, row_base=li.row_base,
                           tx=O.Mvcc(start, tid, inserted=inserted, deleted=deleted))
        assert np.array_equal(got, ref), (start, tid, with_deletes, len(got), len(ref))

    t.set_inserts(b[::-1], e[::-1], ins_ids[::-1])  # any order; disjoint
    snaps = ((10, TXN_START + 1), (10, writer), (30, TXN_START + 2), (10, TXN_START + 3), (50, TXN_START + 4),
             (2, TXN_START + 6), (50, writer))
    for start, tid in snaps:
        check(start, tid, False)
    t.set_deletes(del_rows, del_ids)
    deleted[del_rows] = del_ids
    for start, tid in snaps:
        check(start, tid, True)
    with pytest.raises(L.CubitError):
        t.set_inserts(np.array([0, 5]), np.array([10, 20]), np.array([1, 2]))  # overlap
    with pytest.raises(L.CubitError):
        t.set_inserts(np.array([n - 1]), np.array([n + 1]), np.array([1]))  # past the partition
    t.close()


def test_patched_leaf_cache_across_snapshots(ctx):
    """Committed updates at versions 5 / 20 / 40 plus an uncommitted writer's: patched leaves
    are cached per (predicate, visible version prefix); snapshots that reuse, rebuild and
    bypass the cache, an index rebuild and a new update list all match the oracle."""
    n = 300_000
    a = uniform_i32(21, n, 1000).astype(np.int64)
    t = CubitTable(ctx, n)
    t.add_column(0, a)
    t.build_index(0, L.INDEX_RANGE)
    rng = np.random.default_rng(8)
    rows = rng.choice(n, size=20_000, replace=False).astype(np.int64)
    writer = TXN_START + 3
    vers = np.array([5, 20, 40, writer], dtype=np.uint64)[rng.integers(0, 4, len(rows))]
    vals = rng.integers(0, 1000, len(rows)).astype(np.int64)
    fss = [F.TableFilterSet({0: F.ConstantFilter("<", 300)}),
           F.TableFilterSet({0: F.ConstantFilter("=", 17)}),
           F.TableFilterSet({0: F.ConstantFilter(">=", 950)})]

    def check(start, tid):
        col = O.Column(a, updates=(rows, vals, vers))
        for fs in fss:
            got = t.scan(fs, txn=L.Txn(start, tid))
            ref = O.table_scan([col], F.serialize(fs), n, tx=O.Mvcc(start, tid))
            assert np.array_equal(got, ref), (start, tid)

    t.set_updates(0, rows, vals, vers)
    snaps = ((10, TXN_START + 1), (10, TXN_START + 2), (30, writer), (30, TXN_START + 4), (50, TXN_START + 5),
             (10, TXN_START + 6), (3, TXN_START + 7))
    for st, tid in snaps:
        check(st, tid)
    t.build_index(0, L.INDEX_RANGE, [17, 18, 300, 950])  # new leaves: cached patches dropped
    for st, tid in snaps[:3]:
        check(st, tid)
    vals = (vals + 500) % 1000
    t.set_updates(0, rows, vals, vers)  # new update list
    for st, tid in snaps[:3]:
        check(st, tid)
    t.close()


def test_empty_partition(ctx):
    """An empty table (or a rank whose row range is empty): columns, indexes, MVCC lists and
    every scan form are accepted and return no rows / a zero sum without a launch."""
    from cubit_amd.scan_function import CubitScanFunction

    t = CubitTable(ctx, 0, row_base=100)
    t.add_column(0, np.zeros(0, dtype=np.int32))
    t.add_column(1, np.zeros(0, dtype=np.int64))
    t.add_column(2, np.zeros(0, dtype=np.int64))
    t.add_column(3, np.zeros(0, dtype=np.int64))
    t.build_index(0, L.INDEX_RANGE, [F.date(1994, 1, 1), F.date(1995, 1, 1)])
    t.build_index(1, L.INDEX_RANGE)
    t.build_index(2, L.INDEX_EQUALITY)
    t.set_deletes(np.zeros(0, np.int64), np.zeros(0, np.uint64))
    for txn in (None, L.Txn(10, TXN_START + 1)):
        assert len(t.scan(F.q6_filter_set(), txn=txn)) == 0
        assert len(t.scan(F.q6_filter_set(), txn=txn, ordered=False)) == 0
        assert t.count(F.q6_filter_set(), txn=txn) == 0
        assert t.count(None, txn=txn) == 0
        assert t.sum_product(3, 1, F.q6_filter_set(), txn=txn)[0] == 0
    sf = CubitScanFunction(t, [0, 1, 3], filter_set=F.q6_filter_set())
    loc = sf.init_local()
    assert all(len(c) == 0 for c in sf.function(loc))  # the first chunk is empty: FINISHED
    assert sf.progress() >= 0.0
    sf.close()
    t.close()


def test_q6_with_year_bins_reads_four_bitvectors(ctx, golden):
    """A binned index (year edges) beside the month range index: Q6's one-year shipdate range
    reads one bin instead of two range bitvectors (K 5 → 4); rows identical."""
    li = lineitem(0.1)
    t = q6_table(ctx, li)
    years = [F.date(y, 1, 1) for y in range(1992, 2000)]
    t.build_index(0, L.INDEX_BINS, years)
    got = t.scan(F.q6_filter_set())
    assert np.array_equal(got, oracle_q6(li))
    k, passes = t.last_plan()
    assert k == 4 and passes == 1


@pytest.mark.parametrize("with_range", [True, False])
def test_bins_index_intervals_vs_oracle(ctx, with_range):
    n = 300_007
    a = uniform_i32(11, n, 1000).astype(np.int64)
    valid = np.random.default_rng(5).random(n) > 0.05
    t = CubitTable(ctx, n)
    t.add_column(0, a, validity_from_mask(valid))
    if with_range:
        t.build_index(0, L.INDEX_RANGE, [100, 200, 500, 900])
    edges = [0, 100, 200, 300, 500, 700, 1000]
    t.build_index(0, L.INDEX_BINS, edges)
    col = O.Column(a, validity_from_mask(valid))
    cases = [((">=", 100), ("<", 200)), ((">=", 200), ("<", 700)), ((">", 99), ("<=", 299)), ((">=", 150), ("<", 300)),
             ((">=", 0), ("<", 1000)), ((">=", 500),), (("<", 300),), (("=", 5),), ((">=", 700), ("<", 100)),
             ((">=", 300), ("<", 500), ("<", 400))]
    for c in cases:
        filt = F.ConstantFilter(*c[0]) if len(c) == 1 else F.ConjunctionAndFilter([F.ConstantFilter(*x) for x in c])
        fs = F.TableFilterSet({0: filt})
        got = t.scan(fs)
        ref = O.table_scan([col], F.serialize(fs), n)
        assert np.array_equal(got, ref), c
    # a bin leaf patched for an update the transaction sees
    rows = np.arange(0, n, 13, dtype=np.int64)
    t.set_updates(0, rows, np.full(len(rows), 150), np.full(len(rows), TXN_START + 1, dtype=np.uint64))
    fs = F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", 100), F.ConstantFilter("<", 200)])})
    got = t.scan(fs, txn=L.Txn(2, TXN_START + 1))
    colu = O.Column(a, validity_from_mask(valid), updates=(rows, np.full(len(rows), 150, dtype=np.int64),
                                                           np.full(len(rows), TXN_START + 1, dtype=np.uint64)))
    ref = O.table_scan([colu], F.serialize(fs), n, tx=O.Mvcc(2, TXN_START + 1))
    assert np.array_equal(got, ref)


def test_index_build_statistics_on_device(ctx):
    """Distinct keys come from the device presence bitmap: negative values, NULLs ignored,
    one bitvector per distinct value (range drops the minimum); wide spans sort their keys."""
    n = 200_003
    rng = np.random.default_rng(21)
    a = rng.choice(np.array([-70000, -3, 0, 5, 9, 123456], dtype=np.int64), n)
    valid = rng.random(n) > 0.3
    a_null_only = a.copy()
    a_null_only[~valid] = 777  # a value present only under NULLs must not become a key
    t = CubitTable(ctx, n)
    t.add_column(0, a_null_only, validity_from_mask(valid))
    t.build_index(0, L.INDEX_EQUALITY)
    assert t.index_info(0)[0] == 6
    t.build_index(0, L.INDEX_RANGE)
    assert t.index_info(0)[0] == 5
    col = O.Column(a_null_only, validity_from_mask(valid))
    for c in (-70000, -3, 0, 5, 9, 123456, 777):
        for cmp in ("<", "=", ">="):
            fs = F.TableFilterSet({0: F.ConstantFilter(cmp, c)})
            assert np.array_equal(t.scan(fs), O.table_scan([col], F.serialize(fs), n)), (cmp, c)
    # a span of 2^32 or more: distinct keys by a host sort, refused above 65,536 of them
    many = np.arange(70_001, dtype=np.int64) << 20
    t3 = CubitTable(ctx, len(many))
    t3.add_column(0, many)
    with pytest.raises(Exception, match="distinct values over a span"):
        t3.build_index(0, L.INDEX_RANGE)
    t3.close()
    wide = np.array([-(2 ** 62), 2 ** 62] * 10, dtype=np.int64)
    t2 = CubitTable(ctx, len(wide))
    t2.add_column(0, wide)
    t2.build_index(0, L.INDEX_EQUALITY)
    assert t2.index_info(0)[0] == 2
    t2.build_index(0, L.INDEX_RANGE, [0])  # explicit keys
    fs = F.TableFilterSet({0: F.ConstantFilter("<", 0)})
    assert np.array_equal(t2.scan(fs), np.arange(0, 20, 2))


@pytest.mark.parametrize("sf", [0.1, 1.0])
def test_fused_q6_revenue(ctx, golden, sf):
    """SELECT sum(l_extendedprice*l_discount) WHERE <Q6> in one fused pass: the reference's
    answer file exactly, with l_discount decoded from its range index (3 values) and gathered."""
    li = lineitem(sf)
    t = q6_table(ctx, li)
    t.build_index(0, L.INDEX_BINS, [F.date(y, 1, 1) for y in range(1992, 2000)])
    want = revenue_from_answer(golden["tpch"]["q6_revenue"]["1" if sf == 1.0 else str(sf)]["revenue"])
    rev, n = t.sum_product(3, 1, F.q6_filter_set())
    assert rev == want and n == len(oracle_q6(li))
    assert t.last_sum_decode() == 3
    rev2, n2 = t.sum_product(3, 1, F.q6_filter_set(), gather_b=True)
    assert rev2 == want and n2 == n
    assert t.last_sum_decode() == 0


def test_fused_sum_product_nulls_mvcc_and_fallback(ctx):
    n = 250_000
    rng = np.random.default_rng(31)
    a = rng.integers(-10_000, 10_000, n).astype(np.int64)
    b = rng.integers(0, 12, n).astype(np.int64)
    va = rng.random(n) > 0.1
    t = CubitTable(ctx, n)
    t.add_column(0, a, validity_from_mask(va))
    t.add_column(1, b)
    t.build_index(1, L.INDEX_RANGE)
    fs = F.TableFilterSet({1: F.ConjunctionAndFilter([F.ConstantFilter(">=", 3), F.ConstantFilter("<=", 5)])})
    rows = O.table_scan([O.Column(a, validity_from_mask(va)), O.Column(b)], F.serialize(fs), n)
    keep = rows[va[rows]]
    want = int((a[keep].astype(object) * b[keep].astype(object)).sum())
    for gather in (False, True):
        got, cnt = t.sum_product(0, 1, fs, gather_b=gather)
        assert got == want and cnt == len(rows)
        assert t.last_sum_decode() == (0 if gather else 3)
    # deletes visible to the reader: fused path with the visibility leaf
    dels = np.arange(0, n, 5, dtype=np.int64)
    t.set_deletes(dels, np.full(len(dels), 3, dtype=np.uint64))
    alive = np.ones(n, dtype=bool)
    alive[dels] = False
    keep2 = keep[alive[keep]]
    want2 = int((a[keep2].astype(object) * b[keep2].astype(object)).sum())
    got, _ = t.sum_product(0, 1, fs, txn=L.Txn(10, TXN_START + 1))
    assert got == want2
    # visible updates on b → scan + probe + sum fallback (b NOT NULL, a has NULLs → refused)
    t2 = CubitTable(ctx, n)
    t2.add_column(0, a)
    t2.add_column(1, b)
    t2.build_index(1, L.INDEX_RANGE)
    up = np.arange(0, n, 9, dtype=np.int64)
    t2.set_updates(1, up, np.full(len(up), 4), np.full(len(up), TXN_START + 1, dtype=np.uint64))
    b2 = b.copy()
    b2[up] = 4
    rows2 = np.nonzero((b2 >= 3) & (b2 <= 5))[0]
    want3 = int((a[rows2].astype(object) * b2[rows2].astype(object)).sum())
    got, cnt = t2.sum_product(0, 1, fs, txn=L.Txn(2, TXN_START + 1))
    assert got == want3 and cnt == len(rows2)


def test_index_save_and_load(ctx, tmp_path):
    """Persisted indexes (range, equality, bins) load into a fresh partition and answer the
    same scans; a file for another partition size or a foreign file is refused."""
    li = lineitem(0.01)
    t = q6_table(ctx, li)
    years = [F.date(y, 1, 1) for y in range(1992, 2000)]
    t.build_index(0, L.INDEX_BINS, years)
    for col, enc in ((0, L.INDEX_RANGE), (0, L.INDEX_BINS), (1, L.INDEX_RANGE), (2, L.INDEX_RANGE)):
        t.save_index(col, enc, tmp_path / f"c{col}_{enc}.cubitix")
    t2 = CubitTable(ctx, li.n_rows, li.row_base)
    for c, arr in enumerate((li.l_shipdate, li.l_discount, li.l_quantity, li.l_extendedprice)):
        t2.add_column(c, arr)
    for f in sorted(tmp_path.glob("*.cubitix")):
        col = int(f.name[1])
        t2.load_index(col, f)
    assert t2.index_info(0) == t.index_info(0) and t2.index_info(2) == t.index_info(2)
    got = t2.scan(F.q6_filter_set())
    assert np.array_equal(got, oracle_q6(li))
    assert t2.last_plan() == (4, 1)
    t3 = CubitTable(ctx, li.n_rows - 1)
    t3.add_column(0, li.l_shipdate[:-1])
    with pytest.raises(Exception, match="another size"):
        t3.load_index(0, tmp_path / "c0_0.cubitix")
    junk = tmp_path / "junk.bin"
    junk.write_bytes(b"x" * 200)
    with pytest.raises(Exception, match="not a cubit index"):
        t2.load_index(0, junk)


def test_concurrent_scans_share_a_context(ctx):
    """DuckDB's pipeline threads call the scan concurrently (pipeline.cpp:113-125): scans from
    four threads on one context and table, each with its own output buffers and predicate,
    are each bit-exact (calls serialise on the context's mutex, the GPU work on its stream)."""
    import threading

    li = lineitem(0.01)
    t = q6_table(ctx, li)
    cols = [O.Column(li.l_shipdate), O.Column(li.l_discount), O.Column(li.l_quantity)]
    qty = [1200, 2400, 3600, 4800]
    want = {}
    for q in qty:
        fs = F.TableFilterSet()
        fs.push_filter(0, F.ConstantFilter(">=", F.date(1994, 1, 1)))
        fs.push_filter(0, F.ConstantFilter("<", F.date(1995, 1, 1)))
        fs.push_filter(2, F.ConstantFilter("<", q))
        want[q] = (fs, O.table_scan(cols, F.serialize(fs), li.n_rows, row_base=li.row_base))
    errors = []

    def worker(q):
        try:
            fs, ref = want[q]
            for _ in range(6):
                got = t.scan(fs, ordered=bool(q % 2400 == 0))
                if not np.array_equal(np.sort(got), ref):
                    errors.append((q, len(got), len(ref)))
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((q, repr(e)))

    th = [threading.Thread(target=worker, args=(q,)) for q in qty]
    for x in th:
        x.start()
    for x in th:
        x.join()
    t.close()
    assert not errors, errors


@pytest.mark.parametrize("n", [80_000_017, 140_000_003])
def test_mid_size_grids_scan_count_sum(ctx, n):
    """Partitions of 611 and 1,069 tiles: the decode grid takes one pair per workgroup
    (tiles / 2) below 2 tiles per workgroup and the full persistent grid above; the claim
    ticket's arrivals carry every workgroup's rows across all eight arrival groups. Scan
    (tile runs and ordered), count(*) and the fused sum against numpy on the same rows."""
    v = uniform_i32(7, n, 1_000_000)
    rng = np.random.default_rng(n)
    a = rng.integers(-1_000_000, 1_000_000, n).astype(np.int64)
    b = rng.integers(0, 100, n).astype(np.int64)
    t = CubitTable(ctx, n, row_base=5)
    t.add_column(0, v)
    t.add_column(1, a)
    t.add_column(2, b)
    t.build_index(0, L.INDEX_RANGE, [20_000])
    fs = F.TableFilterSet({0: F.ConstantFilter("<", 20_000)})
    want = np.nonzero(v < 20_000)[0]
    got = t.scan(fs, ordered=False)
    directory, _ = ctx.last_tiles()
    assert int(directory[:, 1].sum()) == len(want)
    assert np.array_equal(runs_in_row_order(got, directory), want + 5)
    assert np.array_equal(t.scan(fs), want + 5)
    assert t.count(fs) == len(want)
    rev, cnt = t.sum_product(1, 2, fs, gather_b=True)
    assert cnt == len(want)
    assert rev == int((a[want].astype(object) * b[want].astype(object)).sum())
    t.close()


@pytest.mark.parametrize("dtype", [np.int32, np.int64])
def test_candidate_check_off_key_constants(ctx, dtype):
    """Constants that are not keys of an edge-keyed range index: each comparison reads the
    constant's bin [k_lo, k_hi) on the raw column (candidate check), including the open bins
    below the first and above the last key, NULL rows, EQ / NE off the keys, and a bin too
    wide for the check (K0 instead). Every result equals the oracle's, also with updates
    visible to the reader (the candidate leaf is patched like any value leaf)."""
    n = 300_001
    rng = np.random.default_rng(77)
    a = rng.integers(-50, 1000, n).astype(dtype)
    valid = rng.random(n) > 0.1
    t = CubitTable(ctx, n, row_base=3)
    t.add_column(0, a, validity_from_mask(valid))
    t.build_index(0, L.INDEX_RANGE, list(range(100, 1000, 100)))
    t2 = CubitTable(ctx, n, row_base=3)  # one key: the bin above it spans ~90 % of the values → K0
    t2.add_column(0, a, validity_from_mask(valid))
    t2.build_index(0, L.INDEX_RANGE, [50])
    col = O.Column(a, validity_from_mask(valid))
    consts = [-51, -50, -7, 0, 99, 100, 101, 150, 199, 555, 900, 901, 999, 1000, 1200]
    for c in consts:
        for cmp in ("<", "<=", ">", ">=", "=", "!="):
            fs = F.TableFilterSet({0: F.ConstantFilter(cmp, c)})
            ref = O.table_scan([col], F.serialize(fs), n, row_base=3)
            assert np.array_equal(t.scan(fs), ref), (c, cmp)
            assert np.array_equal(t2.scan(fs), ref), (c, cmp, "wide bin")
    # Q6-shaped interval off the keys, and updates visible to the reader
    fs = F.TableFilterSet()
    fs.push_filter(0, F.ConstantFilter(">=", 123))
    fs.push_filter(0, F.ConstantFilter("<", 456))
    assert np.array_equal(t.scan(fs), O.table_scan([col], F.serialize(fs), n, row_base=3))
    rows = rng.choice(n, size=5_000, replace=False).astype(np.int64)
    vals = rng.integers(-50, 1000, len(rows)).astype(np.int64)
    vers = np.full(len(rows), 5, dtype=np.uint64)
    t.set_updates(0, rows, vals, vers)
    ucol = O.Column(a, validity_from_mask(valid), updates=(rows, vals, vers))
    for c, cmp in ((150, "<"), (555, ">="), (901, "=")):
        fs = F.TableFilterSet({0: F.ConstantFilter(cmp, c)})
        ref = O.table_scan([ucol], F.serialize(fs), n, row_base=3, tx=O.Mvcc(10, TXN_START + 1))
        assert np.array_equal(t.scan(fs, txn=L.Txn(10, TXN_START + 1)), ref), (c, cmp)
    t.close()
    t2.close()


@pytest.mark.parametrize("width", [1, 2, 3, 4])
@pytest.mark.parametrize("shift", [0, 1])
@pytest.mark.parametrize("n", [1, 7, 8, 9, 4099, 1_000_003])
def test_narrow_checked_round_trips(ctx, width, shift, n):
    """cubit_narrow_checked (the table function's transfer compaction): value - offset as an
    unsigned 1 / 2 / 3 / 4-byte little-endian integer, exact for every value in range, the overflow flag clear; one
    value past the range sets it. shift = 1 puts both operands off 16-byte alignment (the
    one-value-per-store form); lengths around the 8-value packing cover the tail; max_n below the
    count leaves the rest untouched."""
    rng = np.random.default_rng(n * 7 + width + shift)
    for offset in (-12345, 2 ** 40):
        vals = offset + rng.integers(0, 2 ** (8 * width), n, dtype=np.uint64).astype(np.int64)
        vals[0] = offset + 2 ** (8 * width) - 1  # the top of the range
        d_in = ctx.upload(np.concatenate([np.zeros(shift, np.int64), vals]))
        d_cnt = ctx.upload(np.array([n], np.uint64))
        out = ctx.upload(np.full((n + 1) * width, 0xAB, np.uint8))
        flag = ctx.upload(np.zeros(4, np.uint32))
        def run(max_n):
            L.check(ctx.lib.cubit_narrow_checked(ctx.handle, d_in.addr + 8 * shift, d_cnt.ptr, max_n, offset, width,
                                                 out.addr + width * shift, flag.ptr))
            ctx.sync()
            raw = out.download(np.uint8, (n + 1) * width)[width * shift:width * shift + n * width]
            by = raw.reshape(n, width).astype(np.uint64)
            vals_out = sum(by[:, k] << np.uint64(8 * k) for k in range(width))
            return vals_out, int(flag.download(np.uint32, 1)[0])

        got, bad = run(n)
        assert bad == 0
        assert np.array_equal(got.astype(np.int64) + offset, vals), (width, shift, n, offset)
        if n > 8:  # max_n below the count: only the first max_n written
            out.free()
            out = ctx.upload(np.full((n + 1) * width, 0xAB, np.uint8))
            got, _ = run(n // 2)
            assert np.array_equal(got[:n // 2].astype(np.int64) + offset, vals[:n // 2])
            assert (got[n // 2:] == sum(0xAB << (8 * k) for k in range(width))).all()
        vals[n - 1] = offset + 2 ** (8 * width)  # one past the range
        d_in.free()
        d_in = ctx.upload(np.concatenate([np.zeros(shift, np.int64), vals]))
        assert run(n)[1] == 1
