"""The multi-GPU path's partitioned scan on the HIP library, on one GPU.

bench.py --gpus N splits ONE TPC-H table into N order-range partitions (strong scaling), each
a `cubit_table` with row_base = the partition's first global row id. Here SF1 is split the
same way into 8 (and 3) partitions on the one GPU of the test box: every partition is scanned
by libcubitgpu, the per-partition results are concatenated in rank order (tile runs restored
to row order through each scan's tile directory) and compared with the whole-table oracle,
the reference's SF1 Q6 fingerprint and its Q6 revenue. Order-range partitions start at row
ids that are not multiples of 64, so every bitvector word boundary is off the global one.
"""
import numpy as np
import pytest

from conftest import lineitem, revenue_from_answer
from cubit_amd import _lib as L
from cubit_amd import datagen, parallel
from cubit_amd import filters as F
from cubit_amd.table import Context, CubitTable, runs_in_row_order
from oracle import oracle as O

pytestmark = pytest.mark.gpu

MONTHS = [F.date(y, m, 1) for y in range(1992, 1999) for m in range(1, 13)] + [F.date(1999, 1, 1)]
YEARS = [F.date(y, 1, 1) for y in range(1992, 2000)]


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def partition_tables(ctx, sf, world):
    """The bench's strong-scaling partitions of one table, all on this GPU."""
    out = []
    orders = datagen.tpch_orders(sf)
    for r in range(world):
        ob, oe = parallel.partition_orders(orders, r, world)
        li = datagen.tpch_lineitem(sf, ob, oe)
        t = CubitTable(ctx, li.n_rows, li.row_base)
        t.add_column(0, li.l_shipdate)
        t.add_column(1, li.l_discount)
        t.add_column(2, li.l_quantity)
        t.add_column(3, li.l_extendedprice)
        t.build_index(0, L.INDEX_RANGE, MONTHS)
        t.build_index(0, L.INDEX_BINS, YEARS)
        t.build_index(1, L.INDEX_RANGE)
        t.build_index(2, L.INDEX_RANGE)
        out.append((t, li))
    return out


@pytest.mark.parametrize("world", [8, 3])
def test_partitioned_q6_equals_whole_table(ctx, golden, world):
    parts = partition_tables(ctx, 1, world)
    bases = [li.row_base for _, li in parts]
    assert bases[0] == 0 and any(b % 64 for b in bases[1:])  # word boundaries off the global ones
    assert sum(li.n_rows for _, li in parts) == lineitem(1).n_rows
    fs = F.q6_filter_set()
    runs, ordered, counts = [], [], []
    for t, li in parts:
        # tile-run output (the bench's), restored to row order by the scan's directory
        raw = t.scan(fs, ordered=False)
        directory, _ = ctx.last_tiles()
        runs.append(runs_in_row_order(raw, directory))
        ordered.append(t.scan(fs, ordered=True))
        counts.append(t.count(fs))
        assert t.last_plan()[0] == 4  # year bin + 2 discount + 1 quantity leaves
    whole = lineitem(1)
    ref = O.table_scan([O.Column(whole.l_shipdate), O.Column(whole.l_discount), O.Column(whole.l_quantity)],
                       F.serialize(fs), whole.n_rows)
    got = np.concatenate(runs)
    assert np.array_equal(got, ref)
    assert np.array_equal(np.concatenate(ordered), ref)
    assert sum(counts) == len(ref)
    fp = golden["tpch"]["fingerprints"]["sf1_q6"]
    assert len(got) == fp["count"] and int(got.sum()) == fp["sum_rowid"]
    assert int(got.min()) == fp["min"] and int(got.max()) == fp["max"]
    assert O.xor_hash(got) == fp["xor_hash"]
    # each partition's row ids lie in its own global range
    for (t, li), r in zip(parts, runs):
        assert len(r) == 0 or (r.min() >= li.row_base and r.max() < li.row_base + li.n_rows)
    # Q6 revenue: the fused evaluate + probe-sum per partition, summed over the partitions
    total = 0
    for t, li in parts:
        rev, n = t.sum_product(3, 1, fs)
        total += rev
    assert total == revenue_from_answer(golden["tpch"]["q6_revenue"]["1"]["revenue"])
    for t, _ in parts:
        t.close()


def test_partitioned_probe_at_global_row_ids(ctx):
    """The probe of a partition takes global row ids (local + row_base), as the exchanged
    selection vectors carry them."""
    parts = partition_tables(ctx, 0.1, 4)
    fs = F.q6_filter_set()
    for t, li in parts[1:]:
        rows = t.scan(fs)
        d_rows = ctx.upload(rows)
        d_cnt = ctx.upload(np.array([len(rows)], dtype=np.uint64))
        out = ctx.alloc(max(len(rows), 1) * 8)
        t.probe(3, d_rows.addr, d_cnt.addr, len(rows), out.addr)
        assert np.array_equal(out.download(np.int64, len(rows)), li.l_extendedprice[rows - li.row_base])
    for t, _ in parts:
        t.close()


@pytest.mark.parametrize("world,tasks,stage_mb", [(8, 1, None), (8, 4, None), (3, 4, None), (8, 4, "0.15")])
def test_table_function_over_partitions(golden, world, tasks, stage_mb, monkeypatch):
    """One table-function scan over all partitions (cubit_scan_init_global_multi), each on its
    own context — as one process driving one device per partition would hold them, here all on
    device 0: one cursor in row order over every partition's windows (RowGroupCollection's
    NextParallelScan over all row groups, row_group_collection.cpp:174-224), each window copied
    from its own partition, batch index = the partition's first tile + its tile. The chunks
    equal the whole-table oracle, SF1's Q6 fingerprint and its revenue; every task's batch
    indexes ascend. stage_mb 0.15: one staging budget for the whole scan holds the first
    partitions' blocks (≈ 57 KB each), the rest are copied per window."""
    import threading

    if stage_mb is not None:
        monkeypatch.setenv("CUBIT_SCAN_STAGE_MB", stage_mb)

    from cubit_amd import scan_function as S
    from cubit_amd.scan_function import ROW_ID, CubitScanFunction

    ctxs = [Context(0) for _ in range(world)]
    orders = datagen.tpch_orders(1)
    parts = []
    for r in range(world):
        ob, oe = parallel.partition_orders(orders, r, world)
        li = datagen.tpch_lineitem(1, ob, oe)
        t = CubitTable(ctxs[r], li.n_rows, li.row_base)
        for c, arr in enumerate((li.l_shipdate, li.l_discount, li.l_quantity, li.l_extendedprice)):
            t.add_column(c, arr)
        t.build_index(0, L.INDEX_RANGE, MONTHS)
        t.build_index(1, L.INDEX_RANGE)
        t.build_index(2, L.INDEX_RANGE)
        parts.append((t, li))
    tables = [t for t, _ in parts]
    whole = lineitem(1)
    assert S.cardinality(tables) == (whole.n_rows, whole.n_rows)
    assert S.statistics(tables, 3) == (int(whole.l_extendedprice.min()), int(whole.l_extendedprice.max()), False, True)
    fn = CubitScanFunction(tables, [0, 1, 2, 3, ROW_ID], [4, 3, 1], F.q6_filter_set())
    assert fn.max_threads() >= min(tasks, 2)
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

    th = [threading.Thread(target=task, args=(k,)) for k in range(tasks)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    tile_base = np.cumsum([0] + [(li.n_rows + 131071) // 131072 for _, li in parts])
    chunks = []
    for seen in per_task.values():
        idx = [b for b, _ in seen]
        assert idx == sorted(idx)
        chunks += seen
    # batch index = the first tile (over the partitions' tiles) of the chunk's window: a chunk
    # lies in one partition, in tiles from its batch index up to the next batch index present
    bases = np.array([li.row_base for _, li in parts])
    bs = sorted({b for b, _ in chunks})
    nxt = {b: (bs[i + 1] if i + 1 < len(bs) else 1 << 62) for i, b in enumerate(bs)}
    for b, cols in chunks:
        p = np.searchsorted(bases, cols[0], side="right") - 1
        assert np.all(p == p[0])
        tiles = (cols[0] - bases[p[0]]) // 131072 + tile_base[p[0]]
        assert np.all(tiles >= b) and np.all(tiles < nxt[b])
    chunks.sort(key=lambda bc: (bc[0], bc[1][0][0]))
    rows = np.concatenate([c[0] for _, c in chunks])
    ref = O.table_scan([O.Column(whole.l_shipdate), O.Column(whole.l_discount), O.Column(whole.l_quantity)],
                       F.serialize(F.q6_filter_set()), whole.n_rows)
    assert np.array_equal(rows, ref)
    fp = golden["tpch"]["fingerprints"]["sf1_q6"]
    assert len(rows) == fp["count"] and int(rows.sum()) == fp["sum_rowid"] and O.xor_hash(rows) == fp["xor_hash"]
    price = np.concatenate([c[1] for _, c in chunks])
    disc = np.concatenate([c[2] for _, c in chunks])
    assert np.array_equal(price, whole.l_extendedprice[ref]) and np.array_equal(disc, whole.l_discount[ref])
    rev = int((price.astype(object) * disc.astype(object)).sum())
    assert rev == revenue_from_answer(golden["tpch"]["q6_revenue"]["1"]["revenue"])
    assert fn.progress() == pytest.approx(100.0)
    fn.close()
    with pytest.raises(L.CubitError):  # partitions out of row order
        CubitScanFunction(tables[::-1], [ROW_ID], None, F.q6_filter_set())
    for t in tables:
        t.close()
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("tasks", [1, 3])
def test_table_function_over_ragged_partitions(tasks):
    """cubit_scan_init_global_multi over partitions of every awkward kind, on two contexts: an
    empty one, one where nothing qualifies, one with NULL rows in the projected column (the
    others have none: the NULL-ness decision and the transfer width are per partition), one
    with a row base that is not a multiple of 64 and a single ragged tile, and a last one of
    several windows. Every row's value and NULL-ness equal numpy's; batch indexes ascend per
    task and lie in the partition's tiles."""
    import threading

    from cubit_amd.datagen import validity_from_mask
    from cubit_amd.scan_function import ROW_ID, CubitScanFunction

    rng = np.random.default_rng(11)
    sizes = [0, 70_000, 300_001, 77, 900_000]
    ctxs = [Context(0), Context(0)]
    bases, b = [], 5
    for n in sizes:
        bases.append(b)
        b += n + (3 if n == 77 else 0)  # a gap between two partitions' row ranges
    parts, cols = [], []
    for k, (n, base) in enumerate(zip(sizes, bases)):
        a = rng.integers(0, 100, n).astype(np.int32)
        if k == 1:
            a[:] = 500  # nothing passes a < 50
        v = rng.integers(-(1 << 35), 1 << 35, n).astype(np.int64)
        valid = rng.random(n) > 0.3 if k == 2 else np.ones(n, bool)
        t = CubitTable(ctxs[k % 2], n, base)
        t.add_column(0, a)
        t.add_column(1, v, validity_from_mask(valid) if k == 2 else None)
        if n:
            t.build_index(0, L.INDEX_RANGE)
        parts.append(t)
        cols.append((a, v, valid, base))
    fs = F.TableFilterSet({0: F.ConstantFilter("<", 50)})
    fn = CubitScanFunction(parts, [0, 1, ROW_ID], [2, 1], fs)
    out, lock = [], threading.Lock()

    def task():
        local = fn.init_local()
        last = -1
        while True:
            vals, masks = fn.function_validity(local)
            if len(vals[0]) == 0:
                return
            bi = fn.get_batch_index(local)
            assert bi >= last
            last = bi
            with lock:
                out.append((bi, vals, masks))

    th = [threading.Thread(target=task) for _ in range(tasks)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    out.sort(key=lambda x: (x[0], x[1][0][0]))
    rows = np.concatenate([o[1][0] for o in out])
    got_v = np.concatenate([o[1][1] for o in out])
    got_ok = np.concatenate([o[2][1] for o in out])
    want_rows, want_v, want_ok = [], [], []
    tile_base = 0
    for (a, v, valid, base), n in zip(cols, sizes):
        keep = np.flatnonzero(a < 50)
        want_rows.append(keep + base)
        want_v.append(np.where(valid[keep], v[keep], 0))
        want_ok.append(valid[keep])
        bs = sorted({bi for bi, _, _ in out})
        for bi, vals, _ in out:
            sel = (vals[0] >= base) & (vals[0] < base + n)
            if sel.any():  # a chunk lies in one partition, in its window's tiles
                assert sel.all()
                tiles = (vals[0] - base) // 131072 + tile_base
                later = [x for x in bs if x > bi]
                assert np.all(tiles >= bi) and np.all(tiles < (later[0] if later else 1 << 62))
        tile_base += (n + 131071) // 131072
    assert np.array_equal(rows, np.concatenate(want_rows))
    assert np.array_equal(got_ok, np.concatenate(want_ok)) and np.array_equal(got_v, np.concatenate(want_v))
    assert fn.progress() == pytest.approx(100.0)
    fn.close()
    for t in parts:
        t.close()
    for c in ctxs:
        c.close()
