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
