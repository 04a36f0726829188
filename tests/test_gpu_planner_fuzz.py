"""Planner fuzz: random pushed TableFilterSets (constants, IS [NOT] NULL, per-column AND/OR)
plus random cross-column residual AND/OR trees, over columns with different index sets
(range, equality, range + bins, none → K0) and NULLs. Every plan — CONJ / DNF / CNF /
postfix forms, interval folding onto bins, multi-pass materialisation — must return exactly
the oracle's rows, with and without a transaction that sees deletes."""
import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from cubit_amd.table import Context, CubitTable
from oracle import oracle as O

pytestmark = pytest.mark.gpu

TXN_START = 4611686018427388000
CMPS = ["=", "!=", "<", "<=", ">", ">="]


@pytest.fixture(scope="module", params=[L.DECODE_AUTO, L.DECODE_RUNS, L.DECODE_PAIRS], ids=["auto", "runs", "pairs"])
def ctx(request):
    """Both decode kernels: at these sizes the automatic policy picks the pair-claimed one, so
    the run-claimed kernel (production above 2 tiles per workgroup) is forced once."""
    c = Context(0)
    c.set_decode_kernel(request.param)
    yield c
    c.close()


def rand_const_filter(rng, depth=0):
    r = rng.random()
    if depth < 2 and r < 0.25:
        kids = [rand_const_filter(rng, depth + 1) for _ in range(rng.integers(2, 4))]
        return F.ConjunctionAndFilter(kids) if rng.random() < 0.6 else F.ConjunctionOrFilter(kids)
    if r < 0.32:
        return F.IsNullFilter() if rng.random() < 0.5 else F.IsNotNullFilter()
    return F.ConstantFilter(CMPS[rng.integers(0, 6)], int(rng.integers(-5, 60)))


def rand_residual(rng, n_cols, depth=0):
    if depth < 2 and rng.random() < 0.5:
        kids = [rand_residual(rng, n_cols, depth + 1) for _ in range(rng.integers(2, 4))]
        return F.And(*kids) if rng.random() < 0.5 else F.Or(*kids)
    c = int(rng.integers(0, n_cols))
    if rng.random() < 0.1:
        return F.IsNull(c)
    return F.Cmp(c, CMPS[rng.integers(0, 6)], int(rng.integers(-5, 60)))


def test_random_filter_sets_match_oracle(ctx):
    rng = np.random.default_rng(2024)
    n = 400_003  # four tiles: pairs, a lone tile and a tail
    cols, ocols = [], []
    t = CubitTable(ctx, n, row_base=11)
    for c in range(4):
        data = rng.integers(0, 50, n).astype(np.int32 if c % 2 == 0 else np.int64)
        valid = rng.random(n) > (0.15 if c != 1 else 0.0)
        vw = validity_from_mask(valid) if c != 1 else None
        t.add_column(c, data, vw)
        cols.append(data)
        ocols.append(O.Column(data, vw))
    t.build_index(0, L.INDEX_RANGE)                       # exact range
    t.build_index(1, L.INDEX_EQUALITY)                    # equality
    t.build_index(2, L.INDEX_RANGE, [10, 20, 30, 40])     # binned range edges (K0 for others)
    t.build_index(2, L.INDEX_BINS, [0, 10, 20, 30, 40, 50])
    # column 3: no index → every constant goes through K0
    dels = np.arange(0, n, 7, dtype=np.int64)
    deleted = np.full(n, np.uint64(2 ** 64 - 2), dtype=np.uint64)
    deleted[dels] = 5
    for i in range(160):
        filters = {}
        for c in rng.choice(4, size=rng.integers(0, 4), replace=False):
            filters[int(c)] = rand_const_filter(rng)
        fs = F.TableFilterSet(filters)
        residual = rand_residual(rng, 4) if rng.random() < 0.5 else None
        plan = F.serialize(fs, residual)
        ref = O.table_scan(ocols, plan, n, row_base=11)
        got = t.scan(fs, residual)
        assert np.array_equal(got, ref), (i, fs, residual)
        if i % 4 == 0:
            if i == 0:
                t.set_deletes(dels, np.full(len(dels), 5, dtype=np.uint64))
            tx = O.Mvcc(10, TXN_START + 1, deleted=deleted)
            ref_t = O.table_scan(ocols, plan, n, row_base=11, tx=tx)
            got_t = t.scan(fs, residual, txn=L.Txn(10, TXN_START + 1))
            assert np.array_equal(got_t, ref_t), ("txn", i, fs, residual)


def test_random_filter_sets_with_updates_and_deletes(ctx):
    """The same fuzz with an MVCC delta: deletes from two transactions and updates on indexed
    columns (range, equality, bins) from a writer; the writer, a reader that predates it and
    a reader that sees the committed half must each get the oracle's rows."""
    rng = np.random.default_rng(77)
    n = 300_007
    writer = TXN_START + 5
    cols, data = [], []
    t = CubitTable(ctx, n)
    for c in range(3):
        d = rng.integers(0, 50, n).astype(np.int64)
        valid = rng.random(n) > 0.1
        vw = validity_from_mask(valid)
        t.add_column(c, d, vw)
        data.append((d, vw))
    t.build_index(0, L.INDEX_RANGE)
    t.build_index(1, L.INDEX_EQUALITY)
    t.build_index(2, L.INDEX_RANGE, [10, 20, 30, 40])
    t.build_index(2, L.INDEX_BINS, [0, 10, 20, 30, 40, 50])
    upd = {}
    for c in range(3):
        rows = np.sort(rng.choice(n, size=3000, replace=False)).astype(np.int64)
        vals = rng.integers(-5, 56, len(rows)).astype(np.int64)  # also outside the base statistics
        vers = np.where(rng.random(len(rows)) < 0.5, np.uint64(3), np.uint64(writer)).astype(np.uint64)
        t.set_updates(c, rows, vals, vers)
        upd[c] = (rows, vals, vers)
    ocols = [O.Column(d, vw, updates=upd[c]) for c, (d, vw) in enumerate(data)]
    del_rows = np.sort(rng.choice(n, size=20_000, replace=False)).astype(np.int64)
    del_ids = np.where(rng.random(len(del_rows)) < 0.5, np.uint64(4), np.uint64(writer)).astype(np.uint64)
    t.set_deletes(del_rows, del_ids)
    deleted = np.full(n, np.uint64(2 ** 64 - 2), dtype=np.uint64)
    deleted[del_rows] = del_ids
    views = [(2, writer), (2, TXN_START + 6), (10, TXN_START + 7)]
    for i in range(60):
        filters = {}
        for c in rng.choice(3, size=rng.integers(1, 4), replace=False):
            filters[int(c)] = rand_const_filter(rng)
        fs = F.TableFilterSet(filters)
        residual = rand_residual(rng, 3) if rng.random() < 0.4 else None
        plan = F.serialize(fs, residual)
        start, tid = views[i % 3]
        ref = O.table_scan(ocols, plan, n, tx=O.Mvcc(start, tid, deleted=deleted))
        got = t.scan(fs, residual, txn=L.Txn(start, tid))
        assert np.array_equal(got, ref), (i, start, tid, fs, residual)
