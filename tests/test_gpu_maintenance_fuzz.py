"""Maintenance fuzz: a random sequence of appends (ragged sizes, NULLs, values outside the
index statistics, insert ids), update lists (chains of committed versions and a writer's
uncommitted tail), merges of the committed prefix below a horizon, delete lists and scans —
against a host model of the table that the oracle (cpu_ref.c) scans. Every scan, for several
snapshots, must return exactly the oracle's rows; random filter sets and residual trees run
over range (every value), equality, edge-keyed range + bins and unindexed columns.

`run(ctx, seed, n_ops, n0)` is shared with scripts/maintenance_soak.py (long runs).
"""
import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from cubit_amd.table import Context, CubitTable
from oracle import oracle as O

TXN_START = 4611686018427388000
WRITER = TXN_START + 5
NOT_DELETED = np.uint64(2 ** 64 - 2)
CMPS = ["=", "!=", "<", "<=", ">", ">="]
DTYPES = [np.int32, np.int64, np.int64, np.int32]


def rand_const_filter(rng, depth=0):
    r = rng.random()
    if depth < 2 and r < 0.25:
        kids = [rand_const_filter(rng, depth + 1) for _ in range(rng.integers(2, 4))]
        return F.ConjunctionAndFilter(kids) if rng.random() < 0.6 else F.ConjunctionOrFilter(kids)
    if r < 0.3:
        return F.IsNullFilter() if rng.random() < 0.5 else F.IsNotNullFilter()
    return F.ConstantFilter(CMPS[rng.integers(0, 6)], int(rng.integers(-8, 62)))


def rand_residual(rng, depth=0):
    if depth < 2 and rng.random() < 0.5:
        kids = [rand_residual(rng, depth + 1) for _ in range(rng.integers(2, 4))]
        return F.And(*kids) if rng.random() < 0.5 else F.Or(*kids)
    c = int(rng.integers(0, 4))
    if rng.random() < 0.1:
        return F.IsNull(c)
    return F.Cmp(c, CMPS[rng.integers(0, 6)], int(rng.integers(-8, 62)))


class Model:
    """The table as the oracle sees it: base values and validity, per-row insert / delete
    ids, and per-column chronological update lists."""

    def __init__(self, rng, n0, clustered=False):
        self.data = [rng.integers(0, 50, n0).astype(DTYPES[c]) for c in range(4)]
        if clustered:  # columns 0 and 1 ascend with the row (zonemaps skip zones)
            for c in (0, 1):
                self.data[c] = clustered_values(rng, 0, n0, DTYPES[c])
        self.valid = [rng.random(n0) > (0.1 if c in (0, 2) else 0.0) for c in range(4)]
        self.inserted = np.zeros(n0, dtype=np.uint64)
        self.deleted = np.full(n0, NOT_DELETED, dtype=np.uint64)
        self.upd = {}

    @property
    def n(self):
        return len(self.data[0])

    def ocols(self):
        return [O.Column(self.data[c], validity_from_mask(self.valid[c]), updates=self.upd.get(c)) for c in range(4)]

    def merge(self, c, horizon):
        if c not in self.upd:
            return 0
        rows, vals, vers = self.upd[c]
        keep = np.ones(len(rows), dtype=bool)
        merged = 0
        i = 0
        while i < len(rows):
            j = i
            while j < len(rows) and rows[j] == rows[i]:
                j += 1
            p = i
            while p < j and vers[p] < horizon:
                p += 1
            if p > i:
                r = int(rows[i])
                self.data[c][r] = vals[p - 1]
                self.valid[c][r] = True
                keep[i:p] = False
                merged += 1
            i = j
        self.upd[c] = (rows[keep], vals[keep], vers[keep])
        if not keep.any():
            del self.upd[c]
        return merged


def clustered_values(rng, start, n, dtype):
    """rows [start, start + n) of a column that ascends with the row (one value per 20,000
    rows, ±1 jitter): the layout where zonemaps skip zones"""
    return ((np.arange(start, start + n) // 20_000) + rng.integers(0, 2, n)).astype(dtype)


def run(ctx, seed, n_ops, n0, clustered=False):
    rng = np.random.default_rng(seed)
    m = Model(rng, n0, clustered)
    t = CubitTable(ctx, n0, row_base=int(rng.integers(0, 1 << 30)))
    for c in range(4):
        t.add_column(c, m.data[c], validity_from_mask(m.valid[c]) if c in (0, 2) else None)
    t.build_index(0, L.INDEX_RANGE)
    t.build_index(1, L.INDEX_EQUALITY)
    t.build_index(2, L.INDEX_RANGE, [10, 20, 30, 40])
    t.build_index(2, L.INDEX_BINS, [0, 10, 20, 30, 40, 50])
    clock = 3          # last committed id
    floor = 0          # merges fold versions below this: snapshots start at or after it
    counts = {"scan": 0, "append": 0, "updates": 0, "merge": 0, "deletes": 0, "rows_merged": 0, "zones_skipped": 0}
    for _ in range(n_ops):
        op = rng.choice(["scan", "scan", "scan", "append", "updates", "merge", "deletes"])
        if op == "append":
            nb = int(rng.choice([1, 7, 64, 65, 1000, int(rng.integers(1, 150_000))]))
            lo, hi = (-5, 55) if rng.random() < 0.5 else (0, 50)
            bd = [rng.integers(lo, hi, nb).astype(DTYPES[c]) for c in range(4)]
            if clustered:
                for c in (0, 1):
                    bd[c] = clustered_values(rng, m.n, nb, DTYPES[c])
            bv = [rng.random(nb) > (0.1 if c in (0, 2, 3) else 0.0) for c in range(4)]
            iid = int(rng.choice([0, clock, WRITER]))
            t.append({c: bd[c] for c in range(4)}, {c: validity_from_mask(bv[c]) for c in range(4)}, insert_id=iid)
            for c in range(4):
                m.data[c] = np.concatenate([m.data[c], bd[c]])
                m.valid[c] = np.concatenate([m.valid[c], bv[c]])
            m.inserted = np.concatenate([m.inserted, np.full(nb, iid, dtype=np.uint64)])
            m.deleted = np.concatenate([m.deleted, np.full(nb, NOT_DELETED, dtype=np.uint64)])
        elif op == "updates":
            c = int(rng.integers(0, 4))
            k = int(rng.integers(1, max(2, m.n // 50)))
            rows_u = np.sort(rng.choice(m.n, size=min(k, m.n), replace=False))
            rows, vals, vers = [], [], []
            clock += 2
            for r in rows_u:
                nv = int(rng.integers(1, 4))
                vs = sorted(rng.choice(np.arange(1, clock + 1), size=min(nv, clock), replace=False).tolist())
                if rng.random() < 0.2:
                    vs.append(WRITER)
                for v in vs:
                    rows.append(int(r))
                    vals.append(int(rng.integers(-6, 57)))
                    vers.append(v)
            u = (np.array(rows, dtype=np.int64), np.array(vals, dtype=np.int64), np.array(vers, dtype=np.uint64))
            t.set_updates(c, *u)
            m.upd[c] = u
        elif op == "merge":
            c = int(rng.integers(0, 4))
            h = int(rng.integers(floor, clock + 2))
            got = t.merge_updates(c, h)
            exp = m.merge(c, h)
            assert got == exp, ("merge", c, h, got, exp)
            floor = max(floor, h)
            counts["rows_merged"] += got
        elif op == "deletes":
            k = int(rng.integers(0, max(1, m.n // 20)))
            rows_d = np.sort(rng.choice(m.n, size=min(k, m.n), replace=False)).astype(np.int64)
            ids = rng.choice(np.array([1, clock, WRITER], dtype=np.uint64), size=len(rows_d))
            t.set_deletes(rows_d, ids)
            m.deleted = np.full(m.n, NOT_DELETED, dtype=np.uint64)
            m.deleted[rows_d] = ids
        else:
            filters = {int(c): rand_const_filter(rng) for c in rng.choice(4, size=rng.integers(1, 4), replace=False)}
            fs = F.TableFilterSet(filters)
            residual = rand_residual(rng) if rng.random() < 0.4 else None
            plan = F.serialize(fs, residual)
            start = int(rng.choice([max(floor, 2), clock + 1, clock + 3]))
            tid = int(rng.choice([TXN_START + 1, WRITER]))
            tx = O.Mvcc(start, tid, inserted=m.inserted, deleted=m.deleted)
            ref = O.table_scan(m.ocols(), plan, m.n, row_base=t.row_base, tx=tx)
            got = t.scan(fs, residual, txn=L.Txn(start, tid))
            assert np.array_equal(got, ref), ("scan", start, tid, fs, residual, len(got), len(ref))
            live, nz = t.last_zones()
            counts["zones_skipped"] += live < nz
        counts[op] += 1
    t.close()
    return counts


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_maintenance_fuzz(seed):
    ctx = Context(0)
    if seed % 2 == 0:
        ctx.set_decode_kernel(L.DECODE_RUNS)  # the run-claimed decode at small sizes too
    try:
        counts = run(ctx, seed, 60, 150_001)
        assert counts["scan"] > 10
    finally:
        ctx.close()


@pytest.mark.gpu
def test_maintenance_fuzz_clustered():
    """The same sequence on a table whose indexed columns ascend with the row, so scans skip
    zones while appends, merges and updates keep rewriting the bitvectors the zone classes are
    computed from."""
    ctx = Context(0)
    try:
        counts = run(ctx, 4, 60, 1_000_003, clustered=True)
        assert counts["scan"] > 10 and counts["zones_skipped"] > 0, counts
    finally:
        ctx.close()
