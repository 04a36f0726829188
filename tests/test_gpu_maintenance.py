"""Index maintenance: appends (RowGroupCollection::Append with every
BoundIndex::Append, bound_index.hpp:67-70) and the merge of committed updates into the base
(the checkpoint of update chains, update_segment.cpp). After every append or merge:

* every scan equals the oracle (cpu_ref.c's TemplatedScan restatement) over the same rows,
  for readers with and without MVCC snapshots (insert ranges of the appends, update chains);
* every index bitvector is bit-exact against the predicate evaluated on the column as it now
  stands (numpy over the full column), and after appends alone the saved index file is
  byte-identical to one built from scratch over the concatenated column.
"""
import struct

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


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def rand_filter(rng, lo=-6, hi=60, depth=0):
    r = rng.random()
    if depth < 2 and r < 0.2:
        kids = [rand_filter(rng, lo, hi, depth + 1) for _ in range(rng.integers(2, 4))]
        return F.ConjunctionAndFilter(kids) if rng.random() < 0.6 else F.ConjunctionOrFilter(kids)
    if r < 0.28:
        return F.IsNullFilter() if rng.random() < 0.5 else F.IsNotNullFilter()
    return F.ConstantFilter(CMPS[rng.integers(0, 6)], int(rng.integers(lo, hi)))


def rand_filter_set(rng, n_cols):
    return F.TableFilterSet({int(c): rand_filter(rng) for c in rng.choice(n_cols, size=rng.integers(1, n_cols + 1),
                                                                         replace=False)})


# ---------------------------------------------------------------- index file helpers

def read_index(path):
    b = open(path, "rb").read()
    magic, ver, enc, n_rows, nwp, exact, empty, vmin, vmax, n_keys, n_bv = struct.unpack("<8sIIQQIIqqQQ", b[:72])
    assert magic == b"CUBITIX1" and ver in (1, 2)
    h = 72
    col_type, fingerprint = None, None
    if ver == 2:  # the tail: column type, dictionary fingerprint
        col_type, _, fingerprint = struct.unpack("<iIQ", b[72:88])
        h = 88
    keys = np.frombuffer(b[h:h + 8 * n_keys], dtype=np.int64)
    bvs = np.frombuffer(b[h + 8 * n_keys:], dtype=np.uint64).reshape(n_bv, nwp)
    return dict(enc=enc, n_rows=n_rows, nwp=nwp, exact=exact, empty=empty, vmin=vmin, vmax=vmax, keys=keys, bvs=bvs,
                col_type=col_type, fingerprint=fingerprint)


def bits(mask, nwp):
    packed = np.packbits(mask.astype(bool), bitorder="little")
    buf = np.zeros(nwp * 8, dtype=np.uint8)
    buf[:packed.size] = packed
    return buf.view("<u8")


def check_index_bits(t, col, encoding, values, valid, tmp_path):
    """Every bitvector of the column's index equals its predicate on the current column."""
    path = tmp_path / f"ix_{col}_{encoding}.bin"
    t.save_index(col, encoding, path)
    ix = read_index(path)
    assert ix["n_rows"] == len(values)
    v = values.astype(np.int64)
    if valid.any():
        assert ix["vmin"] <= v[valid].min() and ix["vmax"] >= v[valid].max()
    keys = ix["keys"]
    for k in range(ix["bvs"].shape[0]):
        if encoding == L.INDEX_RANGE:
            m = valid & (v < keys[k])
        elif encoding == L.INDEX_EQUALITY:
            m = valid & (v == keys[k])
        else:
            m = valid & (v >= keys[k]) & (v < keys[k + 1])
        assert np.array_equal(ix["bvs"][k], bits(m, ix["nwp"])), (col, encoding, k, int(keys[k]))
    if ix["exact"] and valid.any():  # an every-distinct-value index holds every value as a key
        d = np.unique(v[valid])
        need = d[1:] if encoding == L.INDEX_RANGE else d
        assert np.isin(need, keys).all(), (col, encoding)
    return ix


# ---------------------------------------------------------------- appends

SPECS = [  # (dtype, index definitions, NULL fraction)
    (np.int32, [(L.INDEX_RANGE, None)], 0.1),
    (np.int64, [(L.INDEX_EQUALITY, None)], 0.0),
    (np.int64, [(L.INDEX_RANGE, [10, 20, 30, 40]), (L.INDEX_BINS, [0, 10, 20, 30, 40, 50])], 0.1),
    (np.int32, [], 0.0),
]


def make_batch(rng, n, lo, hi, null_frac):
    data = [rng.integers(lo, hi, n).astype(SPECS[c][0]) for c in range(4)]
    valid = [rng.random(n) >= null_frac[c] for c in range(4)]
    return data, valid


def scan_checks(rng, t, data, valid, inserted, n_checks, views):
    n = len(data[0])
    ocols = [O.Column(data[c], validity_from_mask(valid[c]) if not valid[c].all() else None) for c in range(4)]
    for i in range(n_checks):
        fs = rand_filter_set(rng, 4)
        plan = F.serialize(fs)
        ref = O.table_scan(ocols, plan, n, row_base=t.row_base)
        got = t.scan(fs)
        assert np.array_equal(got, ref), ("no txn", i, fs)
        start, tid = views[i % len(views)]
        tx = O.Mvcc(start, tid, inserted=inserted)
        ref_t = O.table_scan(ocols, plan, n, row_base=t.row_base, tx=tx)
        got_t = t.scan(fs, txn=L.Txn(start, tid))
        assert np.array_equal(got_t, ref_t), ("txn", start, tid, i, fs)
        assert t.count(fs, txn=L.Txn(start, tid)) == len(ref_t)


@pytest.mark.parametrize("n0", [100_003, 0])
def test_append_matches_oracle_and_rebuilt_index(ctx, tmp_path, n0):
    rng = np.random.default_rng(31 + n0)
    writer = TXN_START + 9
    null_frac = [SPECS[c][2] for c in range(4)]
    data, valid = make_batch(rng, n0, 0, 50, null_frac)
    t = CubitTable(ctx, n0, row_base=17)
    for c in range(4):
        t.add_column(c, data[c], validity_from_mask(valid[c]) if null_frac[c] else None)
        for enc, keys in SPECS[c][1]:
            t.build_index(c, enc, keys)
    inserted = np.zeros(n0, dtype=np.uint64)
    views = [(2, TXN_START + 1), (8, TXN_START + 2), (20, writer)]
    # ragged batches: within a word, word-aligned, a tile, and one that crosses the
    # 1,048,576-row padding (the table grows in place); later batches bring values outside
    # [0, 50) (new keys below the old minimum and above the maximum) and column 3's first NULLs
    batches = [(1, 0, 50, 0), (63, 0, 50, 5), (64, -3, 50, 0), (1000, 0, 55, writer),
               (131_073, -3, 55, 12), (1_048_593, -3, 55, 0)]
    for bi, (nb, lo, hi, iid) in enumerate(batches):
        nf = list(null_frac)
        if bi >= 3:
            nf[3] = 0.05
        bd, bv = make_batch(rng, nb, lo, hi, nf)
        vw = {c: validity_from_mask(bv[c]) for c in range(4) if nf[c]}
        t.append({c: bd[c] for c in range(4)}, vw, insert_id=iid)
        for c in range(4):
            data[c] = np.concatenate([data[c], bd[c]])
            valid[c] = np.concatenate([valid[c], bv[c] if nf[c] else np.ones(nb, dtype=bool)])
        inserted = np.concatenate([inserted, np.full(nb, iid, dtype=np.uint64)])
        assert t.n_rows == len(data[0])
        scan_checks(rng, t, data, valid, inserted, 12, views)
    for c in range(4):
        for enc, _ in SPECS[c][1]:
            check_index_bits(t, c, enc, data[c], valid[c], tmp_path)
    # the maintained indexes are the ones a fresh build over the whole column gives
    t2 = CubitTable(ctx, len(data[0]), row_base=17)
    for c in range(4):
        t2.add_column(c, data[c], validity_from_mask(valid[c]) if not valid[c].all() else None)
        for enc, keys in SPECS[c][1]:
            t2.build_index(c, enc, keys)
            a, b = tmp_path / "maintained.bin", tmp_path / "fresh.bin"
            t.save_index(c, enc, a)
            t2.save_index(c, enc, b)
            assert a.read_bytes() == b.read_bytes(), (c, enc)
    t2.close()
    t.close()


def test_append_q6_lineitem_matches_whole_table():
    """SF0.1 lineitem built in two appends of an SF0.01-sized head: Q6 rows and revenue equal
    the whole table's (and the reference answer)."""
    from conftest import lineitem
    li = lineitem(0.1)
    c = Context(0)
    head = 60_000
    t = CubitTable(c, head)
    cols = [li.l_shipdate, li.l_discount, li.l_quantity, li.l_extendedprice]
    for i, a in enumerate(cols):
        t.add_column(i, a[:head])
    months = [F.date(y, m, 1) for y in range(1992, 1999) for m in range(1, 13)] + [F.date(1999, 1, 1)]
    t.build_index(0, L.INDEX_RANGE, months)
    t.build_index(1, L.INDEX_RANGE)
    t.build_index(2, L.INDEX_RANGE)
    mid = head + (li.n_rows - head) // 3
    t.append({i: a[head:mid] for i, a in enumerate(cols)})
    t.append({i: a[mid:] for i, a in enumerate(cols)})
    ocols = [O.Column(a) for a in cols[:3]]
    ref = O.table_scan(ocols, F.serialize(F.q6_filter_set()), li.n_rows)
    got = t.scan(F.q6_filter_set())
    assert np.array_equal(got, ref)
    total, cnt = t.sum_product(3, 1, F.q6_filter_set())
    assert cnt == len(ref)
    assert total == O.sum_product(li.l_extendedprice, li.l_discount, ref)
    t.close()
    c.close()


def test_append_rejects_bad_input(ctx):
    t = CubitTable(ctx, 10)
    t.add_column(0, np.arange(10, dtype=np.int32))
    t.add_column(1, np.arange(10, dtype=np.int64))
    with pytest.raises(ValueError):
        t.append({0: np.arange(3, dtype=np.int64), 1: np.arange(3, dtype=np.int64)})
    lib = t.lib
    import ctypes as C
    a = np.arange(3, dtype=np.int32)
    cid = (C.c_int * 1)(0)
    dptr = (C.c_void_p * 1)(a.ctypes.data)
    assert lib.cubit_table_append(t.handle, 3, cid, dptr, None, 1, 0) == L.ERR_INVALID  # a column missing
    assert t.n_rows == 10
    t.close()


# ---------------------------------------------------------------- merge of committed updates

def build_chains(rng, n, n_rows_upd, versions, writer, lo, hi):
    """Per updated row 1-3 records with ascending versions, sometimes the writer's at the end."""
    rows, vals, vers = [], [], []
    for r in np.sort(rng.choice(n, size=n_rows_upd, replace=False)):
        k = int(rng.integers(1, 4))
        vs = sorted(rng.choice(versions, size=k, replace=False).tolist())
        if rng.random() < 0.25:
            vs.append(writer)
        for v in vs:
            rows.append(int(r))
            vals.append(int(rng.integers(lo, hi)))
            vers.append(v)
    return (np.array(rows, dtype=np.int64), np.array(vals, dtype=np.int64), np.array(vers, dtype=np.uint64))


def merged_base(data, valid, upd, horizon):
    base, ok = data.astype(np.int64).copy(), valid.copy()
    rows, vals, vers = upd
    blocked = set()
    for r, v, ver in zip(rows, vals, vers):
        if r in blocked:
            continue
        if ver < horizon:
            base[r] = v
            ok[r] = True
        else:
            blocked.add(r)
    return base.astype(data.dtype), ok


def test_merge_updates_matches_oracle_and_index_bits(ctx, tmp_path):
    rng = np.random.default_rng(909)
    n = 300_007
    writer = TXN_START + 5
    t = CubitTable(ctx, n, row_base=3)
    data, valid, upd = [], [], []
    defs = [[(L.INDEX_RANGE, None)], [(L.INDEX_EQUALITY, None)],
            [(L.INDEX_RANGE, [10, 20, 30, 40]), (L.INDEX_BINS, [0, 10, 20, 30, 40, 50])]]
    dtypes = [np.int32, np.int64, np.int64]
    for c in range(3):
        d = rng.integers(0, 50, n).astype(dtypes[c])
        ok = rng.random(n) > 0.1
        t.add_column(c, d, validity_from_mask(ok))
        for enc, keys in defs[c]:
            t.build_index(c, enc, keys)
        # updated values reach outside [0, 50): new keys for the exact indexes
        u = build_chains(rng, n, 4000, [2, 4, 6, 8], writer, -4, 56)
        t.set_updates(c, *u)
        data.append(d)
        valid.append(ok)
        upd.append(u)
    dels = np.sort(rng.choice(n, size=5000, replace=False)).astype(np.int64)
    del_ids = np.where(rng.random(len(dels)) < 0.5, np.uint64(3), np.uint64(writer)).astype(np.uint64)
    t.set_deletes(dels, del_ids)
    deleted = np.full(n, np.uint64(2 ** 64 - 2), dtype=np.uint64)
    deleted[dels] = del_ids
    ocols = [O.Column(data[c], validity_from_mask(valid[c]), updates=upd[c]) for c in range(3)]

    def check(views, n_checks, tag):
        for i in range(n_checks):
            fs = F.TableFilterSet({int(c): rand_filter(rng) for c in
                                   rng.choice(3, size=rng.integers(1, 4), replace=False)})
            plan = F.serialize(fs)
            start, tid = views[i % len(views)]
            ref = O.table_scan(ocols, plan, n, row_base=3, tx=O.Mvcc(start, tid, deleted=deleted))
            got = t.scan(fs, txn=L.Txn(start, tid))
            assert np.array_equal(got, ref), (tag, i, start, tid, fs)

    views = [(5, TXN_START + 1), (7, writer), (9, TXN_START + 2)]
    check(views, 12, "before")
    # horizon 5: versions 2 and 4 fold into the base; 6, 8 and the writer's stay
    for c in range(3):
        merged = t.merge_updates(c, 5)
        exp_rows = len({int(r) for r, v in zip(upd[c][0], upd[c][2]) if v < 5})
        assert merged == exp_rows > 0
        base, ok = merged_base(data[c], valid[c], upd[c], 5)
        assert np.array_equal(t.download_column(c), base), c
        for enc, _ in defs[c]:
            check_index_bits(t, c, enc, base, ok, tmp_path)
    check(views, 24, "after horizon 5")
    # horizon past every committed version: only the writer's records stay
    for c in range(3):
        t.merge_updates(c, 9)
        base, ok = merged_base(data[c], valid[c], upd[c], 9)
        assert np.array_equal(t.download_column(c), base), c
        for enc, _ in defs[c]:
            check_index_bits(t, c, enc, base, ok, tmp_path)
    check([(9, TXN_START + 2), (12, writer)], 16, "after horizon 9")
    # then an append on top of the merged base, visible to every snapshot
    nb = 70_001
    bd = [rng.integers(-2, 52, nb).astype(dtypes[c]) for c in range(3)]
    t.append({c: bd[c] for c in range(3)})
    for c in range(3):
        cur, ok = merged_base(data[c], valid[c], upd[c], 9)
        cur = np.concatenate([cur, bd[c]])
        ok = np.concatenate([ok, np.ones(nb, dtype=bool)])
        for enc, _ in defs[c]:
            check_index_bits(t, c, enc, cur, ok, tmp_path)
    t.close()


def test_merge_into_int32_rejects_wide_values(ctx):
    t = CubitTable(ctx, 100)
    t.add_column(0, np.arange(100, dtype=np.int32))
    t.build_index(0, L.INDEX_RANGE)
    t.set_updates(0, np.array([5], dtype=np.int64), np.array([2 ** 40], dtype=np.int64), np.array([1], dtype=np.uint64))
    with pytest.raises(L.CubitError):
        t.merge_updates(0, 10)
    t.close()


def test_appends_concurrent_with_scans(ctx):
    """A writer thread appends batches while a reader thread scans the same table on the same
    context (the context mutex serialises the calls, DuckDB's pipeline threads share one
    context the same way): every scan returns exactly the oracle's rows over some prefix of
    the batches — never a torn state."""
    import threading

    rng = np.random.default_rng(99)
    n0 = 200_003
    batches = [rng.integers(0, 50, int(rng.integers(1, 300_000))).astype(np.int32) for _ in range(12)]
    base = rng.integers(0, 50, n0).astype(np.int32)
    t = CubitTable(ctx, n0)
    t.add_column(0, base)
    t.build_index(0, L.INDEX_RANGE)
    fs = F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", 10), F.ConstantFilter("<", 13)])})
    prefixes = [base]
    for b in batches:
        prefixes.append(np.concatenate([prefixes[-1], b]))
    expected = {len(p): np.flatnonzero((p >= 10) & (p < 13)).astype(np.int64) for p in prefixes}
    errors, seen = [], set()

    def writer():
        try:
            for b in batches:
                t.append({0: b})
        except Exception as e:  # reported below
            errors.append(repr(e))

    def reader():
        try:
            for _ in range(40):
                got = t.scan(fs, capacity=len(prefixes[-1]))  # the table grows under the reader
                ok = [n for n, ref in expected.items() if len(ref) == len(got) and np.array_equal(got, ref)]
                if not ok:
                    errors.append(f"scan of {len(got)} rows matches no prefix")
                seen.update(ok)
        except Exception as e:
            errors.append(repr(e))

    th = [threading.Thread(target=writer), threading.Thread(target=reader)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:3]
    assert np.array_equal(t.scan(fs), expected[len(prefixes[-1])])
    t.close()
