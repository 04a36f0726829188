"""UBIGINT (UINT64) columns over their whole range on the GPU vs the oracle: the column holds the
values' 64 bits and every value-reading kernel compares them unsigned through the key v ^ 2^63
(FilterSelectionSwitch<uint64_t>, column_segment.cpp:278-349: values past 2^63 are the largest,
not negative). Every index encoding, the candidate check, narrowing, zonemaps, MVCC patches,
merges, appends, probes, statistics and the table function, against the oracle's unsigned
restatement on the same inputs."""
import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from cubit_amd.scan_function import ROW_ID, CubitScanFunction
from cubit_amd.table import Context, CubitTable
from oracle import oracle as O

pytestmark = pytest.mark.gpu

TXN_START = 4611686018427388000
CMPS = ["=", "!=", "<", "<=", ">", ">="]
EDGES = [0, 1, 2 ** 32, 2 ** 63 - 1, 2 ** 63, 2 ** 63 + 1, 2 ** 64 - 2, 2 ** 64 - 1]


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def pool_values(rng, k=60):
    """Values over the whole range, the edges around 0, 2^63 and 2^64 included."""
    return np.concatenate([np.array(EDGES, dtype=np.uint64),
                           rng.integers(0, 2 ** 64 - 1, k, dtype=np.uint64, endpoint=True)])


@pytest.mark.parametrize("index", ["none", "range_all", "range_keys", "equality", "bins"])
def test_comparisons_match_oracle(ctx, index):
    rng = np.random.default_rng(5)
    n = 300_007
    pool = pool_values(rng)
    v = pool[rng.integers(0, len(pool), n)]
    valid = rng.random(n) > 0.05
    vw = validity_from_mask(valid)
    t = CubitTable(ctx, n)
    t.add_column(0, v, vw)
    if index == "range_all":
        t.build_index(0, L.INDEX_RANGE)
    elif index == "range_keys":
        t.build_index(0, L.INDEX_RANGE, [2 ** 20, 2 ** 62, 2 ** 63, 2 ** 63 + 2 ** 62, 2 ** 64 - 1])
    elif index == "equality":
        t.build_index(0, L.INDEX_EQUALITY)
    elif index == "bins":
        t.build_index(0, L.INDEX_RANGE)
        t.build_index(0, L.INDEX_BINS, [0, 2 ** 62, 2 ** 63, 2 ** 64 - 1])
    col = O.Column(v, vw)
    for c in EDGES + [int(x) for x in pool[rng.integers(0, len(pool), 6)]] + [2 ** 63 + 12345]:
        for cmp in CMPS:
            fs = F.TableFilterSet({0: F.ConstantFilter(cmp, c)})
            assert np.array_equal(t.scan(fs), O.table_scan([col], F.serialize(fs), n)), (index, cmp, c)
    fs = F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", 2 ** 62), F.ConstantFilter("<", 2 ** 63 + 5)])})
    assert np.array_equal(t.scan(fs), O.table_scan([col], F.serialize(fs), n))
    lo, hi, hn, hv = t.column_statistics(0)
    assert (lo & (2 ** 64 - 1), hi & (2 ** 64 - 1), hn, hv) == (int(v[valid].min()), int(v[valid].max()), True, True)
    t.close()


def test_narrowing_zonemaps_and_probe(ctx):
    rng = np.random.default_rng(6)
    n = 1_000_003
    ints = rng.integers(0, 1000, n).astype(np.int32)
    v = np.sort(rng.integers(0, 2 ** 64 - 1, n, dtype=np.uint64, endpoint=True))  # clustered
    t = CubitTable(ctx, n)
    t.add_column(0, ints)
    t.add_column(1, v)
    t.build_index(0, L.INDEX_RANGE)
    cols = [O.Column(ints), O.Column(v)]
    for (ilo, ihi), (cmp, c) in [((10, 12), (">", 2 ** 63)), ((500, 501), ("<=", 2 ** 62)), ((7, 9), ("!=", int(v[17])))]:
        fs = F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", ilo), F.ConstantFilter("<", ihi)]),
                               1: F.ConstantFilter(cmp, c)})
        for narrowing in (True, False):
            t.use_narrowing(narrowing)
            assert np.array_equal(t.scan(fs), O.table_scan(cols, F.serialize(fs), n)), (cmp, c)
        t.use_narrowing(True)
    fs = F.TableFilterSet({1: F.ConjunctionAndFilter([F.ConstantFilter(">", 2 ** 63 + 2 ** 61),
                                                      F.ConstantFilter("<", 2 ** 63 + 2 ** 62)])})
    rows = t.scan(fs)
    assert np.array_equal(rows, O.table_scan(cols, F.serialize(fs), n))
    ev, nz = t.last_zones()
    assert ev < nz
    est = t.estimate_rows(fs)
    assert len(rows) / 4 <= est <= 4 * len(rows)
    got, ok = t.fetch(1, rows[::29])
    assert ok.all() and np.array_equal(got.view(np.uint64), v[rows[::29]])
    t.close()


@pytest.mark.parametrize("index", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_updates_merges_appends_and_table_function(ctx, index):
    rng = np.random.default_rng(7)
    n = 250_000
    pool = pool_values(rng, 30)
    v = pool[rng.integers(0, len(pool), n)]
    valid = rng.random(n) > 0.03
    vw = validity_from_mask(valid)
    t = CubitTable(ctx, n)
    t.add_column(0, v, vw)
    if index is not None:
        t.build_index(0, index)
    m = 3000
    rows = np.sort(rng.choice(n, m, replace=False)).astype(np.int64)
    new = np.concatenate([pool, np.array([2 ** 63 + 99, 5], dtype=np.uint64)])[rng.integers(0, len(pool) + 2, m)]
    upd_valid = rng.random(m) >= 0.1
    writer = TXN_START + 77
    versions = np.where(rng.random(m) < 0.7, 5, writer).astype(np.uint64)
    t.set_updates(0, rows, new, versions, upd_valid)
    ucol = O.Column(v, vw, updates=(rows, new, versions, upd_valid))
    consts = [0, 2 ** 63, 2 ** 63 + 99, 2 ** 64 - 1, int(pool[9])]
    for txn_id, start in [(writer, 10), (TXN_START + 1, 10), (TXN_START + 2, 3)]:
        txn, tx = L.Txn(start, txn_id), O.Mvcc(start, txn_id)
        for c in consts:
            for cmp in ("=", "<", ">=", "!="):
                fs = F.TableFilterSet({0: F.ConstantFilter(cmp, c)})
                assert np.array_equal(t.scan(fs, txn=txn), O.table_scan([ucol], F.serialize(fs), n, 0, tx)), (cmp, c)
        ids = np.arange(0, n, 97, dtype=np.int64)
        got, ok = t.fetch(0, ids, txn)
        want, wok = O.fetch(ucol, ids, tx=tx, with_valid=True)
        assert np.array_equal(ok, wok) and np.array_equal(got, want)
    t.merge_updates(0, 6)
    committed = versions == 5
    merged, mvalid = v.copy(), valid.copy()
    merged[rows[committed]] = np.where(upd_valid[committed], new[committed], np.uint64(0))
    mvalid[rows[committed]] = upd_valid[committed]
    left = ~committed
    extra = pool[rng.integers(0, len(pool), 20_000)]
    t.append({0: extra})
    allv = np.concatenate([merged, extra])
    allw = validity_from_mask(np.concatenate([mvalid, np.ones(len(extra), bool)]))
    acol = O.Column(allv, allw, updates=(rows[left], new[left], versions[left], upd_valid[left]))
    txn, tx = L.Txn(10, TXN_START + 3), O.Mvcc(10, TXN_START + 3)
    for c in consts:
        for cmp in ("=", "<=", ">"):
            fs = F.TableFilterSet({0: F.ConstantFilter(cmp, c)})
            assert np.array_equal(t.scan(fs, txn=txn), O.table_scan([acol], F.serialize(fs), len(allv), 0, tx))
    # the table function: the committed state (no MVCC view), values crossing at their width
    fs = F.TableFilterSet({0: F.ConstantFilter(">", 2 ** 63)})
    keep = O.table_scan([acol], F.serialize(fs), len(allv), 0, tx)
    fn = CubitScanFunction(t, [ROW_ID, 0], [0, 1], fs, txn=txn)
    from test_gpu_scan_function import drain, ordered

    chunks = drain(fn, 3, validity=True)
    fn.close()
    assert np.array_equal(ordered(chunks, 0), keep)
    want, wok = O.fetch(acol, keep, tx=tx, with_valid=True)
    assert np.array_equal(ordered(chunks, 1), want) and np.array_equal(ordered(chunks, 3), wok)
    t.close()
