"""HUGEINT / UHUGEINT columns on the GPU vs the oracle. The column is a dictionary column over its
values' 16-byte order keys (cubit_key128: big-endian, HUGEINT's sign bit flipped), so its codes are
the values' ranks and a comparison with a 128-bit constant is a comparison of codes (present or
absent from the dictionary) through the same K0 / index / candidate-check / narrowing / zonemap /
MVCC machinery as an INTEGER column. Pinned by the reference's hugeint / uhugeint filter queries
(tests/golden/huge_filter_cases.json); the random cases compare with the oracle's restatement of
FilterSelectionSwitch<hugeint_t / uhugeint_t> (column_segment.cpp:468-479) on 128-bit integers,
across the sign, 2^64 and the type's bounds."""
import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.scan_function import ROW_ID, CubitScanFunction
from cubit_amd.table import Context, CubitTable, Dictionary
from oracle import oracle as O
from test_oracle_huge_filters import CMPS, edges, golden_cases, pool

pytestmark = pytest.mark.gpu

TXN_START = 4611686018427388000


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def gpu_filter(op, v, signed):
    return F.ConstantFilter(op, F.key128(v, signed))


def oracle_filter(op, v):
    return F.ConstantFilter(op, O.huge_ref(v))


def decode(d, codes, ok, signed):
    return [F.value128(d.entry(c), signed) if o else None for c, o in zip(codes, ok)]


@pytest.mark.parametrize("index", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_reference_huge_filter_cases(ctx, index):
    for case in golden_cases():
        h = case["columns"].index("h")
        signed = case["types"][h] == "HUGEINT"
        n = len(case["rows"])
        t = CubitTable(ctx, n)
        d = None
        for j, typ in enumerate(case["types"]):
            vals = [None if r[j] is None else int(r[j]) for r in case["rows"]]
            if j == h:
                d = t.add_huge_column(j, vals, signed)
            else:
                t.add_column(j, np.array(vals, dtype=np.int32))
        if index is not None:
            t.build_index(h, index)
        for q in case["queries"]:
            flt = F.IsNullFilter() if q["cmp"] == "IS NULL" else gpu_filter(q["cmp"], int(q["constant"]), signed)
            rows = t.scan(F.TableFilterSet({h: flt}))
            codes, ok = t.fetch(h, rows)
            vals = decode(d, codes, ok, signed)
            if q["select"] == "COUNT(*)":
                got = [str(len(rows))]
            elif q["select"].startswith("id, FIRST(h), LAST(h)"):
                ids, _ = t.fetch(case["columns"].index("id"), rows)
                assert all(v is None for v in vals)
                got = [f"{i}\tNULL\tNULL" for i in sorted(set(ids.tolist()))]
            else:
                got = [str(v) for v in vals]
                got = sorted(got, key=int) if "ORDER BY" in q["sql"] else got
            assert got == q["rows"], (case["file"], q["sql"], index)
        t.close()


def absent(signed, present):
    """Constants the column does not hold: neighbours of held values and of the bounds."""
    lo, hi = (-(1 << 127), (1 << 127) - 1) if signed else (0, (1 << 128) - 1)
    out = []
    for v in sorted(present)[:: max(1, len(present) // 10)]:
        out += [v - 1, v + 1]
    return [v for v in out + [lo + 2, hi - 2, 2 ** 64 + 7] if lo <= v <= hi and v not in present]


@pytest.mark.parametrize("signed", [True, False])
@pytest.mark.parametrize("index", ["none", "range_all", "range_keys", "equality", "bins"])
def test_random_comparisons_match_oracle(ctx, signed, index):
    rng = np.random.default_rng(31 if signed else 32)
    n = 200_003
    p = pool(signed, rng, 60)
    vals = [None if rng.random() < 0.04 else p[i] for i in rng.integers(0, len(p), n)]
    t = CubitTable(ctx, n)
    t.add_huge_column(0, vals, signed)
    zero = 0 if not signed else -(2 ** 64)
    if index == "range_all":
        t.build_index(0, L.INDEX_RANGE)
    elif index == "range_keys":  # keys given as ints, some absent: constants between them take the candidate check
        t.build_index(0, L.INDEX_RANGE, sorted({zero, 1, 2 ** 63, 2 ** 64, 2 ** 100 + 3}))
    elif index == "equality":
        t.build_index(0, L.INDEX_EQUALITY)
    elif index == "bins":
        t.build_index(0, L.INDEX_RANGE)
        t.build_index(0, L.INDEX_BINS, sorted({zero, 0, 2 ** 64, 2 ** 100, 2 ** 126}))
    col = O.HugeColumn(vals, signed=signed)
    present = {v for v in vals if v is not None}
    consts = edges(signed) + [p[i] for i in rng.integers(0, len(p), 6)] + absent(signed, present)[:12]
    for c in consts:
        for op in CMPS:
            got = t.scan(F.TableFilterSet({0: gpu_filter(op, c, signed)}))
            want = O.table_scan([col], F.serialize(F.TableFilterSet({0: oracle_filter(op, c)})), n)
            assert np.array_equal(got, want), (index, op, c)
    for lo, hi in [(0, 2 ** 64), (-(2 ** 63), 2 ** 63) if signed else (2 ** 63, 2 ** 65), (42, 43)]:
        g = F.ConjunctionAndFilter([gpu_filter(">=", lo, signed), gpu_filter("<", hi, signed)])
        o = F.ConjunctionAndFilter([oracle_filter(">=", lo), oracle_filter("<", hi)])
        assert np.array_equal(t.scan(F.TableFilterSet({0: g})),
                              O.table_scan([col], F.serialize(F.TableFilterSet({0: o})), n)), (lo, hi)
    g = F.ConjunctionOrFilter([gpu_filter("=", 42, signed), gpu_filter(">", 2 ** 100, signed), F.IsNullFilter()])
    o = F.ConjunctionOrFilter([oracle_filter("=", 42), oracle_filter(">", 2 ** 100), F.IsNullFilter()])
    assert np.array_equal(t.scan(F.TableFilterSet({0: g})), O.table_scan([col], F.serialize(F.TableFilterSet({0: o})), n))
    t.close()


@pytest.mark.parametrize("signed", [True, False])
def test_conjunction_zonemaps_probe_and_statistics(ctx, signed):
    """A 128-bit comparison inside a selective conjunction (narrowing), zone skipping on clustered
    values, probed codes decoded to the oracle's values, statistics decoded to min / max."""
    rng = np.random.default_rng(33)
    n = 1_000_003
    ints = rng.integers(0, 1000, n).astype(np.int32)
    p = sorted(set(pool(signed, rng, 300)))
    vals = [p[i] for i in np.sort(rng.integers(0, len(p), n))]  # clustered
    vals = [None if i % 101 == 0 else v for i, v in enumerate(vals)]
    t = CubitTable(ctx, n)
    t.add_column(0, ints)
    d = t.add_huge_column(1, vals, signed)
    t.build_index(0, L.INDEX_RANGE)
    cols = [O.Column(ints), O.HugeColumn(vals, signed=signed)]
    mid = p[len(p) // 2]
    for (ilo, ihi), (op, c) in [((10, 12), (">", mid)), ((500, 501), ("<=", 2 ** 64)), ((0, 3), ("=", p[9])),
                               ((7, 9), ("!=", 0))]:
        lo, hi = F.ConstantFilter(">=", ilo), F.ConstantFilter("<", ihi)
        g = F.TableFilterSet({0: F.ConjunctionAndFilter([lo, hi]), 1: gpu_filter(op, c, signed)})
        o = F.TableFilterSet({0: F.ConjunctionAndFilter([lo, hi]), 1: oracle_filter(op, c)})
        for narrowing in (True, False):
            t.use_narrowing(narrowing)
            assert np.array_equal(t.scan(g), O.table_scan(cols, F.serialize(o), n)), (op, c)
        t.use_narrowing(True)
    a, b = p[len(p) // 3], p[len(p) // 3 + 5]
    g = F.TableFilterSet({1: F.ConjunctionAndFilter([gpu_filter(">=", a, signed), gpu_filter("<", b, signed)])})
    o = F.TableFilterSet({1: F.ConjunctionAndFilter([oracle_filter(">=", a), oracle_filter("<", b)])})
    rows = t.scan(g)
    assert np.array_equal(rows, O.table_scan(cols, F.serialize(o), n))
    ev, nz = t.last_zones()
    assert ev < nz
    ids = rows[::37]
    codes, ok = t.fetch(1, ids)
    want, wok = O.fetch(cols[1], ids, with_valid=True)
    assert np.array_equal(ok, wok) and decode(d, codes, ok, signed) == cols[1].decode(want, wok)
    lo, hi, hn, hv = t.column_statistics(1)
    present = sorted(v for v in set(vals) if v is not None)
    assert (F.value128(d.entry(lo), signed), F.value128(d.entry(hi), signed), hn, hv) == \
        (present[0], present[-1], True, True)
    t.close()


@pytest.mark.parametrize("signed", [True, False])
@pytest.mark.parametrize("index", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_updates_merges_appends_and_table_function(ctx, signed, index):
    rng = np.random.default_rng(34)
    n = 150_000
    p = pool(signed, rng, 40)
    vals = [None if rng.random() < 0.03 else p[i] for i in rng.integers(0, len(p), n)]
    d = Dictionary([F.key128(v, signed) for v in sorted(set(p))])  # every pool value: updates / appends use them
    t = CubitTable(ctx, n)
    t.add_huge_column(0, vals, signed, d)
    if index is not None:
        t.build_index(0, index)
    code = {v: i for i, v in enumerate(sorted(set(p)))}
    m = 2000
    rows = np.sort(rng.choice(n, m, replace=False)).astype(np.int64)
    new = [p[i] for i in rng.integers(0, len(p), m)]
    upd_valid = rng.random(m) >= 0.1
    writer = TXN_START + 77
    versions = np.where(rng.random(m) < 0.7, 5, writer).astype(np.uint64)
    t.set_updates(0, rows, np.array([code[v] for v in new], dtype=np.int64), versions, upd_valid)
    ovals = [v if ok else None for v, ok in zip(new, upd_valid)]
    ucol = O.HugeColumn(vals, signed=signed, updates=(rows, ovals, versions, upd_valid))
    consts = [p[3], p[10], 0, 2 ** 64, edges(signed)[0]]
    for txn_id, start in [(writer, 10), (TXN_START + 1, 10), (TXN_START + 2, 3)]:
        txn, tx = L.Txn(start, txn_id), O.Mvcc(start, txn_id)
        for c in consts:
            for op in ("=", "<", ">=", "!="):
                got = t.scan(F.TableFilterSet({0: gpu_filter(op, c, signed)}), txn=txn)
                want = O.table_scan([ucol], F.serialize(F.TableFilterSet({0: oracle_filter(op, c)})), n, 0, tx)
                assert np.array_equal(got, want), (op, c)
        ids = np.arange(0, n, 97, dtype=np.int64)
        got, ok = t.fetch(0, ids, txn)
        want, wok = O.fetch(ucol, ids, tx=tx, with_valid=True)
        assert np.array_equal(ok, wok) and decode(d, got, ok, signed) == ucol.decode(want, wok)
    t.merge_updates(0, 6)
    committed = versions == 5
    merged = list(vals)
    for r, v, ok, cm in zip(rows, new, upd_valid, committed):
        if cm:
            merged[r] = v if ok else None
    left = ~committed
    extra = [p[i] for i in rng.integers(0, len(p), 10_000)]
    t.append({0: np.array([code[v] for v in extra], dtype=np.int32)})
    allv = merged + extra
    acol = O.HugeColumn(allv, signed=signed, updates=(rows[left], [o for o, k in zip(ovals, left) if k],
                                                      versions[left], upd_valid[left]))
    txn, tx = L.Txn(10, TXN_START + 3), O.Mvcc(10, TXN_START + 3)
    for c in consts:
        for op in ("=", "<=", ">"):
            got = t.scan(F.TableFilterSet({0: gpu_filter(op, c, signed)}), txn=txn)
            want = O.table_scan([acol], F.serialize(F.TableFilterSet({0: oracle_filter(op, c)})), len(allv), 0, tx)
            assert np.array_equal(got, want), ("appended", op, c)
    # the table function: codes cross at their width, decoded through the dictionary
    c = p[len(p) // 2]
    keep = O.table_scan([acol], F.serialize(F.TableFilterSet({0: oracle_filter(">", c)})), len(allv), 0, tx)
    fn = CubitScanFunction(t, [ROW_ID, 0], [0, 1], F.TableFilterSet({0: gpu_filter(">", c, signed)}), txn=txn)
    from test_gpu_scan_function import drain, ordered

    chunks = drain(fn, 3, validity=True)
    fn.close()
    assert np.array_equal(ordered(chunks, 0), keep)
    want, wok = O.fetch(acol, keep, tx=tx, with_valid=True)
    got, gok = ordered(chunks, 1), ordered(chunks, 3)
    assert np.array_equal(gok, wok) and decode(d, got, gok, signed) == acol.decode(want, wok)
    t.close()
