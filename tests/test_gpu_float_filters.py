"""FLOAT / DOUBLE columns on the GPU vs the oracle: DuckDB's floating-point comparisons
(src/common/vector_operations/comparison_operators.cpp:17-88 — NaN equals NaN and is greater than
every other value, -0.0 == +0.0) through every way a scan reaches the column values: K0 over the
raw column, every index encoding (keys given as floats, or every distinct value), the candidate
check between range keys, selection narrowing, zonemaps, MVCC updates (patched leaves), merges,
appends, the probe (bit patterns handed back as stored: -0.0 and NaN payloads survive), the column
statistics and the low-level K0 entry point. Pinned by the reference's nan_test.test /
infinity_test.test table filters (tests/golden/float_filter_cases.json) for both types; the random
cases compare with the oracle's restatement of FilterSelectionSwitch<float / double>
(column_segment.cpp:278-349) on the same inputs."""
import ctypes as C
import json
import math
from collections import Counter
from pathlib import Path

import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from cubit_amd.table import Context, CubitTable
from oracle import oracle as O

pytestmark = pytest.mark.gpu

CASES = json.loads((Path(__file__).resolve().parent / "golden" / "float_filter_cases.json").read_text())["cases"]
TYPES = {"FLOAT": np.float32, "DOUBLE": np.float64}
OPS = {"=": "=", "<>": "!=", "<": "<", "<=": "<=", ">": ">", ">=": ">="}
CMPS = ["=", "!=", "<", "<=", ">", ">="]
TXN_START = 4611686018427388000


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def fval(text, dtype):
    special = {"nan": math.nan, "inf": math.inf, "-inf": -math.inf}
    return dtype(special[text] if text in special else float(text))


def printed(x):
    if math.isnan(x):
        return "nan"
    if math.isinf(x):
        return "inf" if x > 0 else "-inf"
    return f"{x:g}"


def bits_of(vals, dt):
    return O.fp_bits(vals, dt)


def special_values(dt):
    """Every class a comparison must order: both zeros, NaNs of either sign with payloads, ±inf,
    the extreme finite and subnormal values."""
    b = np.uint32 if dt == np.float32 else np.uint64
    nans = [0x7FC00000, 0x7FC00001, 0xFFC00000, 0x7F800001] if dt == np.float32 else \
        [0x7FF8000000000000, 0x7FF8000000000001, 0xFFF8000000000000, 0x7FF0000000000001]
    fi = np.finfo(dt)
    out = [dt(0.0), dt(-0.0), dt(math.inf), dt(-math.inf), fi.max, -fi.max, fi.tiny, -fi.tiny,
           dt(fi.tiny / 4), dt(-fi.tiny / 4), dt(1.0), dt(-1.0), dt(0.5), dt(2.5)]
    out += list(np.array(nans, dtype=b).view(dt))
    return out


def random_column(rng, dt, n, null_frac=0.0, distinct=None):
    """Values from a small pool (so indexes and equality hit), with the special values mixed in."""
    pool = np.concatenate([np.array(special_values(dt), dtype=dt),
                           (rng.standard_normal(distinct or 40) * 1e3).astype(dt)])
    vals = pool[rng.integers(0, len(pool), n)]
    valid = rng.random(n) >= null_frac if null_frac else None
    return vals, pool, valid


def oracle_rows(cols, fs, n, tx=None, residual=None):
    return O.table_scan(cols, F.serialize(fs, residual), n, 0, tx)


# ------------------------------------------------------------------ reference fixtures


def fixture_queries():
    for case in CASES:
        for tname in case["types"]:
            for q in case["queries"]:
                yield pytest.param(case, tname, q, id=f"{Path(case['file']).stem}-{tname}-f{q['cmp']}{q['constant']}")


@pytest.mark.parametrize("index", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
@pytest.mark.parametrize("case,tname,q", list(fixture_queries()))
def test_reference_float_filter_case(ctx, case, tname, q, index):
    dt = TYPES[tname]
    vals = np.array([fval(v, dt) for v in case["inserted"]], dtype=dt)
    t = CubitTable(ctx, len(vals))
    t.add_column(0, vals)
    if index is not None:
        t.build_index(0, index)  # every distinct value
    fs = F.TableFilterSet({0: F.ConstantFilter(OPS[q["cmp"]], fval(q["constant"], dt))})
    rows = t.scan(fs)
    assert Counter(printed(float(vals[r])) for r in rows) == Counter(q["rows"]), q["sql"]
    assert np.array_equal(rows, oracle_rows([O.Column(vals)], fs, len(vals)))


# ------------------------------------------------------------------ random filters vs the oracle


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("index", ["none", "range_all", "range_keys", "equality", "bins"])
def test_random_comparisons_match_oracle(ctx, dt, index):
    rng = np.random.default_rng(11 if dt == np.float32 else 12)
    n = 300_007  # three zones, a ragged tail
    vals, pool, valid = random_column(rng, dt, n, null_frac=0.05)
    vw = validity_from_mask(valid)
    t = CubitTable(ctx, n)
    t.add_column(0, vals, vw)
    if index == "range_all":
        t.build_index(0, L.INDEX_RANGE)
    elif index == "range_keys":  # edges between pool values: constants off the keys take the candidate check
        t.build_index(0, L.INDEX_RANGE, np.array([-1e3, -1.0, -0.0, 1.0, 10.0, math.inf], dtype=dt))
    elif index == "equality":
        t.build_index(0, L.INDEX_EQUALITY)
    elif index == "bins":
        t.build_index(0, L.INDEX_RANGE)
        t.build_index(0, L.INDEX_BINS, np.array([-math.inf, -1.0, 0.0, 1.0, math.inf], dtype=dt))
    col = O.Column(vals, vw)
    consts = list(np.array(special_values(dt), dtype=dt)) + list(pool[rng.integers(0, len(pool), 8)]) + \
        [dt(3.25), dt(-7.0)]
    for c in consts:
        for cmp in CMPS:
            fs = F.TableFilterSet({0: F.ConstantFilter(cmp, dt(c))})
            got = t.scan(fs)
            want = oracle_rows([col], fs, n)
            assert np.array_equal(got, want), (index, cmp, c)
    # two-sided ranges (one folded interval) and an OR across constants
    for lo, hi in [(dt(-1.0), dt(1.0)), (dt(-0.0), dt(0.0)), (dt(-math.inf), dt(math.nan)), (dt(0.5), dt(math.inf))]:
        fs = F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", lo), F.ConstantFilter("<", hi)])})
        assert np.array_equal(t.scan(fs), oracle_rows([col], fs, n)), (lo, hi)
    fs = F.TableFilterSet({0: F.ConjunctionOrFilter([F.ConstantFilter("=", dt(math.nan)),
                                                     F.ConstantFilter("<", dt(-1.0)), F.IsNullFilter()])})
    assert np.array_equal(t.scan(fs), oracle_rows([col], fs, n))


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_conjunction_with_integer_column_narrowing_and_zonemaps(ctx, dt):
    """A float comparison inside a selective conjunction is read only at the kept rows
    (masked_compare); clustered values let the zonemaps skip zones (column_zone_stats on keys)."""
    rng = np.random.default_rng(5)
    n = 1_000_003
    ints = rng.integers(0, 1000, n).astype(np.int32)
    vals = np.sort((rng.standard_normal(n) * 100).astype(dt))  # clustered: zones hold ranges
    vals[:300] = dt(-0.0)  # zone 0 still tops out below the range tested last
    vals[n - 300:] = dt(math.nan)  # NaN is the greatest value: the last zone's maximum
    t = CubitTable(ctx, n)
    t.add_column(0, ints)
    t.add_column(1, vals)
    t.build_index(0, L.INDEX_RANGE)
    cols = [O.Column(ints), O.Column(vals)]
    for (ilo, ihi), (cmp, c) in [((10, 12), (">", dt(0.0))), ((500, 501), ("<=", dt(-50.0))),
                                 ((0, 3), ("=", dt(math.nan))), ((7, 9), ("!=", dt(-0.0)))]:
        fs = F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", ilo), F.ConstantFilter("<", ihi)]),
                               1: F.ConstantFilter(cmp, c)})
        for narrowing in (True, False):
            t.use_narrowing(narrowing)
            for zonemap in (True, False):
                assert np.array_equal(t.scan(fs, zonemap=zonemap), oracle_rows(cols, fs, n)), (cmp, c)
        t.use_narrowing(True)
    # a float range alone on clustered values: the zonemaps skip most zones
    fs = F.TableFilterSet({1: F.ConjunctionAndFilter([F.ConstantFilter(">", dt(150.0)), F.ConstantFilter("<", dt(200.0))])})
    assert np.array_equal(t.scan(fs), oracle_rows(cols, fs, n))
    ev, nz = t.last_zones()
    assert ev < nz
    # the estimate takes values uniform in value space within a zone (not in key space): on
    # clustered values without NaN / inf it lands near the true count
    clean = np.sort((rng.standard_normal(n) * 100).astype(dt))
    t2 = CubitTable(ctx, n)
    t2.add_column(1, clean)
    true = int(((clean > 150) & (clean < 200)).sum())
    est = t2.estimate_rows(fs)
    assert true / 4 <= est <= 4 * true, (est, true)


# ------------------------------------------------------------------ probe, statistics, low-level K0


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_probe_returns_bit_patterns(ctx, dt):
    rng = np.random.default_rng(3)
    n = 70_000
    vals, _, valid = random_column(rng, dt, n, null_frac=0.1)
    vw = validity_from_mask(valid)
    t = CubitTable(ctx, n)
    t.add_column(0, vals, vw)
    ids = np.sort(rng.choice(n, 5000, replace=False)).astype(np.int64)
    got, ok = t.fetch(0, ids)
    want, wok = O.fetch(O.Column(vals, vw), ids, with_valid=True)
    assert np.array_equal(ok, wok)
    assert np.array_equal(got, want)  # -0.0 and every NaN payload as stored
    assert np.array_equal(got[ok], bits_of(vals[ids[ok]], dt))
    assert t.download_column(0).view(np.uint8).tobytes() == vals.view(np.uint8).tobytes()


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_column_statistics_are_patterns_of_the_extremes(ctx, dt):
    vals = np.array([1.5, -0.0, -3.0, 7.0, math.inf, -2.0], dtype=dt)
    t = CubitTable(ctx, len(vals))
    t.add_column(0, vals)
    lo, hi, hn, hv = t.column_statistics(0)
    assert (lo, hi, hn, hv) == (int(bits_of([-3.0], dt)[0]), int(bits_of([math.inf], dt)[0]), False, True)
    vals[2] = dt(math.nan)
    t2 = CubitTable(ctx, len(vals))
    t2.add_column(0, vals)
    lo, hi, _, _ = t2.column_statistics(0)
    assert lo == int(bits_of([-2.0], dt)[0])
    assert math.isnan(np.array([hi], dtype=np.int64).astype(np.uint32 if dt == np.float32 else np.uint64)
                       .view(dt)[0])


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_low_level_k0_matches_oracle_bitvector(ctx, dt):
    rng = np.random.default_rng(9)
    n = 200_000
    vals, _, valid = random_column(rng, dt, n, null_frac=0.02)
    vw = validity_from_mask(valid)
    col = O.Column(vals, vw)
    d_col, d_val = ctx.upload(vals), ctx.upload(vw)
    words = ctx.lib.cubit_padded_words(n)
    out = ctx.alloc(words * 8)
    typ = L.TYPE_FLOAT if dt == np.float32 else L.TYPE_DOUBLE
    for c in [dt(0.0), dt(-0.0), dt(math.nan), dt(math.inf), dt(-1.0)]:
        cb = int(bits_of([c], dt)[0])
        for cmp_i in range(6):
            L.check(ctx.lib.cubit_build_bitvector(ctx.handle, d_col.ptr, typ, d_val.ptr, n, cmp_i, cb, out.ptr))
            ctx.check()
            got = out.download(np.uint64, (n + 63) // 64)
            assert np.array_equal(got, O.build_bitvector(col, n, cmp_i, cb)), (cmp_i, c)


# ------------------------------------------------------------------ MVCC, merges, appends


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("index", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_updates_merges_and_appends(ctx, dt, index):
    rng = np.random.default_rng(21)
    n = 250_000
    vals, pool, valid = random_column(rng, dt, n, null_frac=0.03)
    vw = validity_from_mask(valid)
    t = CubitTable(ctx, n)
    t.add_column(0, vals, vw)
    if index is not None:
        t.build_index(0, index)
    # updates: values from the pool and new ones (-0.0 / NaN payloads / fresh values), some SET NULL,
    # committed (versions below the start) and one writer's own
    m = 4000
    rows = np.sort(rng.choice(n, m, replace=False)).astype(np.int64)
    new = np.concatenate([pool, np.array([12345.5, -0.0], dtype=dt)])[rng.integers(0, len(pool) + 2, m)].astype(dt)
    upd_valid = rng.random(m) >= 0.1
    writer = TXN_START + 77
    versions = np.where(rng.random(m) < 0.7, 5, writer).astype(np.uint64)
    t.set_updates(0, rows, new, versions, upd_valid)
    ucol = O.Column(vals, vw, updates=(rows, new, versions, upd_valid))
    consts = [dt(0.0), dt(math.nan), dt(12345.5), dt(-1.0), dt(math.inf)] + list(pool[:4])
    for txn_id, start in [(writer, 10), (TXN_START + 1, 10), (TXN_START + 2, 3)]:
        txn, tx = L.Txn(start, txn_id), O.Mvcc(start, txn_id)
        for c in consts:
            for cmp in ("=", "<", ">=", "!="):
                fs = F.TableFilterSet({0: F.ConstantFilter(cmp, c)})
                assert np.array_equal(t.scan(fs, txn=txn), oracle_rows([ucol], fs, n, tx)), (txn_id, cmp, c)
        ids = np.arange(0, n, 97, dtype=np.int64)
        got, ok = t.fetch(0, ids, txn)
        want, wok = O.fetch(ucol, ids, tx=tx, with_valid=True)
        assert np.array_equal(ok, wok) and np.array_equal(got, want)
    # merge the committed records (version 5 < horizon 6): the base takes them, the writer's stay
    t.merge_updates(0, 6)
    merged = vals.copy()
    mvalid = valid.copy()
    committed = versions == 5
    merged[rows[committed]] = np.where(upd_valid[committed], new[committed], dt(0.0))
    mvalid[rows[committed]] = upd_valid[committed]
    mvw = validity_from_mask(mvalid)
    left = ~committed
    mcol = O.Column(merged, mvw, updates=(rows[left], new[left], versions[left], upd_valid[left]))
    tx_other = (L.Txn(10, TXN_START + 3), O.Mvcc(10, TXN_START + 3))
    tx_writer = (L.Txn(10, writer), O.Mvcc(10, writer))
    for c in consts:
        for cmp in ("=", "<=", ">"):
            fs = F.TableFilterSet({0: F.ConstantFilter(cmp, c)})
            for txn, tx in (tx_other, tx_writer):
                assert np.array_equal(t.scan(fs, txn=txn), oracle_rows([mcol], fs, n, tx)), (cmp, c)
    # append rows holding new values (an every-distinct-value index gains keys)
    extra, _, _ = random_column(rng, dt, 30_000)
    extra[:5] = np.array([99.0, -0.0, math.nan, 1e30, -5.5], dtype=dt)
    t.append({0: extra})
    allv = np.concatenate([merged, extra])
    allw = validity_from_mask(np.concatenate([mvalid, np.ones(len(extra), bool)]))
    acol = O.Column(allv, allw, updates=(rows[left], new[left], versions[left], upd_valid[left]))
    for c in [dt(99.0), dt(-5.5), dt(0.0), dt(math.nan), dt(1e30)]:
        for cmp in ("=", "<", ">="):
            fs = F.TableFilterSet({0: F.ConstantFilter(cmp, c)})
            txn, tx = tx_other
            assert np.array_equal(t.scan(fs, txn=txn), oracle_rows([acol], fs, len(allv), tx)), (cmp, c)


@pytest.mark.parametrize("index", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_nan_ordering_counts_on_gpu(ctx, dt, index):
    """nan_ordering.test's filtered counts (f > 0: 4, f < 0: 3 over 10,008 rows with two NaNs,
    ±inf and a NULL) through cubit_table_scan's count, with and without an index."""
    from test_oracle_float_filters import ORDERING, ordering_column

    vals, valid = ordering_column(dt)
    t = CubitTable(ctx, len(vals))
    t.add_column(0, vals, validity_from_mask(valid))
    if index is not None:
        t.build_index(0, index)
    for c in ORDERING["counts"]:
        fs = F.TableFilterSet({0: F.ConstantFilter(OPS[c["cmp"]], dt(float(c["constant"])))})
        assert t.count(fs) == c["count"], c["sql"]
    t.close()
