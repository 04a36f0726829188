"""Random filters over the typed columns (round 6) vs the oracle: a DOUBLE and a FLOAT column
holding NaN / ±0 / ±inf / subnormals, a VARCHAR column (dictionary codes; strings with the empty
string, NUL and high bytes, constants present and absent), a full-range UBIGINT column and a HUGEINT
column (codes of a dictionary over 16-byte order keys; values across the sign, 2^64 and the bounds,
constants present and absent; the oracle compares the 128-bit values themselves), each with
NULLs and a random index (none, every-value range, equality, range edges + bins); random pushed
TableFilterSets and residual AND/OR trees over them under three snapshots (committed / writer /
reader deletes, and in every other round update records of each type, SET NULL included); every
scan against the oracle's restatement (FilterSelectionSwitch<float / double / string_t /
uint64_t / hugeint_t>), every third one also through the table function (row ids, values as stored —
FLOAT / DOUBLE patterns, UBIGINT bits, VARCHAR and HUGEINT codes decoded — and NULL-ness against the
oracle's fetch).
scripts/fuzz_soak.py runs typed_round at a larger size for a wall-clock budget."""
import math
import threading

import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from cubit_amd.scan_function import ROW_ID, CubitScanFunction
from cubit_amd.table import Context, CubitTable, Dictionary
from oracle import oracle as O
from test_oracle_huge_filters import oracle_filters

pytestmark = pytest.mark.gpu

TXN_START = 4611686018427388000
CMPS = ["=", "!=", "<", "<=", ">", ">="]
KINDS = ["double", "float", "varchar", "ubigint", "hugeint"]
HUGE = {4: True}  # column 4: HUGEINT (signed)


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def pools(rng):
    """Per kind: the values rows draw from, and constants (the pool plus values absent from it)."""
    fl = [0.0, -0.0, math.inf, -math.inf, math.nan, 1.5, -1.5, 2.5, 1e-40, -3.0, 100.0]
    dbl = np.array(fl + list(rng.standard_normal(12) * 50) + [5e-324, -1e300], dtype=np.float64)
    dbl = np.concatenate([dbl, np.array([0xFFF8000000000001], dtype=np.uint64).view(np.float64)])  # -NaN payload
    flt = np.array(fl + list(rng.standard_normal(12) * 50), dtype=np.float32)
    strs = [b"", b"\x00", b"a", b"a\x00", b"ab", b"b", b"\x80", b"\xff\xff", b"zz", b"A", b"abc" * 5] + \
        [bytes(rng.integers(0, 256, rng.integers(1, 6)).tolist()) for _ in range(10)]
    ub = np.concatenate([np.array([0, 1, 2 ** 63 - 1, 2 ** 63, 2 ** 64 - 1], dtype=np.uint64),
                         rng.integers(0, 2 ** 64 - 1, 15, dtype=np.uint64, endpoint=True)])
    hi = (1 << 127) - 1
    hg = sorted({-hi - 1, -hi, -(2 ** 64), -1, 0, 1, 2 ** 63, 2 ** 64, hi - 1, hi} |
                {int(rng.integers(-2 ** 62, 2 ** 62)) << int(rng.integers(0, 64)) for _ in range(10)})
    consts = {"double": list(dbl) + [3.25, -math.inf],
              "float": list(flt) + [np.float32(3.25)],
              "varchar": strs + [b"a\x01", b"zzz", b"\xff\xff\xff", b"m"],
              "ubigint": [int(x) for x in ub] + [2 ** 63 + 7, 12345],
              "hugeint": hg + [2 ** 64 + 1, -(2 ** 64) - 1, 7, hi - 2]}
    return {"double": dbl, "float": flt, "varchar": strs, "ubigint": ub, "hugeint": hg}, consts


def const_of(kind, c):
    """A constant as the filter classes take it: FLOAT as np.float32, DOUBLE as float, VARCHAR bytes,
    UBIGINT int, HUGEINT its order key."""
    if kind == "hugeint":
        return F.key128(c, True)
    if kind == "float":
        return np.float32(c)
    if kind == "double":
        return float(c)
    return c


def rand_filter(rng, kind, consts, depth=0):
    r = rng.random()
    if depth < 2 and r < 0.2:
        kids = [rand_filter(rng, kind, consts, depth + 1) for _ in range(rng.integers(2, 4))]
        return F.ConjunctionAndFilter(kids) if rng.random() < 0.6 else F.ConjunctionOrFilter(kids)
    if r < 0.27:
        return F.IsNullFilter() if rng.random() < 0.5 else F.IsNotNullFilter()
    cs = consts[kind]
    return F.ConstantFilter(CMPS[rng.integers(0, 6)], const_of(kind, cs[rng.integers(0, len(cs))]))


def rand_residual(rng, consts, depth=0):
    if depth < 2 and rng.random() < 0.5:
        kids = [rand_residual(rng, consts, depth + 1) for _ in range(rng.integers(2, 4))]
        return F.And(*kids) if rng.random() < 0.5 else F.Or(*kids)
    c = int(rng.integers(0, len(KINDS)))
    if rng.random() < 0.1:
        return F.IsNull(c)
    cs = consts[KINDS[c]]
    return F.Cmp(c, CMPS[rng.integers(0, 6)], const_of(KINDS[c], cs[rng.integers(0, len(cs))]))


def typed_round(ctx, seed, n, with_updates, n_cases=24):
    """One random table of the four typed columns and n_cases random scans; returns the scans checked."""
    rng = np.random.default_rng(seed)
    pool, consts = pools(rng)
    row_base = int(rng.integers(0, 1 << 40))
    t = CubitTable(ctx, n, row_base=row_base)
    valid = [rng.random(n) > 0.08 for _ in range(len(KINDS))]
    vw = [validity_from_mask(v) for v in valid]
    dbl = pool["double"][rng.integers(0, len(pool["double"]), n)]
    flt = pool["float"][rng.integers(0, len(pool["float"]), n)]
    strs = [pool["varchar"][i] if ok else None for i, ok in zip(rng.integers(0, len(pool["varchar"]), n), valid[2])]
    ub = pool["ubigint"][rng.integers(0, len(pool["ubigint"]), n)]
    t.add_column(0, dbl, vw[0])
    t.add_column(1, flt, vw[1])
    d = Dictionary(pool["varchar"])
    t.add_string_column(2, strs, d)
    t.add_column(3, ub, vw[3])
    hg = [pool["hugeint"][i] if ok else None for i, ok in zip(rng.integers(0, len(pool["hugeint"]), n), valid[4])]
    dh = Dictionary([F.key128(v, True) for v in pool["hugeint"]])
    t.add_huge_column(4, hg, True, dh)
    for c, kind in enumerate(KINDS):
        choice = rng.integers(0, 4)
        if choice == 1:
            t.build_index(c, L.INDEX_RANGE)
        elif choice == 2:
            t.build_index(c, L.INDEX_EQUALITY)
        elif choice == 3:
            picks = (pool[kind][rng.integers(0, len(pool[kind]), 4)].tolist() if kind not in ("varchar", "hugeint")
                     else [pool[kind][i] for i in rng.integers(0, len(pool[kind]), 4)])
            # distinct (-0.0 and +0.0 are one key), ascending, NaN left out
            keys = sorted({k for k in picks if not (isinstance(k, float) and math.isnan(k))})
            if kind == "float":
                keys = np.array(keys, dtype=np.float32)
            if len(keys) >= 2:
                t.build_index(c, L.INDEX_RANGE, keys)
                t.build_index(c, L.INDEX_BINS, keys)
    writer = TXN_START + 5
    upd = {}
    code = {s: i for i, s in enumerate(d.entries())}
    hcode = {v: i for i, v in enumerate(pool["hugeint"])}  # the pool is sorted: its ranks are the codes
    if with_updates:
        for c, kind in enumerate(KINDS):
            rows = np.sort(rng.choice(n, size=n // 100, replace=False)).astype(np.int64)
            ok = rng.random(len(rows)) > 0.15
            vers = np.where(rng.random(len(rows)) < 0.5, np.uint64(3), np.uint64(writer)).astype(np.uint64)
            pick = rng.integers(0, len(pool[kind]), len(rows))
            if kind in ("varchar", "hugeint"):
                vals = [pool[kind][i] for i in pick]
                cm = code if kind == "varchar" else hcode
                t.set_updates(c, rows, np.array([cm[s] for s in vals], np.int64), vers, ok)
                upd[c] = (rows, [s if k else None for s, k in zip(vals, ok)], vers, ok)
            else:
                vals = pool[kind][pick]
                t.set_updates(c, rows, vals, vers, ok)
                upd[c] = (rows, vals, vers, ok)
    ocols = [O.Column(dbl, vw[0], updates=upd.get(0)), O.Column(flt, vw[1], updates=upd.get(1)),
             O.StringColumn(strs, updates=upd.get(2)), O.Column(ub, vw[3], updates=upd.get(3)),
             O.HugeColumn(hg, signed=True, updates=upd.get(4))]
    del_rows = np.sort(rng.choice(n, size=n // 20, replace=False)).astype(np.int64)
    del_ids = np.where(rng.random(len(del_rows)) < 0.5, np.uint64(4), np.uint64(writer)).astype(np.uint64)
    t.set_deletes(del_rows, del_ids)
    deleted = np.full(n, np.uint64(2 ** 64 - 2), dtype=np.uint64)
    deleted[del_rows] = del_ids
    views = [(2, writer), (2, TXN_START + 6), (10, TXN_START + 7)]
    checks = 0
    for i in range(n_cases):
        cols = rng.choice(len(KINDS), size=rng.integers(0, len(KINDS)), replace=False)
        fs = F.TableFilterSet({int(c): rand_filter(rng, KINDS[c], consts) for c in cols})
        residual = rand_residual(rng, consts) if rng.random() < 0.4 else None
        start, tid = views[i % 3]
        tx = O.Mvcc(start, tid, deleted=deleted)
        ref = O.table_scan(ocols, F.serialize(*oracle_filters(fs, residual, HUGE)), n, row_base=row_base, tx=tx)
        got = np.sort(t.scan(fs, residual, txn=L.Txn(start, tid), ordered=bool(i % 2)))
        if not np.array_equal(got, ref):
            raise AssertionError(f"typed seed {seed} case {i}: {len(got)} vs {len(ref)} rows; {fs} {residual}")
        if i % 3 == 0:
            table_function_check(t, rng, fs, residual, L.Txn(start, tid), ref, ocols, (d, dh), row_base, tx,
                                 f"typed seed {seed} case {i}")
        checks += 1
    t.close()
    return checks


def table_function_check(t, rng, fs, residual, txn, ref, ocols, d, row_base, tx, label):
    keep = [int(c) for c in rng.permutation(len(KINDS))[: int(rng.integers(1, len(KINDS) + 1))]]
    fn = CubitScanFunction(t, list(range(len(KINDS))) + [ROW_ID], [len(KINDS)] + keep, fs, residual, txn=txn)
    parts, lock = [], threading.Lock()

    def task():
        local = fn.init_local()
        while True:
            vals, masks = fn.function_validity(local)
            if len(vals[0]) == 0:
                return
            with lock:
                parts.append((vals, masks))

    th = [threading.Thread(target=task) for _ in range(int(rng.integers(1, 4)))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    fn.close()
    if not parts:
        assert len(ref) == 0, label
        return
    ids = np.concatenate([p[0][0] for p in parts])
    o = np.argsort(ids, kind="stable")
    assert np.array_equal(ids[o], ref), label
    for k, c in enumerate(keep, start=1):
        vals = np.concatenate([p[0][k] for p in parts])[o]
        valid = np.concatenate([p[1][k] for p in parts])[o]
        rv, rvalid = O.fetch(ocols[c], ref, row_base=row_base, tx=tx, with_valid=True)
        assert np.array_equal(valid, rvalid), (label, c)
        if c == 2:  # VARCHAR: codes against the oracle's strings
            assert [d[0].entry(v) if ok else None for v, ok in zip(vals, valid)] == ocols[2].decode(rv, rvalid), label
        elif c == 4:  # HUGEINT: codes against the oracle's 128-bit values
            assert [F.value128(d[1].entry(v)) if ok else None for v, ok in zip(vals, valid)] == \
                ocols[4].decode(rv, rvalid), label
        else:
            assert np.array_equal(vals[valid], rv[rvalid]), (label, c)


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
def test_typed_random_filters_match_oracle(ctx, seed):
    assert typed_round(ctx, 7000 + seed, 300_007, with_updates=bool(seed % 2)) == 24


@pytest.mark.parametrize("tasks", [1, 3])
def test_typed_columns_over_partitions(tasks):
    """A table of DOUBLE, VARCHAR (one dictionary, codes global) and UBIGINT columns held as three
    partitions on three contexts, scanned through one table-function cursor
    (cubit_scan_init_global_multi): rows and values equal the whole-table oracle; the statistics
    callback merges the partitions' bounds in each type's order (DOUBLE by its comparison key —
    a negative maximum is not the largest pattern — and UBIGINT unsigned)."""
    from cubit_amd import scan_function as S

    rng = np.random.default_rng(77)
    n, world = 700_003, 3
    dbl = (rng.standard_normal(n) * 100 - 400).astype(np.float64)  # mostly negative: bit order ≠ value order
    dbl[rng.integers(0, n, 50)] = math.nan
    ub = rng.integers(0, 2 ** 64 - 1, n, dtype=np.uint64, endpoint=True)
    words = [b"", b"a", b"ab", b"b", b"\x80", b"zz"]
    strs = [words[i] for i in rng.integers(0, len(words), n)]
    d = Dictionary(words)
    codes, _ = d.encode(strs)
    ctxs = [Context(0) for _ in range(world)]
    cuts = [0, 250_000, 480_000, n]
    tables = []
    for r in range(world):
        b, e = cuts[r], cuts[r + 1]
        t = CubitTable(ctxs[r], e - b, row_base=b)
        t.add_column(0, dbl[b:e])
        seg = np.ascontiguousarray(codes[b:e])
        L.check(t.lib.cubit_table_add_dict_column(t.handle, 1, d.handle, seg.ctypes.data, None, 0))
        t.types[1] = L.TYPE_VARCHAR
        t.add_column(2, ub[b:e])
        t.build_index(1, L.INDEX_EQUALITY)
        tables.append(t)
    lo, hi, hn, hv = S.statistics(tables, 0)
    finite = dbl[~np.isnan(dbl)]
    assert np.array([lo]).view(np.float64)[0] == finite.min() and math.isnan(np.array([hi]).view(np.float64)[0])
    lo, hi, _, _ = S.statistics(tables, 2)
    assert (lo & (2 ** 64 - 1), hi & (2 ** 64 - 1)) == (int(ub.min()), int(ub.max()))
    ocols = [O.Column(dbl), O.StringColumn(strs), O.Column(ub)]
    for fs in [F.TableFilterSet({0: F.ConstantFilter(">", -350.0), 1: F.ConstantFilter("<=", b"ab")}),
               F.TableFilterSet({2: F.ConstantFilter(">=", 2 ** 63), 1: F.ConstantFilter("!=", b"b")}),
               F.TableFilterSet({0: F.ConstantFilter("=", math.nan)})]:
        ref = O.table_scan(ocols, F.serialize(fs), n)
        fn = S.CubitScanFunction(tables, [0, 1, 2, ROW_ID], [3, 0, 1, 2], fs)
        parts, lock = [], threading.Lock()

        def task():
            local = fn.init_local()
            while True:
                vals = fn.function(local)
                if len(vals[0]) == 0:
                    return
                with lock:
                    parts.append(vals)

        th = [threading.Thread(target=task) for _ in range(tasks)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        fn.close()
        ids = np.concatenate([p[0] for p in parts])
        o = np.argsort(ids, kind="stable")
        assert np.array_equal(ids[o], ref)
        assert np.array_equal(np.concatenate([p[1] for p in parts])[o], O.fp_bits(dbl[ref], np.float64))
        assert [d.entry(c) for c in np.concatenate([p[2] for p in parts])[o]] == [strs[i] for i in ref]
        assert np.array_equal(np.concatenate([p[3] for p in parts])[o].view(np.uint64), ub[ref])
    for t in tables:
        t.close()
    for c in ctxs:
        c.close()
