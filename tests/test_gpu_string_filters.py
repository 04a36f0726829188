"""VARCHAR columns on the GPU vs the oracle. The column is held as int32 codes of an
order-preserving dictionary (cubit_dict: the distinct strings in DuckDB's string order), so a
comparison with a string constant is planned as a comparison of codes (present or absent from the
dictionary) and runs through the same K0 / index / candidate-check / narrowing / zonemap / MVCC
machinery as an INTEGER column. Pinned by the reference's strtest / strings queries
(tests/golden/string_filter_cases.json); the random cases compare with the oracle's restatement of
FilterSelectionSwitch<string_t> (column_segment.cpp:278-349) on real strings (string_type.hpp:
143-206: unsigned bytes, then length), including the empty string, prefixes, NUL and high bytes."""
import json
from pathlib import Path

import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.scan_function import ROW_ID, CubitScanFunction
from cubit_amd.table import Context, CubitTable, Dictionary
from oracle import oracle as O

pytestmark = pytest.mark.gpu

CASES = json.loads((Path(__file__).resolve().parent / "golden" / "string_filter_cases.json").read_text())["cases"]
OPS = {"=": "=", "<>": "!=", "<": "<", "<=": "<=", ">": ">", ">=": ">="}
CMPS = ["=", "!=", "<", "<=", ">", ">="]
TXN_START = 4611686018427388000


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def filter_of(terms):
    fs = [F.ConstantFilter(OPS[op], lit) for op, lit in terms]
    return fs[0] if len(fs) == 1 else F.ConjunctionAndFilter(fs)


def random_strings(rng, n, pool=60):
    alphabet = [0x61, 0x62, 0x7A, 0x00, 0x7F, 0x80, 0xFF, 0x41]  # a b z NUL DEL 0x80 0xff A
    base = [b""] + [bytes(rng.choice(alphabet, rng.integers(1, 14)).tolist()) for _ in range(pool)]
    base += [base[3] + b"a", base[3] + b"\x00", base[3][:1], b"a" * 13, b"a" * 12]
    return [base[i] for i in rng.integers(0, len(base), n)], base


def absent_constants(pool):
    """Strings between, before and after the dictionary's: every comparison must still be exact."""
    return [b"", b"\x00", b"a" * 12 + b"\x00", b"a" * 14, b"\xff" * 20, b"m", pool[5] + b"\x01", pool[7][:-1] + b"\xfe"]


@pytest.mark.parametrize("index", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_reference_string_filter_cases(ctx, index):
    for case in CASES:
        rows = case["rows"]
        for q in case["queries"]:
            vals = [r[q["column"]] for r in rows]
            t = CubitTable(ctx, len(rows))
            t.add_string_column(0, vals)
            if index is not None:
                t.build_index(0, index)
            fs = F.TableFilterSet({0: filter_of(q["terms"])})
            got = t.scan(fs)
            proj = q["project"] if q["project"] is not None else q["column"]
            assert [rows[r][proj] for r in got] == q["rows"], q["sql"]
            assert np.array_equal(got, O.table_scan([O.StringColumn(vals)], F.serialize(fs), len(rows)))
            t.close()


def test_dictionary_order_and_lookup(ctx):
    rng = np.random.default_rng(1)
    vals, pool = random_strings(rng, 5000)
    d = Dictionary(vals)
    assert d.entries() == sorted(set(vals))  # Python's bytes order = DuckDB's string_t order
    for s in set(vals):
        assert d.lookup(s) == (d.entries().index(s), True)
    for s in absent_constants(pool):
        lb, present = d.lookup(s)
        assert present == (s in set(vals))
        assert lb == sum(1 for e in d.entries() if e < s)
    codes, valid = d.encode([vals[0], None, vals[2]])
    assert codes[0] == d.entries().index(vals[0]) and codes[1] == 0 and not valid[1]
    with pytest.raises(L.CubitError):
        d.encode([b"not in it \xfe\xfe"])


@pytest.mark.parametrize("index", ["none", "range_all", "range_keys", "equality", "bins"])
def test_random_comparisons_match_oracle(ctx, index):
    rng = np.random.default_rng(7)
    n = 300_007
    vals, pool = random_strings(rng, n)
    vals = [None if rng.random() < 0.04 else v for v in vals]
    t = CubitTable(ctx, n)
    t.add_string_column(0, vals)
    if index == "range_all":
        t.build_index(0, L.INDEX_RANGE)
    elif index == "range_keys":  # keys given as strings, some absent: constants between them take the candidate check
        t.build_index(0, L.INDEX_RANGE, sorted({b"", b"a", b"aaz", b"b", b"m", b"z\x80", b"\xff"}))
    elif index == "equality":
        t.build_index(0, L.INDEX_EQUALITY)
    elif index == "bins":
        t.build_index(0, L.INDEX_RANGE)
        t.build_index(0, L.INDEX_BINS, [b"", b"a", b"b", b"z", b"\xff\xff"])
    col = O.StringColumn(vals)
    consts = list(pool[:20]) + absent_constants(pool)
    for c in consts:
        for cmp in CMPS:
            fs = F.TableFilterSet({0: F.ConstantFilter(cmp, c)})
            want = O.table_scan([col], F.serialize(fs), n)
            assert np.array_equal(t.scan(fs), want), (index, cmp, c)
    for lo, hi in [(b"a", b"b"), (b"", b"\x00"), (b"b", b"zz"), (pool[4], pool[4] + b"\x00")]:
        fs = F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", lo), F.ConstantFilter("<", hi)])})
        assert np.array_equal(t.scan(fs), O.table_scan([col], F.serialize(fs), n)), (lo, hi)
    fs = F.TableFilterSet({0: F.ConjunctionOrFilter([F.ConstantFilter("=", b""), F.ConstantFilter(">", b"z"),
                                                     F.IsNullFilter()])})
    assert np.array_equal(t.scan(fs), O.table_scan([col], F.serialize(fs), n))
    t.close()


def test_conjunction_with_integer_column_and_probe(ctx):
    """A string comparison inside a selective conjunction (narrowing reads the codes at the kept
    rows only); the probe hands back codes that the dictionary decodes to the oracle's strings."""
    rng = np.random.default_rng(8)
    n = 1_000_003
    ints = rng.integers(0, 1000, n).astype(np.int32)
    vals, pool = random_strings(rng, n, pool=200)
    vals = sorted(vals)  # clustered: the zonemaps on codes skip zones
    vals = [None if i % 101 == 0 else v for i, v in enumerate(vals)]
    t = CubitTable(ctx, n)
    t.add_column(0, ints)
    d = t.add_string_column(1, vals)
    t.build_index(0, L.INDEX_RANGE)
    cols = [O.Column(ints), O.StringColumn(vals)]
    for (ilo, ihi), (cmp, c) in [((10, 12), (">", b"b")), ((500, 501), ("<=", b"a\x80")), ((0, 3), ("=", pool[9])),
                                 ((7, 9), ("!=", b""))]:
        fs = F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", ilo), F.ConstantFilter("<", ihi)]),
                               1: F.ConstantFilter(cmp, c)})
        for narrowing in (True, False):
            t.use_narrowing(narrowing)
            assert np.array_equal(t.scan(fs), O.table_scan(cols, F.serialize(fs), n)), (cmp, c)
        t.use_narrowing(True)
    fs = F.TableFilterSet({1: F.ConjunctionAndFilter([F.ConstantFilter(">=", b"b"), F.ConstantFilter("<", b"z")])})
    rows = t.scan(fs)
    assert np.array_equal(rows, O.table_scan(cols, F.serialize(fs), n))
    ev, nz = t.last_zones()
    assert ev < nz
    ids = rows[::37]
    codes, ok = t.fetch(1, ids)
    want, wok = O.fetch(cols[1], ids, with_valid=True)
    assert np.array_equal(ok, wok)
    assert [d.entry(c) if o else None for c, o in zip(codes, ok)] == cols[1].decode(want, wok)
    lo, hi, hn, hv = t.column_statistics(1)
    present = sorted(v for v in set(vals) if v is not None)
    assert (d.entry(lo), d.entry(hi), hn, hv) == (present[0], present[-1], True, True)
    t.close()


@pytest.mark.parametrize("index", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_updates_merges_and_appends(ctx, index):
    rng = np.random.default_rng(21)
    n = 250_000
    vals, pool = random_strings(rng, n)
    vals = [None if rng.random() < 0.03 else v for v in vals]
    d = Dictionary(pool)  # every pool string: updates and appends may use any of them
    t = CubitTable(ctx, n)
    t.add_string_column(0, vals, d)
    if index is not None:
        t.build_index(0, index)
    code = {s: i for i, s in enumerate(d.entries())}
    m = 3000
    rows = np.sort(rng.choice(n, m, replace=False)).astype(np.int64)
    new = [pool[i] for i in rng.integers(0, len(pool), m)]
    upd_valid = rng.random(m) >= 0.1
    writer = TXN_START + 77
    versions = np.where(rng.random(m) < 0.7, 5, writer).astype(np.uint64)
    t.set_updates(0, rows, np.array([code[s] for s in new], dtype=np.int64), versions, upd_valid)
    ovals = [s if ok else None for s, ok in zip(new, upd_valid)]
    ucol = O.StringColumn(vals, updates=(rows, ovals, versions, upd_valid))
    consts = [pool[3], pool[10], b"m", b""]
    for txn_id, start in [(writer, 10), (TXN_START + 1, 10), (TXN_START + 2, 3)]:
        txn, tx = L.Txn(start, txn_id), O.Mvcc(start, txn_id)
        for c in consts:
            for cmp in ("=", "<", ">=", "!="):
                fs = F.TableFilterSet({0: F.ConstantFilter(cmp, c)})
                assert np.array_equal(t.scan(fs, txn=txn), O.table_scan([ucol], F.serialize(fs), n, 0, tx)), (cmp, c)
        ids = np.arange(0, n, 97, dtype=np.int64)
        got, ok = t.fetch(0, ids, txn)
        want, wok = O.fetch(ucol, ids, tx=tx, with_valid=True)
        assert np.array_equal(ok, wok)
        assert [d.entry(g) if o else None for g, o in zip(got, ok)] == ucol.decode(want, wok)
    t.merge_updates(0, 6)
    committed = versions == 5
    merged = list(vals)
    for r, s, ok, cm in zip(rows, new, upd_valid, committed):
        if cm:
            merged[r] = s if ok else None
    left = ~committed
    mcol = O.StringColumn(merged, updates=(rows[left], [o for o, k in zip(ovals, left) if k], versions[left],
                                           upd_valid[left]))
    for txn, tx in [(L.Txn(10, TXN_START + 3), O.Mvcc(10, TXN_START + 3)), (L.Txn(10, writer), O.Mvcc(10, writer))]:
        for c in consts:
            for cmp in ("=", "<=", ">"):
                fs = F.TableFilterSet({0: F.ConstantFilter(cmp, c)})
                assert np.array_equal(t.scan(fs, txn=txn), O.table_scan([mcol], F.serialize(fs), n, 0, tx)), (cmp, c)
    extra = [pool[i] for i in rng.integers(0, len(pool), 20_000)]
    codes, _ = d.encode(extra)
    t.append({0: codes})
    acol = O.StringColumn(merged + extra, updates=(rows[left], [o for o, k in zip(ovals, left) if k], versions[left],
                                                   upd_valid[left]))
    txn, tx = L.Txn(10, TXN_START + 3), O.Mvcc(10, TXN_START + 3)
    for c in consts:
        for cmp in ("=", "<", ">="):
            fs = F.TableFilterSet({0: F.ConstantFilter(cmp, c)})
            assert np.array_equal(t.scan(fs, txn=txn), O.table_scan([acol], F.serialize(fs), n + len(extra), 0, tx))
    with pytest.raises(L.CubitError):  # a code outside the dictionary
        t.set_updates(0, np.array([1], dtype=np.int64), np.array([len(d)], dtype=np.int64), np.array([5], np.uint64))
    t.close()


@pytest.mark.parametrize("tasks", [1, 4])
def test_string_column_through_table_function(ctx, tasks):
    """A VARCHAR filter and projection through the table function: the row ids equal the oracle's
    scan, and the projected codes (crossing PCIe at the width their statistics allow) decode to the
    oracle's strings, NULL-ness included."""
    rng = np.random.default_rng(9)
    n = 700_001
    vals, pool = random_strings(rng, n)
    vals = [None if rng.random() < 0.05 else v for v in vals]
    t = CubitTable(ctx, n)
    d = t.add_string_column(0, vals)
    t.build_index(0, L.INDEX_RANGE)
    col = O.StringColumn(vals)
    for fs in [F.TableFilterSet({0: F.ConstantFilter("<", b"aa")}),
               F.TableFilterSet({0: F.ConjunctionOrFilter([F.ConstantFilter("=", pool[2]),
                                                           F.ConstantFilter(">", b"z")])})]:
        keep = O.table_scan([col], F.serialize(fs), n)
        fn = CubitScanFunction(t, [ROW_ID, 0], [0, 1], fs)
        from test_gpu_scan_function import drain, ordered

        chunks = drain(fn, tasks, validity=True)
        fn.close()
        assert np.array_equal(ordered(chunks, 0), keep)
        codes, ok = ordered(chunks, 1), ordered(chunks, 3)
        want, wok = O.fetch(col, keep, with_valid=True)
        assert np.array_equal(ok, wok)
        assert [d.entry(c) if o else None for c, o in zip(codes, ok)] == col.decode(want, wok)
    t.close()


def test_index_files_name_their_dictionary(ctx, tmp_path):
    """A saved index on a dictionary column loads beside the same dictionary (scans equal the
    built index's) and is refused against another dictionary or onto a column of another type:
    its codes would name other strings."""
    rng = np.random.default_rng(41)
    n = 100_003
    vals, pool = random_strings(rng, n)
    d = Dictionary(pool)
    t = CubitTable(ctx, n)
    t.add_string_column(0, vals, d)
    t.build_index(0, L.INDEX_EQUALITY)
    path = tmp_path / "eq.cix"
    t.save_index(0, L.INDEX_EQUALITY, path)
    fs = F.TableFilterSet({0: F.ConstantFilter("=", pool[4])})
    want = t.scan(fs)
    u = CubitTable(ctx, n)
    u.add_string_column(0, vals, d)
    u.load_index(0, path)
    assert u.index_info(0)[0] == t.index_info(0)[0]
    assert np.array_equal(u.scan(fs), want)
    other = CubitTable(ctx, n)
    other.add_string_column(0, vals, Dictionary(pool + [b"not in the first one"]))
    with pytest.raises(L.CubitError):
        other.load_index(0, path)
    ints = CubitTable(ctx, n)
    ints.add_column(0, np.zeros(n, dtype=np.int32))
    with pytest.raises(L.CubitError):
        ints.load_index(0, path)
    for x in (t, u, other, ints):
        x.close()


def test_equality_index_plans_intervals_as_one_union(ctx):
    """On an every-value equality index, bounds on one column fold into one interval read as the
    union of the keys inside it, or the valid rows minus the union of those outside — the fewer
    bitvectors (l_shipmode's seven modes: [RAIL, SHIP) reads 2, not 4 + 5) — with NULLs, and
    after update records (a value that is not a key makes the index inexact: K0 then)."""
    rng = np.random.default_rng(43)
    n = 300_007
    modes = [b"AIR", b"FOB", b"MAIL", b"RAIL", b"REG AIR", b"SHIP", b"TRUCK"]
    vals = [None if rng.random() < 0.05 else modes[i] for i in rng.integers(0, 7, n)]
    d = Dictionary(modes + [b"ZZZ"])  # one entry no row holds: an update may bring it in
    t = CubitTable(ctx, n)
    t.add_string_column(0, vals, d)
    t.build_index(0, L.INDEX_EQUALITY)
    col = O.StringColumn(vals)
    cases = [
        ([(">=", b"RAIL"), ("<", b"SHIP")], 2),            # inside: RAIL, REG AIR
        ([(">", b"AIR"), ("<=", b"TRUCK")], 1),            # outside: AIR (valid rows minus it)
        ([(">=", b"B"), ("<", b"S")], 3),                  # absent bounds: FOB, MAIL, RAIL... as codes
        ([(">=", b"MAIL")], 3),                            # one bound: outside AIR, FOB, (ZZZ absent)
        ([("<", b"MAIL"), (">", b"AIR"), ("<=", b"FOB")], 1),
        ([(">", b"TRUCK")], 0),
    ]
    for terms, max_leaves in cases:
        flt = F.ConjunctionAndFilter([F.ConstantFilter(op, c) for op, c in terms]) if len(terms) > 1 else \
            F.ConstantFilter(*terms[0])
        fs = F.TableFilterSet({0: flt})
        want = O.table_scan([col], F.serialize(fs), n)
        assert np.array_equal(t.scan(fs), want), terms
        leaves, _ = t.last_plan()
        assert leaves <= max_leaves + 1, (terms, leaves)  # + the validity leaf
    # an update to a code no row held before: the index stops being every-value, plans fall back
    rows = np.array([5, 17, 900], dtype=np.int64)
    t.set_updates(0, rows, np.array([7, 3, 7], dtype=np.int64), np.array([1, 1, 1], dtype=np.uint64))
    ucol = O.StringColumn(vals, updates=(rows, [b"ZZZ", b"RAIL", b"ZZZ"], np.array([1, 1, 1], dtype=np.uint64)))
    txn, tx = L.Txn(5, TXN_START + 1), O.Mvcc(5, TXN_START + 1)
    for terms, _ in cases:
        flt = F.ConjunctionAndFilter([F.ConstantFilter(op, c) for op, c in terms]) if len(terms) > 1 else \
            F.ConstantFilter(*terms[0])
        fs = F.TableFilterSet({0: flt})
        assert np.array_equal(t.scan(fs, txn=txn), O.table_scan([ucol], F.serialize(fs), n, 0, tx)), terms
    t.close()


def test_device_dictionary_encode_equals_host(ctx):
    """cubit_dict_encode_device (one GPU lane per string, a search of the dictionary's entries in
    unsigned-byte-then-length order) gives the host encoder's codes — strings with NUL and high
    bytes, the empty string, prefixes, NULL rows — and refuses strings the dictionary lacks,
    marking them -1. Device buffers through the C ABI's own allocator."""
    import ctypes as C

    from cubit_amd.datagen import validity_from_mask
    from cubit_amd.table import pack_strings

    lib, h = ctx.lib, ctx.handle
    bufs = []

    def dev(a):
        a = np.ascontiguousarray(a)
        p = C.c_void_p()
        L.check(lib.cubit_dev_alloc(h, max(a.nbytes, 16), C.byref(p)))
        L.check(lib.cubit_memcpy_h2d(h, p, a.ctypes.data, a.nbytes))
        bufs.append(p)
        return p

    def back(p, n):
        out = np.empty(n, np.int32)
        L.check(lib.cubit_memcpy_d2h(h, out.ctypes.data, p, out.nbytes))
        return out

    rng = np.random.default_rng(51)
    vals, pool = random_strings(rng, 400_003, pool=300)
    vals = [None if rng.random() < 0.03 else v for v in vals]
    d = Dictionary(pool)
    want, wvalid = d.encode(vals)
    buf, offs, valid = pack_strings(vals)
    d_codes = dev(np.full(len(vals), 7, np.int32))
    L.check(lib.cubit_dict_encode_device(h, d.handle, dev(buf), dev(offs), len(vals), dev(validity_from_mask(valid)),
                                         d_codes))
    got = back(d_codes, len(vals))
    assert np.array_equal(got[wvalid], want[wvalid]) and (got[~wvalid] == 0).all()
    # two strings the dictionary lacks: refused, their codes -1, the others still encoded
    extra = list(vals[:1000]) + [b"not there", b"\xff" * 40]
    buf, offs, valid = pack_strings(extra)
    d_codes = dev(np.zeros(len(extra), np.int32))
    rc = lib.cubit_dict_encode_device(h, d.handle, dev(buf), dev(offs), len(extra), None, d_codes)
    assert rc == L.ERR_UNSUPPORTED
    got = back(d_codes, len(extra))
    assert got[-2:].tolist() == [-1, -1]
    w2, v2 = d.encode(extra[:1000])
    assert np.array_equal(got[:1000][v2], w2[v2])
    for p in bufs:
        L.check(lib.cubit_dev_free(h, p))
