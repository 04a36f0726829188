"""HUGEINT / UHUGEINT table filters on the oracle (FilterSelectionSwitch<hugeint_t / uhugeint_t>,
column_segment.cpp:468-479: 128-bit comparisons, signed / unsigned), pinned by the reference's own
tests (tests/golden/huge_filter_cases.json, made by make_huge_golden.py from
test/sql/types/{hugeint,uhugeint}/test_*_ops.test, *_null_value.test and
test/sql/storage/types/test_*_storage.test); and the 16-byte order key the GPU path holds such a
column by (cubit_key128 in include/cubit_gpu.h, filters.key128): its byte order must be the values'
order exactly, checked against the oracle's 128-bit comparisons. No GPU."""
import ctypes as C
import json
import subprocess

import numpy as np
import pytest

from cubit_amd import filters as F
from oracle import oracle as O
from test_abi import ROOT

CMPS = ["=", "!=", "<", "<=", ">", ">="]
OPS = {"=": lambda a, b: a == b, "!=": lambda a, b: a != b, "<": lambda a, b: a < b, "<=": lambda a, b: a <= b,
       ">": lambda a, b: a > b, ">=": lambda a, b: a >= b}
I128 = (-(1 << 127), (1 << 127) - 1)
U128 = (0, (1 << 128) - 1)


def golden_cases():
    return json.loads((ROOT / "tests" / "golden" / "huge_filter_cases.json").read_text())["cases"]


def edges(signed):
    lo, hi = I128 if signed else U128
    e = [lo, lo + 1, hi - 1, hi, 0, 1, 42, 2 ** 63 - 1, 2 ** 63, 2 ** 64 - 1, 2 ** 64, 2 ** 64 + 1, 2 ** 100]
    if signed:
        e += [-1, -2, -(2 ** 63), -(2 ** 63) - 1, -(2 ** 64), -(2 ** 64) - 1, -(2 ** 100)]
    return [v for v in e if lo <= v <= hi]


def pool(signed, rng, k=80):
    lo, hi = I128 if signed else U128
    out = edges(signed)
    for _ in range(k):
        bits = int(rng.integers(1, 128))
        v = int.from_bytes(rng.bytes(16), "big") >> (128 - bits)
        if signed and rng.random() < 0.5:
            v = -v - 1
        out.append(min(max(v, lo), hi))
    return out


def huge_filter(op, v):
    """A comparison on a HUGEINT column as the oracle takes it: the constant's ohuge address."""
    return F.ConstantFilter(op, O.huge_ref(v))


def oracle_filters(fs, residual, huge):
    """A filter set + residual written for the GPU (constants on HUGEINT / UHUGEINT columns as their
    order keys, filters.key128) restated for the oracle (those constants as ohuge addresses);
    huge = {column: signed}."""
    def tf(f, signed):
        if isinstance(f, F.ConstantFilter):
            return F.ConstantFilter(f.comparison, O.huge_ref(F.value128(f.constant, signed)))
        if isinstance(f, (F.ConjunctionAndFilter, F.ConjunctionOrFilter)):
            return type(f)([tf(c, signed) for c in f.child_filters])
        return f

    def rf(r):
        if isinstance(r, F.Cmp) and r.column in huge:
            return F.Cmp(r.column, r.comparison, O.huge_ref(F.value128(r.constant, huge[r.column])))
        if isinstance(r, (F.And, F.Or)):
            return type(r)(*[rf(c) for c in r.children])
        return r

    out = F.TableFilterSet()
    for c, f in fs.filters.items():
        out.filters[c] = tf(f, huge[c]) if c in huge else f
    return out, (None if residual is None else rf(residual))


def answer(case, q, rows, cols):
    """The query's result lines from the rows its pushed filter kept (as sqllogictest prints them)."""
    h = case["columns"].index("h")
    vals = cols[h].decode(*O.fetch(cols[h], rows, with_valid=True))
    sel = q["select"]
    if sel == "COUNT(*)":
        return [str(len(rows))]
    if sel.startswith("id, FIRST(h), LAST(h)"):  # GROUP BY id over rows whose h IS NULL
        ids = O.fetch(cols[case["columns"].index("id")], rows)
        return [f"{i}\tNULL\tNULL" for i in sorted(set(ids.tolist()))]
    out = [str(v) for v in vals]
    return sorted(out, key=int) if "ORDER BY" in q["sql"] else out


def columns_of(case):
    cols = []
    for j, t in enumerate(case["types"]):
        vals = [None if r[j] is None else int(r[j]) for r in case["rows"]]
        if t in ("HUGEINT", "UHUGEINT"):
            cols.append(O.HugeColumn(vals, signed=t == "HUGEINT"))
        else:
            cols.append(O.Column(np.array(vals, dtype=np.int32)))
    return cols


@pytest.mark.parametrize("case", golden_cases(), ids=lambda c: c["file"].rsplit("/", 1)[1])
def test_oracle_matches_reference_rows(case):
    cols = columns_of(case)
    h = case["columns"].index("h")
    n = len(case["rows"])
    for q in case["queries"]:
        flt = F.IsNullFilter() if q["cmp"] == "IS NULL" else huge_filter(q["cmp"], int(q["constant"]))
        rows = O.table_scan(cols, F.serialize(F.TableFilterSet({h: flt})), n)
        assert answer(case, q, rows, cols) == q["rows"], q["sql"]


@pytest.mark.parametrize("signed", [True, False])
def test_oracle_compares_128_bit_values(signed):
    rng = np.random.default_rng(11 if signed else 12)
    vals = pool(signed, rng)
    vals = [vals[i] for i in rng.integers(0, len(vals), 5000)] + [None] * 40
    rng.shuffle(vals)
    col = O.HugeColumn(vals, signed=signed)
    n = len(vals)
    ok = np.array([v is not None for v in vals])
    for c in edges(signed) + [vals[i] for i in rng.integers(0, n, 8) if vals[i] is not None]:
        for op in CMPS:
            got = O.table_scan([col], F.serialize(F.TableFilterSet({0: huge_filter(op, c)})), n)
            want = np.array([i for i, v in enumerate(vals) if v is not None and OPS[op](v, c)], dtype=np.int64)
            assert np.array_equal(got, want), (op, c)
    # NULL tests and a disjunction across the sign / 2^64 boundaries
    got = O.table_scan([col], F.serialize(F.TableFilterSet({0: F.IsNullFilter()})), n)
    assert np.array_equal(got, np.flatnonzero(~ok))
    b = 2 ** 64 if not signed else -1
    fs = F.TableFilterSet({0: F.ConjunctionOrFilter([F.IsNullFilter(), huge_filter(">", b)])})
    got = O.table_scan([col], F.serialize(fs), n)
    assert np.array_equal(got, np.array([i for i, v in enumerate(vals) if v is None or v > b], dtype=np.int64))


@pytest.mark.parametrize("signed", [True, False])
def test_oracle_update_records_carry_128_bit_values(signed):
    rng = np.random.default_rng(13)
    p = pool(signed, rng, 20)
    n = 3000
    vals = [p[i] for i in rng.integers(0, len(p), n)]
    rows = np.sort(rng.choice(n, 200, replace=False)).astype(np.int64)
    new = [None if rng.random() < 0.1 else p[i] for i in rng.integers(0, len(p), 200)]
    ver = np.where(rng.random(200) < 0.6, 5, 4611686018427388000 + 9).astype(np.uint64)
    col = O.HugeColumn(vals, signed=signed, updates=(rows, new, ver))
    tx = O.Mvcc(10, 4611686018427388000 + 1)
    seen = list(vals)
    for r, v, t in zip(rows, new, ver):
        if t == 5:
            seen[r] = v
    got_v, got_ok = O.fetch(col, np.arange(n), tx=tx, with_valid=True)
    assert col.decode(got_v, got_ok) == seen
    for c in edges(signed)[:6]:
        for op in CMPS:
            got = O.table_scan([col], F.serialize(F.TableFilterSet({0: huge_filter(op, c)})), n, 0, tx)
            want = [i for i, v in enumerate(seen) if v is not None and OPS[op](v, c)]
            assert got.tolist() == want, (op, c)


# ---- the order key (C header helpers, compiled here) ---------------------------------------------
SRC = r"""
#include "cubit_gpu.h"
void key128(int type, uint64_t lower, uint64_t upper, unsigned char *key) { cubit_key128(type, lower, upper, key); }
void value128(int type, const unsigned char *key, uint64_t *lower, uint64_t *upper) {
    cubit_value128(type, key, lower, upper);
}
"""


@pytest.fixture(scope="module")
def keylib(tmp_path_factory):
    d = tmp_path_factory.mktemp("key128")
    (d / "k.c").write_text(SRC)
    so = d / "k.so"
    subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-Werror", "-shared", "-fPIC", "-I", str(ROOT / "include"),
                    str(d / "k.c"), "-o", str(so)], check=True)
    lib = C.CDLL(str(so))
    lib.key128.argtypes = [C.c_int, C.c_uint64, C.c_uint64, C.c_void_p]
    lib.value128.argtypes = [C.c_int, C.c_void_p, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    return lib


@pytest.mark.parametrize("signed", [True, False])
def test_key_bytes_order_as_the_values(keylib, signed):
    """cubit_key128 == filters.key128; unsigned byte order of the keys == the oracle's 128-bit
    comparisons; cubit_value128 inverts the key."""
    rng = np.random.default_rng(14)
    vals = pool(signed, rng, 200)
    typ = 11 if signed else 12
    keys = []
    for v in vals:
        u = v & ((1 << 128) - 1)
        buf = (C.c_ubyte * 16)()
        keylib.key128(typ, u & (2 ** 64 - 1), u >> 64, buf)
        k = bytes(buf)
        assert k == F.key128(v, signed) and F.value128(k, signed) == v
        lo, hi = C.c_uint64(), C.c_uint64()
        keylib.value128(typ, buf, C.byref(lo), C.byref(hi))
        assert (hi.value << 64 | lo.value) == u
        keys.append(k)
    col = O.HugeColumn(vals, signed=signed)
    n = len(vals)
    for j in rng.integers(0, n, 25):
        for cmp, op in enumerate(CMPS):
            words = O.build_bitvector(col, n, cmp, O.huge_ref(vals[j]))
            want = [bool((int(words[i >> 6]) >> (i & 63)) & 1) for i in range(n)]
            assert [OPS[op](k, keys[j]) for k in keys] == want, (op, vals[j])
