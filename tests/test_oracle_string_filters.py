"""VARCHAR table filters on the oracle (FilterSelectionSwitch<string_t>,
src/storage/table/column_segment.cpp:278-349, with string_t's operators, src/include/duckdb/common/
types/string_type.hpp:143-206: the bytes compared as unsigned, a prefix before its extensions),
pinned by the reference's strtest / strings queries (tests/golden/string_filter_cases.json), and
the restated order checked against Python's bytes order (the same rule, computed independently)."""
import json
from pathlib import Path

import numpy as np
import pytest

from cubit_amd import filters as F
from oracle import oracle as O

CASES = json.loads((Path(__file__).resolve().parent / "golden" / "string_filter_cases.json").read_text())["cases"]
OPS = {"=": "=", "<>": "!=", "<": "<", "<=": "<=", ">": ">", ">=": ">="}


def filter_of(terms):
    fs = [F.ConstantFilter(OPS[op], lit) for op, lit in terms]
    return fs[0] if len(fs) == 1 else F.ConjunctionAndFilter(fs)


def fixture_queries():
    for case in CASES:
        for q in case["queries"]:
            yield pytest.param(case, q, id=f"{case['table']}-{q['sql']}")


def printed(v):
    return "NULL" if v is None else v


@pytest.mark.parametrize("case,q", list(fixture_queries()))
def test_reference_string_filter_case(case, q):
    rows = case["rows"]
    # every column as strings (the integer id column of strtest is only projected)
    cols = [O.StringColumn([r[j] for r in rows]) for j in range(len(case["columns"]))]
    fs = F.TableFilterSet({q["column"]: filter_of(q["terms"])})
    got = O.table_scan(cols, F.serialize(fs), len(rows))
    proj = q["project"] if q["project"] is not None else q["column"]
    assert [printed(rows[r][proj]) for r in got] == q["rows"], q["sql"]


def random_strings(rng, n, pool=60):
    """Short strings over a small alphabet with high bytes, NUL, empty strings and prefix chains."""
    alphabet = [0x61, 0x62, 0x7A, 0x00, 0x7F, 0x80, 0xFF, 0x41]  # a b z NUL DEL 0x80 0xff A
    base = [b""] + [bytes(rng.choice(alphabet, rng.integers(1, 14)).tolist()) for _ in range(pool)]
    base += [base[3] + b"a", base[3] + b"\x00", base[3][:1], b"a" * 13, b"a" * 12]
    return [base[i] for i in rng.integers(0, len(base), n)], base


def test_order_matches_python_bytes():
    rng = np.random.default_rng(3)
    vals, pool = random_strings(rng, 2000)
    vals = [None if i % 17 == 0 else v for i, v in enumerate(vals)]
    col = O.StringColumn(vals)
    for c in pool[:25] + [b"zzz", b"", b"\xff\xff"]:
        for op, pred in [("=", lambda v: v == c), ("!=", lambda v: v != c), ("<", lambda v: v < c),
                         ("<=", lambda v: v <= c), (">", lambda v: v > c), (">=", lambda v: v >= c)]:
            fs = F.TableFilterSet({0: F.ConstantFilter(op, c)})
            got = O.table_scan([col], F.serialize(fs), len(vals)).tolist()
            want = [i for i, v in enumerate(vals) if v is not None and pred(v)]
            assert got == want, (op, c)


def test_fetch_returns_strings_with_updates():
    rng = np.random.default_rng(4)
    vals, pool = random_strings(rng, 500)
    rows = np.array([3, 10, 10, 77], dtype=np.int64)
    new = [b"new", None, b"newer", b""]
    ver = np.array([5, 5, 7, 5], dtype=np.uint64)
    col = O.StringColumn(vals, updates=(rows, new, ver))
    tx = O.Mvcc(6, 1 << 62)
    ids = np.array([3, 10, 77, 4], dtype=np.int64)
    got, ok = O.fetch(col, ids, tx=tx, with_valid=True)
    assert col.decode(got, ok) == [b"new", None, b"", vals[4]]
    fs = F.TableFilterSet({0: F.ConstantFilter("=", b"new")})
    assert 3 in O.table_scan([col], F.serialize(fs), 500, tx=tx).tolist()


def test_ubigint_compares_unsigned():
    """FilterSelectionSwitch<uint64_t> on the oracle: values past 2^63 are the largest (numpy's
    unsigned order), NULL rows never pass."""
    rng = np.random.default_rng(5)
    edges = np.array([0, 1, 2 ** 63 - 1, 2 ** 63, 2 ** 64 - 1], dtype=np.uint64)
    v = np.concatenate([edges, rng.integers(0, 2 ** 64 - 1, 3000, dtype=np.uint64, endpoint=True)])
    valid = rng.random(len(v)) > 0.1
    from cubit_amd.datagen import validity_from_mask

    col = O.Column(v, validity_from_mask(valid))
    for c in [int(x) for x in edges] + [int(v[9])]:
        for op, f in [("=", np.equal), ("!=", np.not_equal), ("<", np.less), ("<=", np.less_equal),
                      (">", np.greater), (">=", np.greater_equal)]:
            fs = F.TableFilterSet({0: F.ConstantFilter(op, c)})
            want = np.flatnonzero(f(v, np.uint64(c)) & valid)
            assert np.array_equal(O.table_scan([col], F.serialize(fs), len(v)), want), (op, c)
