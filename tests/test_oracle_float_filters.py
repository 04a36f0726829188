"""FLOAT / DOUBLE table filters on the oracle (FilterSelectionSwitch<float / double>,
src/storage/table/column_segment.cpp:278-349, with DuckDB's floating-point operators,
src/common/vector_operations/comparison_operators.cpp:17-88: NaN equals NaN and is greater
than everything; -0.0 == +0.0), pinned by the reference's nan_test.test and infinity_test.test
(tests/golden/float_filter_cases.json) for both types."""
import json
import math
from collections import Counter
from pathlib import Path

import numpy as np
import pytest

from cubit_amd import filters as F
from oracle import oracle as O

CASES = json.loads((Path(__file__).resolve().parent / "golden" / "float_filter_cases.json").read_text())["cases"]
TYPES = {"FLOAT": np.float32, "DOUBLE": np.float64}
OPS = {"=": "=", "<>": "!=", "<": "<", "<=": "<=", ">": ">", ">=": ">="}


def fval(text, dtype):
    special = {"nan": math.nan, "inf": math.inf, "-inf": -math.inf}
    return dtype(special[text] if text in special else float(text))


def printed(x):
    """A value as the reference's tests print it."""
    if math.isnan(x):
        return "nan"
    if math.isinf(x):
        return "inf" if x > 0 else "-inf"
    return f"{x:g}"


def fixture_queries():
    for case in CASES:
        for tname in case["types"]:
            for q in case["queries"]:
                yield pytest.param(case, tname, q, id=f"{Path(case['file']).stem}-{tname}-f{q['cmp']}{q['constant']}")


def run_oracle(values, dtype, cmp, const):
    col = O.Column(np.array(values, dtype=dtype))
    fs = F.TableFilterSet({0: F.ConstantFilter(cmp, dtype(const))})
    return O.table_scan([col], F.serialize(fs), len(values))


@pytest.mark.parametrize("case,tname,q", list(fixture_queries()))
def test_reference_float_filter_case(case, tname, q):
    dt = TYPES[tname]
    vals = [fval(v, dt) for v in case["inserted"]]
    rows = run_oracle(vals, dt, OPS[q["cmp"]], fval(q["constant"], dt))
    got = Counter(printed(float(vals[r])) for r in rows)
    assert got == Counter(q["rows"]), q["sql"]


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_signed_zero_and_nan_payloads(dt):
    """-0.0 == +0.0 (IEEE ==, EqualsFloat), and every NaN — whatever its sign and payload —
    equals every other NaN and is greater than +inf (GreaterThanFloat)."""
    bits = np.uint32 if dt == np.float32 else np.uint64
    pos_nan = np.array([0x7FC00001 if dt == np.float32 else 0x7FF8000000000001], dtype=bits).view(dt)[0]
    neg_nan = np.array([0xFFC00000 if dt == np.float32 else 0xFFF8000000000000], dtype=bits).view(dt)[0]
    vals = [dt(-0.0), dt(0.0), dt(1.5), dt(-2.5), dt(math.inf), dt(-math.inf), pos_nan, neg_nan]
    n = len(vals)

    def rows(cmp, c):
        return set(run_oracle(vals, dt, cmp, c).tolist())

    assert rows("=", dt(0.0)) == rows("=", dt(-0.0)) == {0, 1}
    assert rows("<", dt(0.0)) == rows("<", dt(-0.0)) == {3, 5}
    assert rows("<=", dt(-0.0)) == {0, 1, 3, 5}
    assert rows(">", dt(-0.0)) == {2, 4, 6, 7}
    assert rows(">=", dt(0.0)) == {0, 1, 2, 4, 6, 7}
    assert rows("!=", dt(0.0)) == {2, 3, 4, 5, 6, 7}
    assert rows("=", pos_nan) == rows("=", neg_nan) == {6, 7}
    assert rows(">", dt(math.inf)) == {6, 7}
    assert rows("<", neg_nan) == set(range(6))
    assert rows("<=", pos_nan) == set(range(n))
    assert rows(">", pos_nan) == set()
    assert rows(">=", neg_nan) == {6, 7}


ORDERING = json.loads((Path(__file__).resolve().parent / "golden" / "float_filter_cases.json").read_text())["ordering"]


def ordering_column(dt):
    """nan_ordering.test's table: the values and the NULL mask."""
    special = {"nan": math.nan, "infinity": math.inf, "inf": math.inf, "-infinity": -math.inf, "-inf": -math.inf}
    vals, valid = [], []
    for v, k in ORDERING["inserted"]:
        vals += [dt(0.0) if v == "null" else dt(special.get(v, v) if v in special else float(v))] * k
        valid += [v != "null"] * k
    return np.array(vals, dtype=dt), np.array(valid)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_nan_ordering_counts_and_order(dt):
    """nan_ordering.test: COUNT(*) WHERE f > 0 = 4 and WHERE f < 0 = 3 over its 10,008 rows (two
    NaNs, ±inf, NULL), on the oracle; and the total order its ORDER BY prints (-inf < -1 < 1 < inf <
    nan, NULL first) is the order of the C ABI's comparison keys (cubit_fp_key, restated here as
    numpy: every NaN → one key above +inf, -x → -pattern(x))."""
    from cubit_amd.datagen import validity_from_mask

    vals, valid = ordering_column(dt)
    col = O.Column(vals, validity_from_mask(valid))
    for c in ORDERING["counts"]:
        fs = F.TableFilterSet({0: F.ConstantFilter(OPS[c["cmp"]], dt(float(c["constant"])))})
        assert len(O.table_scan([col], F.serialize(fs), len(vals))) == c["count"], c["sql"]
    first6 = vals[:6][valid[:6]]
    bits = O.fp_bits(first6, dt).astype(np.uint64) if dt == np.float32 else O.fp_bits(first6, dt).view(np.uint64)
    width = 32 if dt == np.float32 else 64
    sign = bits >> np.uint64(width - 1)
    mag = bits & np.uint64((1 << (width - 1)) - 1)
    nan = mag > np.uint64(0x7F800000 if dt == np.float32 else 0x7FF0000000000000)
    nan_key = 0x7FC00000 if dt == np.float32 else 0x7FF8000000000000
    key = np.where(nan, nan_key, np.where(sign == 1, -mag.astype(np.int64), mag.astype(np.int64)))
    order = ["NULL"] + [printed(float(x)) for x in first6[np.argsort(key, kind="stable")]]
    want = [x if x in ("NULL", "nan", "inf", "-inf") else f"{float(x):g}" for x in ORDERING["order_by_f"]]
    assert order == want
