"""test/sql/filter/test_transitive_filters.test on the oracle: the 40 one-table queries
`WHERE <i cmp constant> AND <j cmp i>` — the constant comparison pushed into the scan (the oracle's
TemplatedScan restatement), the column-to-column comparison DuckDB keeps in a filter above it
applied to the scan's rows — each query's rows in the file's order."""
import numpy as np

from cubit_amd import filters as F
from oracle import oracle as O


_OPS = {"=": lambda a, b: a == b, "<": lambda a, b: a < b, "<=": lambda a, b: a <= b, ">": lambda a, b: a > b,
        ">=": lambda a, b: a >= b}


def transitive_filter_cases(golden):
    """test/sql/filter/test_transitive_filters.test: (vals1 columns, [(TableFilterSet pushed on i,
    residual comparison of j with i, expected rows)])."""
    c = golden["cases"]["transitive_filters"]
    rows = np.array(c["rows"], dtype=np.int64)
    out = []
    for q in c["queries"]:
        op, k = q["constant"]
        out.append((F.TableFilterSet({0: F.ConstantFilter(op, k)}), _OPS[q["residual"]], q["rows"], q["where"]))
    return rows[:, 0].copy(), rows[:, 1].copy(), out


def test_transitive_filters_reference_case(golden):
    """The scan with the pushed constant comparison on i (oracle), then the column-to-column
    comparison DuckDB keeps above the scan: every one of the 40 queries' rows, in row order."""
    i, j, cases = transitive_filter_cases(golden)
    cols = [O.Column(i), O.Column(j)]
    for fs, residual, want, where in cases:
        rows = O.table_scan(cols, F.serialize(fs), len(i))
        got = [[int(i[r]), int(j[r])] for r in rows if residual(j[r], i[r])]
        assert got == want, where
