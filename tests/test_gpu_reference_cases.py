"""The reference's own SQL test cases (tests/golden/reference_cases.json, each citing its
.test file) through the C ABI on the GPU, with and without bitmap indexes."""
import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.table import Context, CubitTable
from test_oracle_tpch import residual_from_json

pytestmark = pytest.mark.gpu

TXN_START = 4611686018427388000


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_zonemap_segment(ctx, golden, encoding):
    c = golden["cases"]["zonemap_segment"]
    data = np.repeat(np.array(c["values"], dtype=np.int32), c["block_rows"])
    t = CubitTable(ctx, len(data))
    t.add_column(0, data)
    if encoding is not None:
        t.build_index(0, encoding)
    for k, want in c["expected_sum_eq"].items():
        rows = t.scan(F.TableFilterSet({0: F.ConstantFilter("=", int(k))}))
        got = int(data[rows].astype(np.int64).sum()) if len(rows) else None
        assert got == want, k


def test_interleaved_versions(ctx, golden):
    data = np.array([1, 2], dtype=np.int32)
    t1, t2 = TXN_START + 10, TXN_START + 11
    t = CubitTable(ctx, 2)
    t.add_column(0, data)
    exp = golden["cases"]["interleaved_versions"]["steps"]

    def s(start, tid):
        r = t.scan(F.TableFilterSet(), txn=L.Txn(start, tid))
        return int(data[r].sum()) if len(r) else None

    t.set_deletes(np.array([0, 1]), np.array([t1, t2], dtype=np.uint64))
    assert s(5, t1) == exp[0]["expect"]["con1"]
    assert s(5, t2) == exp[0]["expect"]["con2"]
    assert s(5, TXN_START + 12) == exp[0]["expect"]["con3"]
    t.set_deletes(np.array([0, 1]), np.array([6, t2], dtype=np.uint64))  # con1 committed at 6
    assert s(5, t2) == exp[1]["expect"]["con2"]
    assert s(7, TXN_START + 13) == 2


@pytest.mark.parametrize("index", [False, True])
def test_table_or_pushdown(ctx, golden, index):
    c = golden["cases"]["table_or_pushdown"]
    data = np.array(c["rows"], dtype=np.int32)
    t = CubitTable(ctx, len(data))
    t.add_column(0, data)
    t.add_column(1, data.copy())
    if index:
        t.build_index(0, L.INDEX_RANGE)
        t.build_index(1, L.INDEX_EQUALITY)
    for q in c["queries"]:
        rows = t.scan(None, residual_from_json(q["tree"]))
        assert data[rows].tolist() == q["expect"], q["sql"]
