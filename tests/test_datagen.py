"""Generator plumbing: partitioned generation equals the full table (what the multi-GPU
bench relies on), and the synthetic columns are row-addressable."""
import numpy as np

from cubit_amd import datagen


def test_partitioned_lineitem_equals_full(li01):
    full = li01
    o = datagen.tpch_orders(0.1)
    cut = [0, o // 3, 2 * o // 3, o]
    parts = [datagen.tpch_lineitem(0.1, cut[i], cut[i + 1]) for i in range(3)]
    assert parts[0].row_base == 0
    for p in parts:
        s = slice(p.row_base, p.row_base + p.n_rows)
        assert np.array_equal(p.l_shipdate, full.l_shipdate[s])
        assert np.array_equal(p.l_extendedprice, full.l_extendedprice[s])
    assert sum(p.n_rows for p in parts) == full.n_rows


def test_lineitem_domains(li01):
    assert li01.l_quantity.min() == 100 and li01.l_quantity.max() == 5000
    assert li01.l_discount.min() == 0 and li01.l_discount.max() == 10
    # shipdate range 1992-01-02 .. 1998-12-01
    from cubit_amd.filters import date

    assert li01.l_shipdate.min() >= date(1992, 1, 2) and li01.l_shipdate.max() <= date(1998, 12, 1)


def test_uniform_i32_row_addressable():
    a = datagen.uniform_i32(42, 5000, 1_000_000)
    b = datagen.uniform_i32(42, 1000, 1_000_000, row_begin=2000)
    assert np.array_equal(a[2000:3000], b)
    assert a.min() >= 0 and a.max() < 1_000_000
