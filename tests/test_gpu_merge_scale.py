"""The update merge's checkpoint fast path at scale (cubit_table_merge_updates with every record
below the horizon and one record per row: the list is merged from its device copy,
cubit_capi.hip `const bool all`), the shape of round 5's r05u2 fault (612 M rows, 6.12 M
records, a 50-key range index, merge_words_kernel) and a multi-stride shape checked leaf by leaf.

Reference semantics: a checkpoint folds each row's committed update into the base
(UpdateSegment, update_segment.cpp:1074-1199; the visible value is the newest record,
update_info.hpp:44-55); every index leaf must then equal its predicate over the merged column.
"""
import ctypes as C

import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from cubit_amd.table import Context, CubitTable
from test_gpu_maintenance import check_index_bits

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def unique_rows(rng, n, m):
    """About m distinct sorted rows of [0, n) (np.unique of m·1.01 draws, cut to m)."""
    r = np.unique(rng.integers(0, n, int(m * 1.01) + 16))
    return r[:m].astype(np.int64)


def k0_count(ctx, t, col, cmp, c):
    """Rows of the column matching `cmp c`, by K0 over its current device values (an
    independent kernel: compare → bitvector → count)."""
    dptr, typ = t.column_data(col)
    n = t.n_rows
    words = ctx.alloc(L.gpu_lib().cubit_padded_words(n) * 8)
    cnt = ctx.alloc(16)
    try:
        leaf = (C.c_void_p * 1)(words.addr)
        prog = (C.c_int32 * 1)(0)
        L.check(ctx.lib.cubit_build_bitvector(ctx.handle, C.c_void_p(dptr), typ, None, n, cmp, c,
                                              C.c_void_p(words.addr)))
        L.check(ctx.lib.cubit_bitvector_eval(ctx.handle, leaf, 1, 0, prog, 1, n, 0, None, 0, C.c_void_p(cnt.addr),
                                             None, L.SCAN_COUNT_ONLY))
        ctx.check()
        return int(cnt.download(np.uint64, 1)[0])
    finally:
        words.free()
        cnt.free()


def test_merge_all_path_multi_stride_bit_exact(ctx, tmp_path):
    """> 1,048,576 records (more than one grid stride of merge_words_kernel: 4,096 blocks × 4
    waves × 64 records), a ragged row count, new values past the old keys, SET NULL records:
    the merged column and every leaf of a range index and a bins index, bit-exact."""
    rng = np.random.default_rng(61)
    n = 60_000_011
    base = (rng.integers(1, 51, n) * 100).astype(np.int64)
    ok = rng.random(n) > 0.02
    base[~ok] = 0
    t = CubitTable(ctx, n, row_base=7)
    t.add_column(0, base, validity_from_mask(ok))
    t.build_index(0, L.INDEX_RANGE)
    t.build_index(0, L.INDEX_BINS, [0, 1000, 2000, 3000, 4000, 5000])
    rows = unique_rows(rng, n, 1_200_000)
    assert len(rows) > 4096 * 4 * 64
    vals = (rng.integers(0, 53, len(rows)) * 100).astype(np.int64)  # 0 and 5100, 5200: outside the base keys
    valid = rng.random(len(rows)) > 0.1
    t.set_updates(0, rows, vals, np.full(len(rows), 3, dtype=np.uint64), valid)
    merged = t.merge_updates(0, 4)
    assert merged == len(rows)
    want, want_ok = base.copy(), ok.copy()
    want[rows] = np.where(valid, vals, 0)
    want_ok[rows] = valid
    assert np.array_equal(t.download_column(0), want)
    check_index_bits(t, 0, L.INDEX_RANGE, want, want_ok, tmp_path)
    check_index_bits(t, 0, L.INDEX_BINS, want, want_ok, tmp_path)
    # and scans read the merged leaves: a range and an IS NULL against numpy
    got = t.scan(F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", 2500),
                                                              F.ConstantFilter("<", 5150)])}))
    assert np.array_equal(got, np.flatnonzero(want_ok & (want >= 2500) & (want < 5150)) + 7)
    assert np.array_equal(t.scan(F.TableFilterSet({0: F.IsNullFilter()})), np.flatnonzero(~want_ok) + 7)
    t.close()


def test_merge_all_path_at_the_r05u2_shape(ctx):
    """The shape that faulted in round 5 (scripts/merge_timing.py: 612 M rows, 1 % of rows
    updated per rep, a range index over 50 values, two merges back to back): the merged column
    equals numpy's, and every key's leaf counts what K0 counts over the merged column."""
    rng = np.random.default_rng(5)
    n = 612_000_000
    col = (rng.integers(1, 51, n) * 100).astype(np.int64)
    t = CubitTable(ctx, n)
    t.add_column(2, col)
    t.build_index(2, L.INDEX_RANGE)
    for rep in range(2):
        rows = unique_rows(rng, n, n // 100)
        vals = (rng.integers(1, 51, len(rows)) * 100).astype(np.int64)
        t.set_updates(2, rows, vals, np.ones(len(rows), dtype=np.uint64))
        assert t.merge_updates(2, 2) == len(rows)
        col[rows] = vals
    assert np.array_equal(t.download_column(2), col)
    del col
    bad = []
    for k in range(1, 52):
        c = k * 100
        ix = t.count(F.TableFilterSet({2: F.ConstantFilter("<", c)}))
        k0 = k0_count(ctx, t, 2, L.CMP_LT, c)
        if ix != k0:
            bad.append((c, ix, k0))
    assert not bad, bad[:4]
    t.close()
