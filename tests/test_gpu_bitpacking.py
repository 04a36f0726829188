"""K5 on the GPU: DuckDB BITPACKING segments (built by the oracle's restatement of the
reference compressor) uploaded through cubit_table_add_bitpacked_column and unpacked by
the HIP kernel must give back every valid value bit-exactly (read through the probe), and
the unpacked column must index and scan like a plain one."""
import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from cubit_amd.table import Context, CubitTable
from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def probe_all(ctx, t, col, n, row_base=0):
    ids = ctx.upload(np.arange(n, dtype=np.int64) + row_base)
    cnt = ctx.upload(np.array([n], dtype=np.uint64))
    out = ctx.alloc(n * 8)
    t.probe(col, ids.addr, cnt.addr, n, out.addr)
    return out.download(np.int64, n)


CASES = {
    "constant": lambda rng, n: np.full(n, -7, np.int32),
    "ap64": lambda rng, n: (np.arange(n, dtype=np.int64) * -3 + 10 ** 15),
    "sorted32": lambda rng, n: np.cumsum(rng.integers(0, 9, n)).astype(np.int32),
    "rand32": lambda rng, n: rng.integers(-1000, 1000, n).astype(np.int32),
    "rand64": lambda rng, n: rng.integers(-2 ** 40, 2 ** 40, n).astype(np.int64),
    "wide64": lambda rng, n: rng.integers(-2 ** 62, 2 ** 62, n).astype(np.int64),
    "dates": lambda rng, n: (8035 + rng.integers(0, 2526, n)).astype(np.int32),
}


@pytest.mark.parametrize("mode", ["auto", "for", "delta_for", "constant_delta"])
@pytest.mark.parametrize("name", sorted(CASES))
def test_unpack_matches_values(ctx, name, mode):
    rng = np.random.default_rng(abs(hash((name, mode))) % 2 ** 32)
    n = 200_003  # 98 groups, a partial last group, several segments for the wide cases
    v = CASES[name](rng, n)
    c = O.bp_compress(v, None, mode)
    assert c is not None
    t = CubitTable(ctx, n, row_base=5)
    t.add_bitpacked_column(0, c.data, c.seg_off, c.seg_count, v.dtype)
    got = probe_all(ctx, t, 0, n, row_base=5)
    assert np.array_equal(got, v.astype(np.int64)), (name, mode, sorted(set(O.bp_group_modes(c))))
    assert np.array_equal(t.download_column(0), v)


def test_nulls_index_and_scan(ctx):
    rng = np.random.default_rng(8)
    n = 300_007
    v = rng.integers(0, 60, n).astype(np.int32)
    valid = rng.random(n) > 0.2
    valid[4096:6144] = False  # an all-NULL group (CONSTANT)
    c = O.bp_compress(v, valid, "auto")
    vw = validity_from_mask(valid)
    t = CubitTable(ctx, n)
    t.add_bitpacked_column(0, c.data, c.seg_off, c.seg_count, np.int32, validity=vw)
    got = probe_all(ctx, t, 0, n)
    assert np.array_equal(got[valid], v[valid].astype(np.int64))
    t.build_index(0, L.INDEX_RANGE)
    col = O.Column(v, vw)
    for f in (F.ConstantFilter("<", 10), F.ConstantFilter(">=", 30), F.IsNullFilter(),
              F.ConjunctionAndFilter([F.ConstantFilter(">", 5), F.ConstantFilter("<=", 25)])):
        fs = F.TableFilterSet({0: f})
        assert np.array_equal(t.scan(fs), O.table_scan([col], F.serialize(fs), n)), f


def test_malformed_segments_are_refused(ctx):
    v = np.arange(10_000, dtype=np.int64) * 7
    c = O.bp_compress(v, None, "for")
    t = CubitTable(ctx, len(v))
    with pytest.raises(Exception, match="rows"):
        t.add_bitpacked_column(0, c.data, c.seg_off, c.seg_count - 1, np.int64)  # row count mismatch
    bad = c.data.copy()
    bad[:8] = np.frombuffer(np.uint64(len(bad) * 4).tobytes(), np.uint8)  # metadata past the end
    with pytest.raises(Exception, match="metadata"):
        t.add_bitpacked_column(0, bad, c.seg_off, c.seg_count, np.int64)
    with pytest.raises(Exception, match="metadata|truncated|out of bounds"):
        t.add_bitpacked_column(0, c.data[: len(c.data) // 2], c.seg_off, c.seg_count, np.int64)


@pytest.mark.parametrize("name", ["l_shipdate", "l_discount", "l_quantity", "l_extendedprice"])
def test_bench_packer_lineitem(ctx, name):
    """bench.py's K5 leg input (CONSTANT/FOR segments from libcubit_datagen) at SF1: the GPU
    unpack equals the column and the oracle's decode of the same bytes."""
    from cubit_amd import datagen

    li = datagen.tpch_lineitem(1.0, columns=(name,))
    v = getattr(li, name)
    b = datagen.bitpack_for(v)
    t = CubitTable(ctx, len(v))
    t.add_bitpacked_column(0, b.data, b.seg_off, b.seg_count, v.dtype)
    got = t.download_column(0)
    assert np.array_equal(got, v)
    col = O.BitpackedColumn(b.data, b.seg_off, None, b.seg_count, v.dtype)
    assert np.array_equal(O.bp_decode(col), got)
    t.close()


@pytest.mark.parametrize("mode", ["auto", "for", "delta_for", "constant_delta"])
@pytest.mark.parametrize("name", ["rand32", "rand64", "sorted32", "dates", "wide64", "constant"])
def test_filter_straight_from_segments(ctx, name, mode):
    """Constant comparisons on an unindexed bitpacked column run unpack + compare in one pass
    over the segments (bitpacked_compare_kernel): the rows must equal the plain-column K0's and
    the oracle's, for every comparison, with NULLs, and with small segments whose row counts
    leave groups off the 64-row word boundaries (words shared by two groups)."""
    rng = np.random.default_rng(abs(hash((name, mode, "f"))) % 2 ** 32)
    n = 300_017
    v = CASES[name](rng, n)
    valid = rng.random(n) > 0.1
    # segments cut at ragged rows (100,003 and 170,001): groups that start and end off the 64-row
    # word boundaries (the compressor's own segments always end on whole groups)
    parts, offs, counts, pos = [], [], [], 0
    for a, b in ((0, 100_003), (100_003, 170_001), (170_001, n)):
        c = O.bp_compress(v[a:b], valid[a:b], mode, block_size=65536)
        assert c is not None
        data = np.concatenate([c.data, np.zeros((-len(c.data)) % 8, np.uint8)])
        parts.append(data)
        offs.append(c.seg_off + pos)
        counts.append(c.seg_count)
        pos += len(data)
    vw = validity_from_mask(valid)
    t = CubitTable(ctx, n, row_base=11)
    t.add_bitpacked_column(0, np.concatenate(parts), np.concatenate(offs).astype(np.uint64),
                           np.concatenate(counts).astype(np.uint64), v.dtype, validity=vw)
    other = rng.integers(0, 4, n).astype(np.int64)
    t.add_column(1, other)
    t.build_index(1, L.INDEX_RANGE)
    cols = [O.Column(v, vw), O.Column(other)]
    picks = rng.choice(v[valid], size=6) if valid.any() else np.zeros(6, v.dtype)
    consts = [int(x) for x in picks] + [int(v.min()) - 1, int(v.max()) + 1]
    for i, k in enumerate(consts):
        cmp = ["=", "!=", "<", "<=", ">", ">="][i % 6]
        for fs in (F.TableFilterSet({0: F.ConstantFilter(cmp, k)}),
                   F.TableFilterSet({0: F.ConstantFilter(cmp, k), 1: F.ConstantFilter("<", 2)})):
            ref = O.table_scan(cols, F.serialize(fs), n, row_base=11)
            t.use_packed_filter(True)
            got = t.scan(fs)
            packed = t.last_packed()
            live = t.last_zones()[0]
            t.use_packed_filter(False)
            plain = t.scan(fs)
            assert np.array_equal(got, ref), (name, mode, cmp, k)
            assert np.array_equal(plain, ref), (name, mode, cmp, k)
            # the leaf came from the segments (unless the zonemaps ruled every zone out: then
            # no leaf is built at all)
            assert packed == (1 if live else 0), (name, mode, cmp, k, packed, live)
    t.use_packed_filter(True)
    t.close()


@pytest.mark.parametrize("mode", ["auto", "for", "delta_for", "constant_delta"])
def test_fused_sum_reads_packed_column(ctx, mode):
    """SELECT sum(a * b) WHERE <filter> with a read at the qualifying rows straight from its
    BITPACKING segments (the default for such a column: group record → the value's w bits;
    DELTA_FOR rows from the unpacked column): equal to the same sum over the plain column
    (CUBIT_SUM_PLAIN_A) and to numpy,
    for every group mode, with NULLs in a, several segments and a row base."""
    rng = np.random.default_rng({"auto": 1, "for": 2, "delta_for": 3, "constant_delta": 4}[mode])
    n = 600_011
    a = rng.integers(-2 ** 23, 2 ** 23, n).astype(np.int64)
    if mode == "constant_delta":
        a = (np.arange(n, dtype=np.int64) * 3 - 5)
    elif mode == "delta_for":
        a = np.cumsum(rng.integers(0, 100, n)).astype(np.int64)
    a[100_000:104_096] = 42  # a constant group or two
    b = rng.integers(0, 11, n).astype(np.int64)
    key = rng.integers(0, 100, n).astype(np.int32)
    valid_a = np.ones(n, dtype=bool)  # NULLs in a few groups (the delta modes need all-valid groups)
    valid_a[200_000:220_000] = rng.random(20_000) > 0.3
    c = O.bp_compress(a, valid_a, mode)
    modes = set(O.bp_group_modes(c))
    assert {"auto": "for", "for": "for", "delta_for": "delta_for", "constant_delta": "constant_delta"}[mode] in modes
    t = CubitTable(ctx, n, row_base=11)
    t.add_bitpacked_column(0, c.data, c.seg_off, c.seg_count, np.int64, validity=validity_from_mask(valid_a))
    t.add_column(1, b)
    t.add_column(2, key)
    t.build_index(2, L.INDEX_RANGE)
    for f in (F.ConstantFilter("<", 3), F.ConstantFilter(">=", 60), F.ConstantFilter("=", 50)):
        fs = F.TableFilterSet({2: f})
        keep = {"<": key < 3, ">=": key >= 60, "=": key == 50}[f.comparison] & valid_a
        want = int((a[keep].astype(object) * b[keep].astype(object)).sum())
        s_plain, n_plain = t.sum_product(0, 1, fs, gather_b=True, packed_a=False)
        assert not t.last_sum_packed()
        s_packed, n_packed = t.sum_product(0, 1, fs, gather_b=True)
        assert t.last_sum_packed()
        assert s_plain == want and s_packed == want, (mode, f.comparison)
        assert n_plain == n_packed
    t.close()


# ---------------------------------------------------------------- segments DuckDB itself wrote

from test_oracle_bitpacking import REF_SEGMENTS, reference_segment  # noqa: E402


@pytest.mark.parametrize("s", REF_SEGMENTS, ids=[s["name"] for s in REF_SEGMENTS])
def test_gpu_reads_duckdb_written_segment(ctx, s):
    """BITPACKING bytes exactly as DuckDB v1.1.2 stored them (tests/golden/
    bitpacking_reference_segments.json: FOR, DELTA_FOR and CONSTANT_DELTA groups, INT32 and
    INT64, NULL rows, a 49-group segment with a partial last group) through K5: the unpacked
    column, the packed-segment filter and the fused sum that reads the column at the
    qualifying rows from the segments must give the reference's values."""
    col, values, valid = reference_segment(s)
    n = s["count"]
    t = CubitTable(ctx, n, row_base=3)
    vw = validity_from_mask(valid)
    t.add_bitpacked_column(0, col.data, col.seg_off, col.seg_count, values.dtype, validity=vw)
    got = t.download_column(0)
    assert np.array_equal(got[valid], values[valid])
    assert np.array_equal(got, O.bp_decode(col))  # NULL slots: the stored filler, as the oracle reads it
    oc = O.Column(values.astype(np.int64) if values.dtype.kind == "u" else values, vw)  # UBIGINT offsets < 2^63
    lo, hi = int(values[valid].min()), int(values[valid].max())
    mid = int(np.median(values[valid]))
    for cmp, k in (("=", mid), ("!=", mid), ("<", mid), (">=", mid), ("<=", lo), (">", hi - 1), ("<", lo)):
        fs = F.TableFilterSet({0: F.ConstantFilter(cmp, k)})
        ref = O.table_scan([oc], F.serialize(fs), n, row_base=3)
        t.use_packed_filter(True)
        assert np.array_equal(t.scan(fs), ref), (s["name"], cmp, k)
        t.use_packed_filter(False)
        assert np.array_equal(t.scan(fs), ref), (s["name"], cmp, k)
    if values.dtype == np.int64:
        # SELECT sum(v * 1) WHERE v < mid, v read from the segments at the qualifying rows
        t.add_column(1, np.ones(n, dtype=np.int64))
        keep = valid & (values < mid)
        fs = F.TableFilterSet({0: F.ConstantFilter("<", mid)})
        total, cnt = t.sum_product(0, 1, fs, gather_b=True)
        assert t.last_sum_packed()
        assert total == int(values[keep].sum()) and cnt == int(keep.sum())
    t.close()


# ---------------------------------------------------------------- the FTS index's segments

from test_oracle_bitpacking import FTS, FTS_BP, check_fts_invariants, fts_decoded, fts_segment  # noqa: E402


def test_gpu_reads_the_fts_index_segments(ctx):
    """The BITPACKING segments of the reference's huggingface_index.db FTS index (FOR groups of
    7, 8 and 11 bits, CONSTANT_DELTA; tests/golden/bitpacking_reference_segments_fts.json)
    through K5: each unpacked column equals the restatement's decode, the unpacked columns
    satisfy the FTS definitions (docs.len = terms per doc, dict.df = distinct docs per term,
    every termid present, Σ len / 153 = avgdl), and comparisons through the packed-segment filter
    equal the oracle's scan."""
    cols = fts_decoded()
    for s in FTS_BP:
        col = fts_segment(s)
        n = s["count"]
        t = CubitTable(ctx, n, row_base=0)
        t.add_bitpacked_column(0, col.data, col.seg_off, col.seg_count, np.int64)
        got = t.download_column(0)
        assert np.array_equal(got, cols[s["name"]]), s["name"]
        cols[s["name"]] = got
        oc = O.Column(got)
        mid = int(np.median(got))
        for cmp, k in (("<", mid), (">=", mid), ("=", mid), ("<", int(got.min()) + 1)):
            fs = F.TableFilterSet({0: F.ConstantFilter(cmp, k)})
            ref = O.table_scan([oc], F.serialize(fs), n)
            t.use_packed_filter(True)
            assert np.array_equal(t.scan(fs), ref), (s["name"], cmp, k)
            t.use_packed_filter(False)
        t.close()
    check_fts_invariants(cols)
    assert FTS["stats_avgdl"] > 0


# ---------------------------------------------------------------- every integral type

from test_oracle_bitpacking import (FORCED, INT_DTYPES, bitwidth_tables, filter_pushdown_column,  # noqa: E402
                                    typed_case)


def packed_table(ctx, c, dtype, n, valid=None, row_base=0):
    t = CubitTable(ctx, n, row_base=row_base)
    vw = None if valid is None else validity_from_mask(valid)
    t.add_bitpacked_column(0, c.data, c.seg_off, c.seg_count, dtype, validity=vw)
    return t, vw


@pytest.mark.parametrize("mode", ["auto"] + FORCED)
@pytest.mark.parametrize("dtype", INT_DTYPES)
def test_every_type_unpacks_and_filters(ctx, dtype, mode):
    """Segments of every integral T (INT8 … UBIGINT; header fields of T's size, packed runs off
    the 4-byte alignment for 1- and 2-byte T, T's wrap-around arithmetic in descending
    DELTA_FOR / CONSTANT_DELTA groups) unpack into the INT32 / INT64 column to the oracle's
    values, and the filter straight from the segments equals the oracle's scan of them, for
    every comparison. UBIGINT keeps its 64 bits over the whole range (values past 2^63
    included) and compares them unsigned, as the oracle's FilterSelectionSwitch<uint64_t>."""
    ubig = np.dtype(dtype) == np.uint64
    v, valid, c = typed_case(dtype, mode)
    n = len(v)
    t, vw = packed_table(ctx, c, dtype, n, valid, row_base=7)
    got = t.download_column(0)
    assert got.dtype == (np.int32 if np.dtype(dtype).itemsize <= 2 or dtype is np.int32 else
                         np.uint64 if ubig else np.int64)
    assert np.array_equal(got[valid], v[valid].astype(got.dtype)), (np.dtype(dtype).name, mode)
    wide = v if ubig else v.astype(np.int64)
    oc = O.Column(wide, vw)
    rng = np.random.default_rng(11)
    picks = [int(x) for x in rng.choice(wide[valid], 4)] + [int(wide[valid].min()), int(wide[valid].max())]
    for i, k in enumerate(picks):
        cmp = ["=", "!=", "<", "<=", ">", ">="][i % 6]
        fs = F.TableFilterSet({0: F.ConstantFilter(cmp, k)})
        ref = O.table_scan([oc], F.serialize(fs), n, row_base=7)
        t.use_packed_filter(True)
        assert np.array_equal(t.scan(fs), ref), (np.dtype(dtype).name, mode, cmp, k)
        assert t.last_packed() in (0, 1)
        t.use_packed_filter(False)
        assert np.array_equal(t.scan(fs), ref), (np.dtype(dtype).name, mode, cmp, k)
    t.close()


@pytest.mark.parametrize("mode", FORCED)
@pytest.mark.parametrize("bits", [8, 16, 32, 64])
def test_bitwidths_reference_case_on_gpu(ctx, bits, mode):
    """bitpacking_bitwidths.test_slow through K5: each table's unpacked column has the
    reference's distinct-value counts (bits or bits - 1 values, 2,048 rows each), and an
    equality scan (straight from the segments where the type allows) finds each value's 2,048
    rows — UBIGINT's 2^63 included, read back and compared unsigned."""
    for name, v in bitwidth_tables(bits).items():
        c = O.bp_compress(v, None, mode)
        t = CubitTable(ctx, len(v))
        t.add_bitpacked_column(0, c.data, c.seg_off, c.seg_count, v.dtype)
        got = t.download_column(0)
        assert np.array_equal(got, v.astype(got.dtype)), (name, mode)
        vals, counts = np.unique(got, return_counts=True)
        assert len(vals) == (bits - 1 if name == "test_signed_pos" else bits) and set(counts.tolist()) == {2048}
        t.use_packed_filter(True)
        for k in (int(vals[0]), int(vals[-1])):
            rows = t.scan(F.TableFilterSet({0: F.ConstantFilter("=", k)}))
            assert len(rows) == 2048 and np.all(got[rows] == k), (name, mode, k)
        t.close()


@pytest.mark.parametrize("mode", FORCED)
@pytest.mark.parametrize("dtype", INT_DTYPES + [np.bool_])
def test_nullpack_reference_case_on_gpu(ctx, dtype, mode):
    """bitpacking_bitwidths.test_slow:101-117 through K5: AVG of the unpacked column = 0.5."""
    dt = np.int8 if dtype is np.bool_ else dtype
    v = ((np.arange(12000) // 3000) % 2).astype(dt)
    c = O.bp_compress(v, None, mode)
    t = CubitTable(ctx, len(v))
    t.add_bitpacked_column(0, c.data, c.seg_off, c.seg_count, dt)
    assert t.download_column(0).mean() == 0.5
    t.close()


@pytest.mark.parametrize("mode", FORCED)
def test_nulls_reference_case_on_gpu(ctx, mode):
    """bitpacking_nulls.test through K5: sum 70,694,000, min 0, max 9,999 over the valid rows —
    the sum from the fused sum-product reading the column straight from its segments."""
    i = np.arange(10000, dtype=np.int64)
    v = np.concatenate([np.full(10000, 1337, np.int64), i, i // 2])
    valid = np.tile(i % 5 != 0, 3)
    c = O.bp_compress(v, valid.astype(np.uint8), mode)
    n = len(v)
    t, _ = packed_table(ctx, c, np.int64, n, valid)
    got = t.download_column(0)[valid]
    assert (int(got.min()), int(got.max())) == (0, 9999)
    t.add_column(1, np.ones(n, np.int64))
    t.add_column(2, np.zeros(n, np.int32))
    t.build_index(2, L.INDEX_RANGE)
    total, cnt = t.sum_product(0, 1, F.TableFilterSet({2: F.ConstantFilter("=", 0)}), gather_b=True)
    assert (total, cnt) == (70694000, n)  # cnt: the rows the filter passes (NULL a adds nothing)
    t.close()


def test_delta_full_range_reference_case_on_gpu(ctx):
    """bitpacking_delta.test_slow's UBIGINT column (0 and 2^64 - 1 alternating) through K5: read
    back bit-exact, and the unsigned comparisons split it as the reference's SUM / COUNT see it —
    2^64 - 1 is the greatest value, not -1."""
    v = np.where(np.arange(100_000) % 2 == 0, np.uint64(0), np.uint64(2 ** 64 - 1)).astype(np.uint64)
    c = O.bp_compress(v, None, "for")
    t = CubitTable(ctx, len(v))
    t.add_bitpacked_column(0, c.data, c.seg_off, c.seg_count, np.uint64)
    assert np.array_equal(t.download_column(0), v)
    for cmp, k, want in ((">", 0, 50_000), ("=", 2 ** 64 - 1, 50_000), ("<", 2 ** 63, 50_000), (">=", 0, 100_000),
                         ("<=", 2 ** 64 - 2, 50_000)):
        rows = t.scan(F.TableFilterSet({0: F.ConstantFilter(cmp, k)}))
        assert len(rows) == want, (cmp, k)
        assert np.array_equal(rows, O.table_scan([O.Column(v)], F.serialize(F.TableFilterSet(
            {0: F.ConstantFilter(cmp, k)})), len(v)))
    lo, hi, _, _ = t.column_statistics(0)
    assert (lo & (2 ** 64 - 1), hi & (2 ** 64 - 1)) == (0, 2 ** 64 - 1)
    t.close()


@pytest.mark.parametrize("mode", ["auto"] + FORCED)
def test_filter_pushdown_reference_case_on_gpu(ctx, mode):
    """bitpacking_filter_pushdown.test through K5: WHERE col = 1337 straight from the segments →
    SUM 13371337, MIN = MAX = 1337, COUNT 10001 (col read back by the probe); WHERE id = 5000 on
    the other column → col 5000."""
    col, ids = filter_pushdown_column()
    c = O.bp_compress(col, None, mode)
    n = len(col)
    t, _ = packed_table(ctx, c, np.int32, n)
    t.add_column(1, ids)
    t.use_packed_filter(True)
    rows = t.scan(F.TableFilterSet({0: F.ConstantFilter("=", 1337)}))
    vals = probe_all(ctx, t, 0, n)[rows]
    assert (int(vals.sum()), int(vals.min()), int(vals.max()), len(vals)) == (13371337, 1337, 1337, 10001)
    rows = t.scan(F.TableFilterSet({1: F.ConstantFilter("=", 5000)}))
    assert probe_all(ctx, t, 0, n)[rows].tolist() == [5000]
    t.close()


@pytest.mark.parametrize("dtype", INT_DTYPES + [np.bool_])
def test_plain_columns_of_every_type(ctx, dtype):
    """cubit_table_add_column with a narrower or unsigned type code (TINYINT … UBIGINT vectors
    as DuckDB holds them) widens the values on the device into an INT32 / INT64 column; index
    scans, unindexed comparisons and the probe then equal numpy on the widened values. UBIGINT
    keeps its 64 bits over the whole range and compares them unsigned (the probe hands the bits
    back as int64)."""
    rng = np.random.default_rng(abs(hash(np.dtype(dtype).name)) % 2 ** 32)
    n = 300_007
    ubig = np.dtype(dtype) == np.uint64
    if dtype is np.bool_:
        v = rng.random(n) < 0.3
    else:
        info = np.iinfo(dtype)
        v = rng.integers(info.min, info.max, n, dtype=dtype, endpoint=True)
        v[:1000] = info.min
    wide = v if ubig else v.astype(np.int64)  # UBIGINT: numpy's unsigned order is the reference's
    valid = rng.random(n) > 0.1
    t = CubitTable(ctx, n, row_base=9)
    t.add_column(0, v, validity=validity_from_mask(valid))
    got = t.download_column(0)
    assert got.dtype == (np.int32 if np.dtype(dtype).itemsize <= 2 or dtype is np.int32 else
                         np.uint64 if ubig else np.int64)
    assert np.array_equal(got[valid], wide[valid])
    probed = probe_all(ctx, t, 0, n, row_base=9)
    assert np.array_equal((probed.view(np.uint64) if ubig else probed)[valid], wide[valid])
    k = int(np.median(wide[valid]))
    for cmp, mask in (("<", wide < k), (">=", wide >= k), ("=", wide == int(wide[valid][0]))):
        kk = int(wide[valid][0]) if cmp == "=" else k
        fs = F.TableFilterSet({0: F.ConstantFilter(cmp, kk)})
        ref = np.flatnonzero(mask & valid).astype(np.int64) + 9
        assert np.array_equal(t.scan(fs), ref), (np.dtype(dtype).name, cmp)
    if np.dtype(dtype).itemsize <= 2:
        t.build_index(0, L.INDEX_EQUALITY)
        fs = F.TableFilterSet({0: F.ConstantFilter("=", int(wide[valid][1]))})
        ref = np.flatnonzero((wide == int(wide[valid][1])) & valid).astype(np.int64) + 9
        assert np.array_equal(t.scan(fs), ref)
    if ubig:  # a range index with keys across 2^63: leaves, the candidate check and the statistics
        keys = [2 ** 62, 2 ** 63 - 1, 2 ** 63, 2 ** 63 + 2 ** 61, 2 ** 64 - 5]
        t.build_index(0, L.INDEX_RANGE, keys)
        for kk in keys + [2 ** 63 + 12345, 3, 2 ** 64 - 1]:
            for cmp, op in (("<", np.less), (">=", np.greater_equal), ("=", np.equal)):
                fs = F.TableFilterSet({0: F.ConstantFilter(cmp, kk)})
                ref = np.flatnonzero(op(wide, np.uint64(kk)) & valid).astype(np.int64) + 9
                assert np.array_equal(t.scan(fs), ref), (cmp, kk)
        lo, hi, _, _ = t.column_statistics(0)
        assert (lo & (2 ** 64 - 1), hi & (2 ** 64 - 1)) == (int(wide[valid].min()), int(wide[valid].max()))
    t.close()


@pytest.mark.parametrize("mode", ["auto", "for", "delta_for", "constant_delta"])
def test_fused_sum_reads_uint32_segments(ctx, mode):
    """The fused sum reading `a` at the qualifying rows straight from UINTEGER segments (an
    INT64 column of 32-bit T: CONSTANT / CONSTANT_DELTA / FOR values taken in T's arithmetic,
    including descending runs whose deltas wrap in uint32): equal to numpy and to the plain
    column's sum."""
    rng = np.random.default_rng({"auto": 11, "for": 12, "delta_for": 13, "constant_delta": 14}[mode])
    n = 300_007
    a = rng.integers(0, 2 ** 32 - 1, n, dtype=np.uint64).astype(np.uint32)
    a[:2048] = 7
    a[2048:4096] = (4_000_000_000 - 3 * np.arange(2048)).astype(np.uint32)   # constant step -3
    a[4096:6144] = np.sort(rng.integers(0, 2 ** 31, 2048, dtype=np.uint64))[::-1].astype(np.uint32)
    c = O.bp_compress(a, None, mode)
    assert c is not None
    b = rng.integers(0, 11, n).astype(np.int64)
    key = rng.integers(0, 100, n).astype(np.int32)
    t = CubitTable(ctx, n, row_base=2)
    t.add_bitpacked_column(0, c.data, c.seg_off, c.seg_count, np.uint32)
    assert np.array_equal(t.download_column(0), a.astype(np.int64))
    t.add_column(1, b)
    t.add_column(2, key)
    t.build_index(2, L.INDEX_RANGE)
    for f in (F.ConstantFilter("<", 5), F.ConstantFilter(">=", 90)):
        fs = F.TableFilterSet({2: f})
        keep = key < 5 if f.comparison == "<" else key >= 90
        want = int((a[keep].astype(object) * b[keep].astype(object)).sum())
        s_packed, _ = t.sum_product(0, 1, fs, gather_b=True)
        assert t.last_sum_packed()
        s_plain, _ = t.sum_product(0, 1, fs, gather_b=True, packed_a=False)
        assert s_packed == want and s_plain == want, (mode, f.comparison)
    t.close()
