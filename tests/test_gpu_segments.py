"""Columns whose DuckDB segments mix codecs (cubit_table_add_segment_column): DuckDB's checkpoint
picks a codec per row group (ColumnDataCheckpointer), so one column may hold UNCOMPRESSED,
CONSTANT, RLE and BITPACKING segments side by side. Each row group here is written by the
oracle's restatement of its codec (bp_compress, rle_compress; a CONSTANT group as its value;
UNCOMPRESSED as the values' bytes); the GPU column equals the values at every valid row for every
integer T, and scans over it (unindexed, range, equality) equal the oracle's."""
import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from cubit_amd.table import Context, CubitTable
from oracle import oracle as O

pytestmark = pytest.mark.gpu

RG = 122_880
DTYPES = [np.int8, np.int16, np.int32, np.int64, np.uint8, np.uint16, np.uint32, np.uint64]


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def mixed_column(rng, dt, n_groups, tail):
    """Values, validity and segments: row group g written with codec g mod 4 (shuffled)."""
    dt = np.dtype(dt)
    info = np.iinfo(dt)
    n = n_groups * RG + tail
    vals = np.empty(n, dtype=dt)
    ok = rng.random(n) > 0.05
    segs = []
    codecs = rng.permutation(np.resize([L.CODEC_UNCOMPRESSED, L.CODEC_CONSTANT, L.CODEC_RLE, L.CODEC_BITPACKING],
                                       n_groups + (1 if tail else 0)))
    for g, codec in enumerate(codecs.tolist()):
        lo, hi = g * RG, min(n, (g + 1) * RG)
        m = hi - lo
        if codec == L.CODEC_CONSTANT:
            c = dt.type([info.min, info.max, 0, 7][int(rng.integers(0, 4))])
            vals[lo:hi] = c
            ok[lo:hi] = True  # a CONSTANT segment's rows are all valid and equal
            segs.append((codec, int(c), m))
        elif codec == L.CODEC_RLE:
            v = np.repeat(rng.integers(0, 50, m).astype(dt), rng.integers(1, 200, m))[:m]
            vals[lo:hi] = v
            data, offs, rows = O.rle_compress(v, ok[lo:hi], row_group=RG)
            for o, r, nxt in zip(offs.tolist(), rows.tolist(), offs.tolist()[1:] + [len(data)]):
                segs.append((codec, data[o:nxt].tobytes(), r))
        elif codec == L.CODEC_BITPACKING:
            span = min(1000, int(info.max) // 4)  # max - min must fit T (bp_compress refuses otherwise)
            v = (rng.integers(0, span, m) + (int(info.max) // 4 if info.max > 4000 else 0)).astype(dt)
            vals[lo:hi] = v
            bp = O.bp_compress(v, ok[lo:hi].astype(np.uint8), "auto")
            for o, size, r in zip(bp.seg_off.tolist(), bp.seg_size.tolist(), bp.seg_count.tolist()):
                segs.append((codec, bp.data[o:o + size].tobytes(), r))
        else:
            v = rng.integers(0, min(3000, int(info.max)), m).astype(dt)  # few distinct: the equality index takes them
            v[:2] = [info.min, info.max]
            vals[lo:hi] = v
            segs.append((codec, v.tobytes(), m))
    return vals, ok, segs


@pytest.mark.parametrize("dt", DTYPES)
def test_mixed_codecs_every_type(ctx, dt):
    rng = np.random.default_rng(np.dtype(dt).itemsize * 13 + "iu".index(np.dtype(dt).kind))
    vals, ok, segs = mixed_column(rng, dt, 6, 5_001)
    vw = validity_from_mask(ok)
    t = CubitTable(ctx, len(vals))
    t.add_segment_column(0, segs, dt, vw)
    got = t.download_column(0)
    want = vals.astype(np.uint64) if np.dtype(dt) == np.uint64 else vals.astype(np.int64)
    held = got.view(np.uint64) if np.dtype(dt) == np.uint64 else got.astype(np.int64)
    assert np.array_equal(held[ok], want[ok])
    ocol = O.Column(want.astype(np.uint64) if np.dtype(dt) == np.uint64 else
                    want.astype(np.int32 if t.types[0] == L.TYPE_INT32 else np.int64), vw)
    consts = [0, 7, 49, int(np.iinfo(dt).max), int(np.iinfo(dt).min)]
    for enc in (None, L.INDEX_RANGE, L.INDEX_EQUALITY):
        if enc is not None:
            t.build_index(0, enc)
        for c in consts:
            for op in ("=", "<", ">=", "!="):
                fs = F.TableFilterSet({0: F.ConstantFilter(op, c)})
                assert np.array_equal(t.scan(fs), O.table_scan([ocol], F.serialize(fs), len(vals))), (dt, enc, op, c)
    t.close()


def test_single_codec_columns_match_their_own_entry_points(ctx):
    """All-RLE and all-BITPACKING columns through the mixed entry point equal
    cubit_table_add_rle_column's and cubit_table_add_bitpacked_column's; a bad codec is refused."""
    rng = np.random.default_rng(5)
    v = np.repeat(rng.integers(0, 9, 50_000).astype(np.int32), rng.integers(1, 30, 50_000))[:700_000]
    data, offs, rows = O.rle_compress(v)
    a, b = CubitTable(ctx, len(v)), CubitTable(ctx, len(v))
    a.add_rle_column(0, data, offs, rows, np.int32)
    segs = [(L.CODEC_RLE, data[o:nx].tobytes(), r)
            for o, r, nx in zip(offs.tolist(), rows.tolist(), offs.tolist()[1:] + [len(data)])]
    b.add_segment_column(0, segs, np.int32)
    assert np.array_equal(a.download_column(0), b.download_column(0))
    bp = O.bp_compress(v.astype(np.int64), None, "auto")
    a.add_bitpacked_column(1, bp.data, bp.seg_off, bp.seg_count, np.int64)
    b.add_segment_column(1, [(L.CODEC_BITPACKING, bp.data[o:o + s].tobytes(), r)
                             for o, s, r in zip(bp.seg_off.tolist(), bp.seg_size.tolist(), bp.seg_count.tolist())],
                         np.int64)
    assert np.array_equal(a.download_column(1), b.download_column(1))
    with pytest.raises(L.CubitError):
        b.add_segment_column(2, [(9, b"\0" * 8, len(v))], np.int32)
    a.close()
    b.close()
