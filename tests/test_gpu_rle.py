"""DuckDB RLE segments on the GPU (cubit_table_add_rle_column): the runs read on the host, expanded
by rle_expand_kernel. The reference's own RLE segments (huggingface_index.db: terms.docid,
terms.fieldid) expand to the oracle's decode; segments the restated compressor writes — every
integer T, NULLs, runs of 65,535 rows and their zero-length follow-ups, runs across tile
boundaries, several segments, one-row runs filling a tile's LDS window — expand to the
values, and scans over them (unindexed, range, equality) equal the oracle's; malformed segments
are refused."""
import json
from pathlib import Path

import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from cubit_amd.table import Context, CubitTable
from oracle import oracle as O
from test_oracle_rle import DTYPES, runs_column

pytestmark = pytest.mark.gpu

FTS = json.loads((Path(__file__).resolve().parent / "golden" / "bitpacking_reference_segments_fts.json").read_text())
RLE = [s for s in FTS["segments"] if s["compression"] == "rle"]


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


def held(t, col, dt):
    """The column as held, compared as the values (UINT64: the bits)."""
    got = t.download_column(col)
    return got.view(np.uint64) if np.dtype(dt) == np.uint64 else got.astype(np.int64)


@pytest.mark.parametrize("s", RLE, ids=[s["name"] for s in RLE])
def test_reference_segments(ctx, s):
    seg = np.frombuffer(bytes.fromhex(s["segment_hex"]), np.uint8)
    want = O.rle_decode(seg, [0], [s["count"]], np.int64)
    t = CubitTable(ctx, s["count"])
    t.add_rle_column(0, seg, [0], [s["count"]], np.int64)
    assert np.array_equal(t.download_column(0), want)
    lo, hi, _, _ = t.column_statistics(0)
    assert (lo, hi) == (s["statistics"]["min"], s["statistics"]["max"])
    t.build_index(0, L.INDEX_EQUALITY)
    for c in (0, 1, 76, 152):
        fs = F.TableFilterSet({0: F.ConstantFilter("=", c)})
        assert np.array_equal(t.scan(fs), np.flatnonzero(want == c))
    t.close()


@pytest.mark.parametrize("dt", DTYPES)
def test_compressed_segments_every_type(ctx, dt):
    rng = np.random.default_rng(np.dtype(dt).itemsize * 11 + "iu".index(np.dtype(dt).kind))
    v = runs_column(rng, dt, 600_000)
    ok = rng.random(len(v)) > 0.05
    ok[:70_000] = False
    data, offs, rows = O.rle_compress(v, ok)
    vw = validity_from_mask(ok)
    t = CubitTable(ctx, len(v))
    t.add_rle_column(0, data, offs, rows, dt, vw)
    got = held(t, 0, dt)
    want = O.rle_decode(data, offs, rows, dt)
    assert np.array_equal(got, want.astype(np.uint64) if np.dtype(dt) == np.uint64 else want.astype(np.int64))
    col = O.Column(want.astype(np.uint64) if np.dtype(dt) == np.uint64 else
                   want.astype(np.int32 if t.types[0] == L.TYPE_INT32 else np.int64), vw)
    for enc in (None, L.INDEX_RANGE, L.INDEX_EQUALITY):
        if enc is not None:
            t.build_index(0, enc)
        for c in [int(x) for x in np.unique(v)[:3]] + [int(np.iinfo(dt).max)]:
            for op in ("=", "<", ">=", "!="):
                fs = F.TableFilterSet({0: F.ConstantFilter(op, c)})
                assert np.array_equal(t.scan(fs), O.table_scan([col], F.serialize(fs), len(v))), (dt, enc, op, c)
    t.close()


def test_many_short_runs_and_segments(ctx):
    """One-row runs (a tile's 2,048 runs fill its whole LDS window), over a hundred segments of
    5,000 runs, and a partition of one row."""
    rng = np.random.default_rng(9)
    v = rng.integers(-1000, 1000, 1_000_003).astype(np.int32)  # every run one row
    data, offs, rows = O.rle_compress(v, block_size=8 + 6 * 5000)  # 5,000 runs per segment
    assert len(offs) > 100
    t = CubitTable(ctx, len(v))
    t.add_rle_column(0, data, offs, rows, np.int32)
    assert np.array_equal(t.download_column(0), v)
    t.close()
    one = np.array([42], np.int64)
    data, offs, rows = O.rle_compress(one)
    t = CubitTable(ctx, 1)
    t.add_rle_column(0, data, offs, rows, np.int64)
    assert t.download_column(0).tolist() == [42]
    t.close()


def test_malformed_segments_are_refused(ctx):
    v = np.repeat(np.arange(10, dtype=np.int64), 100)
    data, offs, rows = O.rle_compress(v)
    t = CubitTable(ctx, len(v))
    with pytest.raises(L.CubitError):  # the runs cover fewer rows than the segment claims
        t.add_rle_column(0, data, offs, rows + 1, np.int64)
    bad = data.copy()
    bad[:8] = np.frombuffer((10 ** 6).to_bytes(8, "little"), np.uint8)  # run lengths past the bytes
    with pytest.raises(L.CubitError):
        t.add_rle_column(0, bad, offs, rows, np.int64)
    t.add_rle_column(0, data, offs, rows, np.int64)
    assert np.array_equal(t.download_column(0), v)
    t.close()


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
def test_reference_rle_cases(ctx, encoding):
    """The reference's RLE .test cases (rle_filter_pushdown, rle_index_fetch, rle_medium,
    rle_nulls_edge_case): the INTEGER column registered from RLE segments, the id column beside it
    (INTEGER, or VARCHAR as dictionary codes), every query's pushed filter on the GPU and its
    aggregates over the probed values = the file's results."""
    from test_oracle_rle import rle_case_aggregates, rle_case_filters, rle_case_table

    cases = json.loads((Path(__file__).resolve().parent / "golden" / "reference_cases.json").read_text())["rle_cases"]
    for name, case in cases.items():
        vals, ok, ids = rle_case_table(case)
        data, offs, rows = O.rle_compress(vals, ok)
        t = CubitTable(ctx, len(vals))
        t.add_rle_column(0, data, offs, rows, np.int32, None if ok.all() else validity_from_mask(ok))
        id_is_str = case["id"] == "VARCHAR"
        d = None
        if ids is not None:
            if id_is_str:
                d = t.add_string_column(1, ids)
            else:
                t.add_column(1, ids)
        if encoding is not None:
            t.build_index(0, encoding)
        for q in case["queries"]:
            fl = rle_case_filters(q, id_is_str)
            fs = F.TableFilterSet({c: F.ConstantFilter(op, k) for c, (op, k) in (fl or {}).items()})
            got = t.scan(fs)
            v, vok = t.fetch(0, got)
            gv = np.zeros(len(vals), np.int32)
            gok = np.zeros(len(vals), bool)
            gv[got], gok[got] = v, vok
            gid = None
            if ids is not None:
                iv, _ = t.fetch(1, got)
                gid = {r: (d.entry(c) if id_is_str else int(c)) for r, c in zip(got.tolist(), iv.tolist())}
            agg = rle_case_aggregates(got, gv, gok, gid, id_is_str)
            assert {k: agg.get(k) for k in q["expect"]} == q["expect"], (name, q, encoding)
        t.close()
