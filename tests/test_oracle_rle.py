"""DuckDB's RLE codec restated (oracle.rle_compress / rle_decode, src/storage/compression/rle.cpp),
pinned by the two RLE segments DuckDB wrote into the reference's data/storage/
huggingface_index.db.gz (terms.docid, terms.fieldid: tests/golden/bitpacking_reference_segments_fts.json):
the decoder reads them to the statistics their DataPointers store and to the FTS definitions
(docs.len = terms per doc), and the compressor writes their bytes exactly from the decoded
values. The restatement's corner cases — runs of 65,535 rows and their zero-length follow-ups,
leading NULLs, NULL-only row groups, segments split at the block's entry limit — round-trip for
every integer T. No GPU."""
import json
from pathlib import Path

import numpy as np
import pytest

from oracle import oracle as O

FTS = json.loads((Path(__file__).resolve().parent / "golden" / "bitpacking_reference_segments_fts.json").read_text())
RLE = [s for s in FTS["segments"] if s["compression"] == "rle"]


def seg_bytes(s):
    return np.frombuffer(bytes.fromhex(s["segment_hex"]), np.uint8)


@pytest.mark.parametrize("s", RLE, ids=[s["name"] for s in RLE])
def test_reference_rle_segments_decode_to_their_statistics_and_reencode_byte_for_byte(s):
    got = O.rle_decode(seg_bytes(s), [0], [s["count"]], np.int64)
    assert len(got) == s["count"]
    assert (int(got.min()), int(got.max())) == (s["statistics"]["min"], s["statistics"]["max"])
    data, offs, rows = O.rle_compress(got)
    assert offs.tolist() == [0] and rows.tolist() == [s["count"]]
    assert data.tobytes() == bytes.fromhex(s["segment_hex"])


def test_reference_rle_docids_count_each_docs_terms():
    """fts_indexing.cpp:110-116: docs.len[d] = rows of terms with docid d — docs.len is the
    BITPACKING segment's fixture values, terms.docid the RLE segment's decode."""
    by = {s["name"]: s for s in FTS["segments"]}
    docid = O.rle_decode(seg_bytes(by["terms.docid"]), [0], [5468], np.int64)
    assert np.bincount(docid, minlength=153).tolist() == by["docs.len"]["values"]


DTYPES = [np.int8, np.int16, np.int32, np.int64, np.uint8, np.uint16, np.uint32, np.uint64]


def runs_column(rng, dt, n, long_runs=True):
    info = np.iinfo(dt)
    pool = np.array([info.min, info.max, 0, 1, info.max // 3], dtype=dt)
    lens = rng.integers(1, 40, 4000)
    if long_runs:  # exact multiples of the limit and runs past it
        lens[::97] = 65535 * rng.integers(1, 3, len(lens[::97]))
        lens[5::131] = 65536
    vals = pool[rng.integers(0, len(pool), len(lens))]
    v = np.repeat(vals, lens)[:n]
    return v


@pytest.mark.parametrize("dt", DTYPES)
def test_round_trip_every_type_with_nulls_and_limits(dt):
    rng = np.random.default_rng(np.dtype(dt).itemsize * 7 + (dt in (np.uint8, np.uint16, np.uint32, np.uint64)))
    v = runs_column(rng, dt, 700_000)
    ok = rng.random(len(v)) > 0.05
    ok[:70_000] = False  # leading NULLs past the limit in the first row group
    ok[245_760:368_640] = False  # a NULL-only row group
    data, offs, rows = O.rle_compress(v, ok)
    assert int(rows.sum()) == len(v)
    got = O.rle_decode(data, offs, rows, dt)
    assert np.array_equal(got[ok], v[ok])


def test_zero_length_entries_and_segment_splits():
    """A run of exactly 65,535 rows is followed by a zero-length entry (RLEState::Update writes the
    full run, restarts at 0, and the next value flushes the empty one); a small block splits the
    entries over segments of (block - 8) / (sizeof(T) + 2) entries."""
    v = np.repeat(np.array([7, 9], np.int32), [65535, 3])
    data, offs, rows = O.rle_compress(v)
    b = data.tobytes()
    off = int.from_bytes(b[:8], "little")
    counts = np.frombuffer(b[off:], "<u2").tolist()
    assert counts == [65535, 0, 3]
    assert np.array_equal(O.rle_decode(data, offs, rows, np.int32), v)
    w = np.arange(1000, dtype=np.int64)
    data, offs, rows = O.rle_compress(w, block_size=8 + 10 * 100)  # 100 entries per segment
    assert len(offs) == 10 and rows.tolist() == [100] * 10
    assert np.array_equal(O.rle_decode(data, offs, rows, np.int64), w)


# ---- the reference's RLE .test cases (tests/golden/reference_cases.json "rle_cases") ------------
def rle_case_table(case):
    """(col INT32 values, col valid, id values or None): the case's runs; id as the inserts make it
    (range(10,000) as INTEGER or as VARCHAR strings)."""
    vals = np.concatenate([np.full(k, 0 if v is None else v, np.int32) for v, k in case["col"]])
    ok = np.concatenate([np.full(k, v is not None) for v, k in case["col"]])
    ids = None
    if case["id"] == "INTEGER":
        ids = np.arange(len(vals), dtype=np.int32)
    elif case["id"] == "VARCHAR":
        ids = [str(i).encode() for i in range(len(vals))]
    return vals, ok, ids


def rle_case_aggregates(rows, vals, ok, ids, id_is_str):
    """The aggregates the files select, over the rows a query kept."""
    out = {"count_star": len(rows)}
    v = vals[rows][ok[rows]]
    if len(v):
        out.update(sum=int(v.astype(np.int64).sum()), min=int(v.min()), max=int(v.max()))
    out["count"] = len(v)
    if ids is not None and len(rows):
        sel = [ids[r] for r in rows.tolist()]
        lo, hi = min(sel), max(sel)
        out.update(min_id=lo.decode() if id_is_str else int(lo), max_id=hi.decode() if id_is_str else int(hi))
    return out


def rle_case_filters(q, id_is_str):
    """The query's pushed filter over (col = column 0, id = column 1)."""
    if q["where"] is None:
        return None
    name, op, c = q["where"]
    if name == "id" and id_is_str:
        c = str(c).encode()
    return {0 if name == "col" else 1: ("=", c) if op == "=" else (op, c)}


@pytest.fixture(scope="module")
def rle_cases():
    g = json.loads((Path(__file__).resolve().parent / "golden" / "reference_cases.json").read_text())
    return g["rle_cases"]


def test_reference_rle_cases_on_the_oracle(rle_cases):
    """Each case's INTEGER column written as RLE segments by the restated compressor and read back
    by the restated decoder, then every query's pushed filter and aggregates against the file's
    results (rle_nulls_edge_case: 65,535 leading NULLs — the run-length limit — then 1, 2, 3)."""
    from cubit_amd import filters as F
    from cubit_amd.datagen import validity_from_mask

    for name, case in rle_cases.items():
        vals, ok, ids = rle_case_table(case)
        data, offs, rows = O.rle_compress(vals, ok)
        dec = O.rle_decode(data, offs, rows, np.int32)
        assert np.array_equal(dec[ok], vals[ok]), name
        id_is_str = case["id"] == "VARCHAR"
        cols = [O.Column(dec, None if ok.all() else validity_from_mask(ok))]
        if ids is not None:
            cols.append(O.StringColumn(ids) if id_is_str else O.Column(ids))
        for q in case["queries"]:
            fl = rle_case_filters(q, id_is_str)
            fs = F.TableFilterSet({c: F.ConstantFilter(op, k) for c, (op, k) in (fl or {}).items()})
            got_rows = O.table_scan(cols, F.serialize(fs), len(vals))
            agg = rle_case_aggregates(got_rows, dec, ok, ids, id_is_str)
            assert {k: agg.get(k) for k in q["expect"]} == q["expect"], (name, q)
    # the edge case's segment: the NULL run at the limit, then one entry per value
    vals, ok, _ = rle_case_table(rle_cases["rle_nulls_edge_case"])
    data, offs, rows = O.rle_compress(vals, ok)
    b = data.tobytes()
    off = int.from_bytes(b[:8], "little")
    assert np.frombuffer(b[off:], "<u2").tolist() == [65535, 1, 1, 1]
    assert np.frombuffer(b[8:8 + 16], "<i4").tolist() == [np.iinfo(np.int32).min, 1, 2, 3]
