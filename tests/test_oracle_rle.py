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
