"""Extract the BITPACKING segments of data/storage/huggingface_index.db.gz — a full-text-search
index that DuckDB (v0.10.0, storage version 64, the format the v1.1.2 reader attaches in
test/sql/attach/attach_huggingface_index.test) wrote — into
tests/golden/bitpacking_reference_segments_fts.json. Run in the build container (where
/root/reference exists); the JSON is data only: segment bytes exactly as stored, each segment's
statistics as its DataPointer stores them, the RLE segments of the same tables, and the stats
table's avgdl.

Why these segments pin the decoder beyond the values of storage_version.db: they are FOR groups
of 7, 8 and 11 bits (widths the other file does not have) whose values are tied together by the
FTS extension's own definitions (extension/fts/fts_indexing.cpp:83-149):
  docs(docid = rowid, name = the input id, len = count(term) of the doc's terms rows)   :83-87, 110-116
  dict(termid = row_number() - 1 over the distinct terms, df = count(distinct docid))  :118-144
  terms(docid, fieldid, termid)                                                         :92-108, 126-134
  stats(num_docs = count(docid), avgdl = sum(len) / count(len))                         :146-149
terms.docid and terms.fieldid are RLE segments (src/storage/compression/rle.cpp: 8-byte header =
offset of the uint16 run lengths, then the run values), so docs.len — FOR, 153 values — is
pinned value by value by the RLE column (stored here as `values`); dict.df and terms.termid —
FOR, 1,558 and 5,468 values — are pinned jointly (every termid's distinct docids = its df, every
termid 0..1557 present) and by their statistics; the CONSTANT_DELTA columns by their definitions.

Locating segments: as make_bitpacking_golden.py (DataPointer byte shape, BinarySerializer field
ids + LEB128); the statistics follow the compression type as field 104 (serialize_storage.cpp:27-34,
base_statistics.cpp:311-336, numeric_stats.cpp:420-532: field 200 holds the minimum, 201 the
maximum)."""
import gzip
import json
import struct
from pathlib import Path

from make_bitpacking_golden import BLOCK_ALLOC, HEADER, sleb, uleb

REF = Path("/root/reference")
DB = REF / "data/storage/huggingface_index.db.gz"
OUT = Path(__file__).resolve().parent / "bitpacking_reference_segments_fts.json"
CONSTANT, RLE, BITPACKING = 2, 3, 6  # compression_type.hpp


def numeric_stats(d, q):
    """(has_null, has_no_null, min, max) of an integer column's BaseStatistics at field 104."""
    assert d[q:q + 2] == b"\x68\x00"
    q += 2
    out = {}
    while True:
        fid = struct.unpack_from("<H", d, q)[0]
        q += 2
        if fid == 0xFFFF:
            return out
        if fid in (100, 101):
            out["has_null" if fid == 100 else "has_no_null"] = bool(d[q])
            q += 1
        elif fid == 102:
            _, q = uleb(d, q)
        elif fid == 103:
            while True:
                f2 = struct.unpack_from("<H", d, q)[0]
                q += 2
                if f2 == 0xFFFF:
                    break
                has, v = False, None
                while True:
                    f3 = struct.unpack_from("<H", d, q)[0]
                    q += 2
                    if f3 == 0xFFFF:
                        break
                    if f3 == 100:
                        has = bool(d[q])
                        q += 1
                    else:
                        v, q = sleb(d, q)
                out["min" if f2 == 200 else "max"] = v if has else None
        else:
            raise SystemExit(f"unexpected statistics field {fid}")


def pointers(d):
    """Every DataPointer: (tuple_count, block_id, offset, compression, offset of its statistics)."""
    out, p = [], 0
    while True:
        p = d.find(b"\x66\x00\x64\x00", p)
        if p < 0:
            return out
        q = p + 4
        bid, q = sleb(d, q)
        off = 0
        if d[q:q + 2] == b"\x65\x00":
            off, q = uleb(d, q + 2)
        if d[q:q + 4] == b"\xff\xff\x67\x00":
            count = None
            for back in range(3, 14):
                if d[p - back:p - back + 2] == b"\x65\x00":
                    c, e = uleb(d, p - back + 2)
                    if e == p:
                        count = c
                        break
            out.append((count, bid, off, d[q + 4], q + 5))
        p += 1


def segment(d, bid, off, comp, count):
    pos = HEADER + bid * BLOCK_ALLOC + 8 + off
    if comp == BITPACKING:
        size = struct.unpack_from("<Q", d, pos)[0]  # end of the metadata (bitpacking.cpp FlushSegment)
    else:  # RLE: the run lengths end the segment; runs are read until they cover the rows
        rle_off = struct.unpack_from("<Q", d, pos)[0]
        runs, covered = 0, 0
        while covered < count:
            covered += struct.unpack_from("<H", d, pos + rle_off + 2 * runs)[0]
            runs += 1
        size = rle_off + 2 * runs
    return d[pos:pos + size]


def rle_values(seg, count):
    """The RLE column's values (rle.cpp RLEScanState: values from byte 8, uint16 run lengths at
    the header's offset) — BIGINT runs."""
    rle_off = struct.unpack_from("<Q", seg, 0)[0]
    out, i = [], 0
    while len(out) < count:
        v = struct.unpack_from("<q", seg, 8 + 8 * i)[0]
        n = struct.unpack_from("<H", seg, rle_off + 2 * i)[0]
        out += [v] * n
        i += 1
    return out


def avgdl(d):
    """stats.avgdl: the DOUBLE column's one value, as its CONSTANT segment's statistics hold it
    (min = max; a double statistic is the value's 8 raw bytes)."""
    for count, bid, off, comp, q in pointers(d):
        if count == 1 and comp == CONSTANT:
            s = d[q:q + 64]
            k = s.find(b"\xc8\x00\x64\x00\x01\x65\x00")
            # 8 raw bytes then the end of the object (num_docs, a BIGINT, is a 2-byte LEB128)
            if k >= 0 and s[:2] == b"\x68\x00" and s[k + 15:k + 17] == b"\xff\xff":
                return struct.unpack_from("<d", s, k + 7)[0]
    raise SystemExit("stats.avgdl not found")


def main():
    d = gzip.decompress(DB.read_bytes())
    assert d[8:12] == b"DUCK" and struct.unpack_from("<Q", d, 12)[0] == 64, "storage version 64 expected"
    # (count, compression, statistics) → column, in the file's table order: dict(termid, term, df),
    # docs(docid, name, len), terms(docid, fieldid, termid), data(act, prompt, __hf_index_id)
    found = {}
    for count, bid, off, comp, q in pointers(d):
        if comp not in (BITPACKING, RLE) or bid < 0:
            continue
        st = numeric_stats(d, q)
        seg = segment(d, bid, off, comp, count)
        key = (count, comp)
        found.setdefault(key, []).append({"count": count, "compression": "bitpacking" if comp == BITPACKING else "rle",
                                          "block_id": bid, "block_offset": off, "statistics": st,
                                          "segment_hex": seg.hex()})
    names = {(1558, BITPACKING): ["dict.termid", "dict.df"],
             (153, BITPACKING): ["docs.docid", "docs.name", "docs.len", "data.__hf_index_id"],
             (5468, RLE): ["terms.docid", "terms.fieldid"],
             (5468, BITPACKING): ["terms.termid"]}
    segs = []
    for key, cols in names.items():
        got = found.pop(key)
        assert len(got) == len(cols), (key, len(got))
        for name, s in zip(cols, got):
            s["name"] = name
            segs.append(s)
    assert not found, found.keys()
    by = {s["name"]: s for s in segs}
    docid = rle_values(bytes.fromhex(by["terms.docid"]["segment_hex"]), 5468)
    fieldid = rle_values(bytes.fromhex(by["terms.fieldid"]["segment_hex"]), 5468)
    assert min(docid) == by["terms.docid"]["statistics"]["min"] and max(docid) == by["terms.docid"]["statistics"]["max"]
    assert set(fieldid) == {0, 1}
    length = [0] * 153
    for x in docid:
        length[x] += 1
    dl = avgdl(d)
    assert abs(sum(length) / 153 - dl) < 1e-9, (sum(length) / 153, dl)
    ref = {
        "dict.termid": ({"range": [0, 1558]}, "row_number() OVER () - 1 (fts_indexing.cpp:118-125)"),
        "docs.docid": ({"range": [0, 153]}, "rowid of the input table (fts_indexing.cpp:83-87)"),
        "docs.name": ({"range": [0, 153]}, "the input id __hf_index_id, 0 … 152 (its DataPointer statistics)"),
        "data.__hf_index_id": ({"range": [0, 153]}, "the input table's id column, 0 … 152 (its statistics)"),
        "docs.len": (length, "count(term) per docid over terms (fts_indexing.cpp:110-116), counted from the "
                             "RLE segment terms.docid; Σ len / 153 = stats.avgdl"),
        "dict.df": (None, "count(distinct docid) per termid over terms (fts_indexing.cpp:137-144): pinned jointly "
                          "with terms.termid"),
        "terms.termid": (None, "the dict termid of each terms row (fts_indexing.cpp:126-134): every termid "
                               "0 … 1557 appears, and its rows' distinct docids number dict.df[termid]"),
    }
    for s in segs:
        if s["compression"] == "bitpacking":
            s["dtype"] = "int64"
            s["values"], s["reference"] = ref[s["name"]]
    OUT.write_text(json.dumps({
        "source": str(DB.relative_to(REF)) + " (gzip; a full-text-search index DuckDB v0.10.0 wrote in storage "
                  "version 64, attached by test/sql/attach/attach_huggingface_index.test)",
        "what": "BITPACKING segments of the FTS tables (FOR groups of 7, 8 and 11 bits; CONSTANT_DELTA), bytes "
                "exactly as stored, with each segment's DataPointer statistics; the RLE segments terms.docid and "
                "terms.fieldid; stats.avgdl. values = what the FTS definitions give (null: pinned jointly, see "
                "`invariants`)",
        "invariants": ["docs.len[d] = #rows of terms with docid d (values, from the RLE column)",
                       "dict.df[t] = #distinct docid over rows of terms with termid t",
                       "terms.termid takes every value 0 … 1557",
                       "every segment's decoded min / max = its DataPointer statistics",
                       "sum(docs.len) / 153 = stats.avgdl"],
        "stats_avgdl": dl,
        "generator": "tests/golden/make_bitpacking_golden_fts.py",
        "segments": segs}, indent=1) + "\n")
    print(f"wrote {len(segs)} segments to {OUT}")


if __name__ == "__main__":
    main()
