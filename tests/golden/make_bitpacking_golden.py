"""Extract the BITPACKING column segments that DuckDB v1.1.2 itself wrote into a database
file the reference ships, with the values the reference says those columns hold, into
tests/golden/bitpacking_reference_segments.json. Run in the build container (where
/root/reference exists); the JSON is data only — segment bytes exactly as stored, plus
expected values taken from the reference's table definitions, never from a decoder.

Source file: test/sql/storage_version/storage_version.db (storage version 64, read by the
reference's own storage_version.test_slow), built by generate_storage_version.sql. Its
BITPACKING segments belong to:
  * big_integers.i      BIGINT  range(0, 100000)          generate_storage_version.sql:83-88
                                                          (storage_version.test_slow: COUNT 100000, SUM 4999950000)
  * base_table.i        BIGINT  range(4)                  generate_storage_version.sql:94
  * the child columns of test_all_types()'s fixed-size arrays
    (src/function/table/system/test_all_types.cpp:215-276; all_types = SELECT * FROM test_all_types()):
      fixed_int_array          INTEGER[3]    rows [NULL,2,3], [4,5,6], NULL
      fixed_nested_int_array   INTEGER[3][3] rows [[NULL,2,3],NULL,[NULL,2,3]], [[4,5,6],[NULL,2,3],[4,5,6]], NULL
      struct_of_fixed_array.a  INTEGER[3]    as fixed_int_array
      list_of_fixed_int_array  INTEGER[3][]  rows [min,max,min], [max,min,max], NULL  (its list child)
      fixed_array_of_int_list  INTEGER[][3]  rows [[],L,[]], [L,[],L], NULL with L = [42,999,NULL,NULL,-42]
                                             (the list offsets column: running ends, packed as uint64_t)
    A NULL array keeps its child slots; they are NULL (their stored bytes are whatever the
    compressor put there and are not compared).

Locating a segment: the table data's DataPointers (serialize_storage.cpp:27-34: field 100
row_start, 101 tuple_count, 102 block_pointer {100 block_id, 101 offset}, 103
compression_type, …, BinarySerializer field ids + LEB128) are found in the metadata by that
byte shape with compression_type = COMPRESSION_BITPACKING (6, compression_type.hpp:23); the
segment lies at file offset 3·4096 + block_id·block_alloc_size + 8 (block checksum) + offset
(single_file_block_manager.cpp), and its first 8 bytes give the end of its metadata, i.e. its
size (bitpacking.cpp FlushSegment)."""
import json
import struct
from pathlib import Path

REF = Path("/root/reference")
DB = REF / "test/sql/storage_version/storage_version.db"
OUT = Path(__file__).resolve().parent / "bitpacking_reference_segments.json"
HEADER = 3 * 4096
BLOCK_ALLOC = 262144
BITPACKING = 6


def uleb(d, p):
    r = s = 0
    while True:
        b = d[p]
        p += 1
        r |= (b & 0x7F) << s
        s += 7
        if not b & 0x80:
            return r, p


def sleb(d, p):
    r = s = 0
    while True:
        b = d[p]
        p += 1
        r |= (b & 0x7F) << s
        s += 7
        if not b & 0x80:
            if b & 0x40:
                r -= 1 << s
            return r, p


def data_pointers(d):
    """(tuple_count, block_id, offset, compression) of every DataPointer in the file."""
    out, p = [], 0
    while True:
        p = d.find(b"\x66\x00\x64\x00", p)  # field 102 block_pointer { field 100 block_id
        if p < 0:
            return out
        q = p + 4
        bid, q = sleb(d, q)
        off = 0
        if d[q:q + 2] == b"\x65\x00":
            off, q = uleb(d, q + 2)
        if d[q:q + 4] == b"\xff\xff\x67\x00":  # end of block_pointer, field 103 compression
            comp = d[q + 4]
            count = None
            for back in range(3, 14):  # field 101 tuple_count ends where field 102 starts
                if d[p - back:p - back + 2] == b"\x65\x00":
                    c, e = uleb(d, p - back + 2)
                    if e == p:
                        count = c
                        break
            out.append((count, bid, off, comp))
        p += 1


N = None
# running list ends: [], L, [] | L, [], L | the NULL row's three lists, length 0 each (L has 5 elements)
L_ENDS = [0, 5, 5, 10, 10, 15, 15, 15, 15]
EXPECTED = {
    # name: (dtype, values with None = NULL — or {"range": [a, b]} for a, a+1, …, b-1 —, reference line)
    "big_integers.i": ("int64", {"range": [0, 100000]}, "generate_storage_version.sql:83-88"),
    "base_table.i": ("int64", [0, 1, 2, 3], "generate_storage_version.sql:94"),
    "all_types.fixed_int_array (child)": ("int32", [N, 2, 3, 4, 5, 6, N, N, N], "test_all_types.cpp:215-219"),
    "all_types.struct_of_fixed_array.a (child)": ("int32", [N, 2, 3, 4, 5, 6, N, N, N], "test_all_types.cpp:253-261"),
    "all_types.fixed_nested_int_array (child)": ("int32", [N, 2, 3, N, N, N, N, 2, 3, 4, 5, 6, N, 2, 3, 4, 5, 6] + [N] * 9,
                                                 "test_all_types.cpp:228-235"),
    "all_types.list_of_fixed_int_array (list child)": ("int32", [N, 2, 3, 4, 5, 6, N, 2, 3, 4, 5, 6, N, 2, 3, 4, 5, 6],
                                                       "test_all_types.cpp:270-276"),
    # LIST offsets are bit-packed as uint64_t (bitpacking.cpp:976-977)
    "all_types.fixed_array_of_int_list (list offsets)": ("uint64", L_ENDS, "test_all_types.cpp:263-268, 99-104"),
}


def attribute(count, seg):
    """Which column a segment holds: by its row count and, where counts coincide, by the
    storage order of all_types' columns (fixed_int_array precedes struct_of_fixed_array)."""
    if count == 100000:
        return "big_integers.i"
    if count == 4:
        return "base_table.i"
    if count == 27:
        return "all_types.fixed_nested_int_array (child)"
    if count == 18:
        return "all_types.list_of_fixed_int_array (list child)"
    if count == 9:
        mode = struct.unpack_from("<I", seg, struct.unpack_from("<Q", seg, 0)[0] - 4)[0] >> 24
        return "all_types.fixed_array_of_int_list (list offsets)" if mode == 4 else "all_types.fixed_int_array (child)"
    raise SystemExit(f"unattributed BITPACKING segment of {count} rows")


def main():
    d = DB.read_bytes()
    assert d[8:12] == b"DUCK" and struct.unpack_from("<Q", d, 12)[0] == 64, "storage version 64 expected"
    segs = []
    seen_nine = 0
    for count, bid, off, comp in data_pointers(d):
        if comp != BITPACKING:
            continue
        pos = HEADER + bid * BLOCK_ALLOC + 8 + off
        size = struct.unpack_from("<Q", d, pos)[0]
        seg = d[pos:pos + size]
        name = attribute(count, seg)
        if name == "all_types.fixed_int_array (child)":
            seen_nine += 1
            if seen_nine == 2:
                name = "all_types.struct_of_fixed_array.a (child)"
        dtype, values, line = EXPECTED[name]
        n_values = values["range"][1] - values["range"][0] if isinstance(values, dict) else len(values)
        assert n_values == count, name
        segs.append({"name": name, "dtype": dtype, "count": count, "segment_hex": seg.hex(),
                     "values": values, "reference": line,
                     "file_offset": pos, "block_id": bid, "block_offset": off})
    assert sorted(s["name"] for s in segs) == sorted(EXPECTED), [s["name"] for s in segs]
    OUT.write_text(json.dumps({
        "source": str(DB.relative_to(REF)) + " (DuckDB v1.1.2 storage version 64; read back by "
                  "test/sql/storage_version/storage_version.test_slow)",
        "what": "BITPACKING segment images exactly as DuckDB wrote them (8-byte header = end of metadata, "
                "group data, metadata words read downward), with the values the reference's table definitions "
                "give (null = NULL row; its stored bytes are not compared)",
        "generator": "tests/golden/make_bitpacking_golden.py",
        "segments": segs}, indent=1) + "\n")
    print(f"wrote {len(segs)} segments to {OUT}")


if __name__ == "__main__":
    main()
