"""The BITPACKING restatement (oracle/bitpacking_ref.c) against the reference's own
bitpacking tests: the values each test reads back after a checkpoint under every forced
mode, and the mode DuckDB's Flush picks (test/sql/storage/compression/bitpacking/*.test)."""
import numpy as np
import pytest

from oracle import oracle as O

MODES = ["auto", "for", "delta_for", "constant_delta", "constant"]


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("dtype", [np.int32, np.int64])
def test_constant_delta_reference_case(mode, dtype):
    """bitpacking_constant_delta.test: INSERT 2+i*2 FROM range(0,5) under each forced mode →
    SELECT * returns 2,4,6,8,10."""
    v = (2 + np.arange(5) * 2).astype(dtype)
    c = O.bp_compress(v, None, mode)
    assert c is not None
    assert O.bp_decode(c).tolist() == [2, 4, 6, 8, 10]
    # Flush's choice: forced FOR / DELTA_FOR are honoured, AUTO / CONSTANT / CONSTANT_DELTA
    # take CONSTANT_DELTA (one distinct delta)
    want = {"for": "for", "delta_for": "delta_for"}.get(mode, "constant_delta")
    assert O.bp_group_modes(c) == [want]


def test_range_130000_reference_case():
    """bitpacking_constant_delta.test: INT64 range(0,130000) → avg(c) = 64999.5."""
    v = np.arange(130000, dtype=np.int64)
    c = O.bp_compress(v, None, "auto")
    d = O.bp_decode(c)
    assert d.mean() == 64999.5 and np.array_equal(d, v)
    assert set(O.bp_group_modes(c)) == {"constant_delta"}


@pytest.mark.parametrize("mode", MODES)
def test_round_trips_and_segments(mode):
    rng = np.random.default_rng(5)
    cases = [
        np.full(5000, -7, np.int32),
        np.cumsum(rng.integers(0, 9, 20000)).astype(np.int32),             # sorted: DELTA_FOR
        rng.integers(-1000, 1000, 100_000).astype(np.int32),               # FOR, width 11
        rng.integers(-2 ** 40, 2 ** 40, 300_000).astype(np.int64),         # FOR, several segments
        (np.arange(9000, dtype=np.int64) * -3 + 10 ** 15),                 # CONSTANT_DELTA, negative delta
        np.array([np.iinfo(np.int32).min, np.iinfo(np.int32).max] * 3000, np.int32),  # max-min overflows
    ]
    for v in cases:
        c = O.bp_compress(v, None, mode)
        if c is None:  # not bitpackable: only the overflowing column
            assert v.dtype == np.int32 and v.min() == np.iinfo(np.int32).min
            continue
        assert np.array_equal(O.bp_decode(c), v)
        assert c.seg_off[0] == 0 and np.all(c.seg_off % 8 == 0)
        assert int(c.seg_count.sum()) == len(v)
    big = O.bp_compress(rng.integers(-2 ** 40, 2 ** 40, 300_000).astype(np.int64), None, mode)
    assert len(big.seg_off) > 1 and np.all(big.seg_size <= O.DUCKDB_BLOCK_SIZE)


def test_nulls_and_all_null_groups():
    rng = np.random.default_rng(6)
    v = rng.integers(0, 500, 10_000).astype(np.int32)
    valid = rng.random(10_000) > 0.3
    valid[2048:4096] = False  # an all-NULL group → CONSTANT
    c = O.bp_compress(v, valid, "auto")
    d = O.bp_decode(c)
    assert np.array_equal(d[valid], v[valid])
    assert O.bp_group_modes(c)[1] == "constant"


@pytest.mark.parametrize("kind", ["dates", "wide64", "constant", "price"])
def test_bench_packer_decodes_with_oracle(kind, li01):
    """bench.py's K5 input generator (libcubit_datagen cubit_bitpack_for) writes segments the
    oracle's restatement of the reference decoder reads back exactly."""
    from cubit_amd import datagen

    rng = np.random.default_rng(3)
    n = 400_009
    v = {"dates": li01.l_shipdate[:n],
         "wide64": rng.integers(-2 ** 62, 2 ** 62, n).astype(np.int64),
         "constant": np.full(n, 42, np.int32),
         "price": li01.l_extendedprice[:n]}[kind]
    b = datagen.bitpack_for(v)
    col = O.BitpackedColumn(b.data, b.seg_off, None, b.seg_count, v.dtype)
    assert np.array_equal(O.bp_decode(col), v)
    assert set(O.bp_group_modes(col)) <= {"constant", "for"}


# ---------------------------------------------------------------- segments DuckDB itself wrote

import json
from pathlib import Path

REF_SEGMENTS = json.loads((Path(__file__).resolve().parent / "golden" / "bitpacking_reference_segments.json")
                          .read_text())["segments"]


def reference_segment(s):
    """(segment bytes as a one-segment BitpackedColumn, expected values, validity) of a fixture
    entry (tests/golden/make_bitpacking_golden.py: bytes exactly as DuckDB v1.1.2 stored them)."""
    raw = np.frombuffer(bytes.fromhex(s["segment_hex"]), dtype=np.uint8)
    data = np.zeros((len(raw) + 7) // 8 * 8 + 8, dtype=np.uint8)  # the decoder may read a word past the end
    data[: len(raw)] = raw
    dt = np.dtype(s["dtype"])
    vals = s["values"]
    if isinstance(vals, dict):
        vals = list(range(*vals["range"]))
    valid = np.array([v is not None for v in vals])
    values = np.array([0 if v is None else v for v in vals], dtype=dt)
    col = O.BitpackedColumn(data, np.array([0], np.uint64), np.array([len(raw)], np.uint64),
                            np.array([s["count"]], np.uint64), dt)
    return col, values, valid


def packed_tail_masked(seg: bytes, tsize: int, count: int) -> bytes:
    """A one-group FOR / DELTA_FOR segment with the packed bits past value `count` zeroed: DuckDB
    packs whole 32-value blocks from a reused buffer, so those bits are left-overs, not data."""
    b = bytearray(seg)
    end = int.from_bytes(b[:8], "little")
    meta = int.from_bytes(b[end - 4:end], "little")
    mode, off = meta >> 24, meta & 0xFFFFFF
    if mode not in (4, 5) or count > 2048:
        return bytes(b)
    fields = 3 if mode == 4 else 2  # DELTA_FOR: FOR, width, delta offset; FOR: FOR, width
    width = int.from_bytes(b[off + tsize: off + 2 * tsize], "little", signed=True)
    packed = off + fields * tsize
    blocks = (count + 31) // 32
    for bit in range(count * width, blocks * 32 * width):
        b[packed + bit // 8] &= ~(1 << (bit % 8)) & 0xFF
    return bytes(b)


def test_reference_segments_cover_three_modes():
    modes = set()
    for s in REF_SEGMENTS:
        col, _, _ = reference_segment(s)
        modes |= set(O.bp_group_modes(col))
    assert modes == {"for", "delta_for", "constant_delta"}
    assert {s["dtype"] for s in REF_SEGMENTS} == {"int32", "int64"}


@pytest.mark.parametrize("s", REF_SEGMENTS, ids=[s["name"] for s in REF_SEGMENTS])
def test_decode_of_duckdb_written_segment(s):
    """The restatement's scan (BitpackingScanPartial, bitpacking.cpp:779-868) reads each segment
    DuckDB wrote back to the values the reference's table definitions give (NULL rows aside)."""
    col, values, valid = reference_segment(s)
    got = O.bp_decode(col)
    assert np.array_equal(got[valid], values[valid])


@pytest.mark.parametrize("s", REF_SEGMENTS, ids=[s["name"] for s in REF_SEGMENTS])
def test_compressor_writes_duckdbs_bytes(s):
    """The restatement's writer (BitpackingCompressState, bitpacking.cpp:375-540) given the same
    values and NULLs produces the same segment, byte for byte — header, group fields, packed
    bits of every value, metadata words — up to the left-over bits DuckDB packs past the last
    value of a 32-value block."""
    col, values, valid = reference_segment(s)
    ours = O.bp_compress(values, None if valid.all() else valid.astype(np.uint8), "auto")
    assert ours is not None and len(ours.seg_off) == 1
    ref = bytes.fromhex(s["segment_hex"])
    mine = bytes(ours.data[: int(ours.seg_size[0])])
    tsize = np.dtype(s["dtype"]).itemsize
    assert len(mine) == len(ref)
    assert packed_tail_masked(mine, tsize, s["count"]) == packed_tail_masked(ref, tsize, s["count"])
