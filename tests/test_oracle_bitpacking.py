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
    """A FOR / DELTA_FOR segment with the packed bits of its last group past the segment's last
    value zeroed: DuckDB packs whole 32-value blocks from a reused buffer, so those bits are
    left-overs, not data."""
    b = bytearray(seg)
    end = int.from_bytes(b[:8], "little")
    last = (count - 1) // 2048  # metadata words are read downward from `end`, one per group
    meta = int.from_bytes(b[end - 4 * (last + 1):end - 4 * last], "little")
    mode, off = meta >> 24, meta & 0xFFFFFF
    count -= 2048 * last  # values of the last group
    if mode not in (4, 5):
        return bytes(b)
    fields = 3 if mode == 4 else 2  # DELTA_FOR: FOR, width, delta offset; FOR: FOR, width
    width = int.from_bytes(b[off + tsize: off + 2 * tsize], "little", signed=True)
    packed = off + fields * tsize
    blocks = (count + 31) // 32
    for bit in range(count * width, blocks * 32 * width):
        b[packed + bit // 8] &= ~(1 << (bit % 8)) & 0xFF
    # and the alignment gap between the last group's data and the metadata words (FlushSegment
    # moves the metadata down to the data's aligned end; the gap keeps what the buffer held)
    data_end = packed + blocks * 32 * width // 8
    b[data_end:end - 4 * (last + 1)] = bytes(max(0, end - 4 * (last + 1) - data_end))
    return bytes(b)


def test_reference_segments_cover_three_modes():
    modes = set()
    for s in REF_SEGMENTS:
        col, _, _ = reference_segment(s)
        modes |= set(O.bp_group_modes(col))
    assert modes == {"for", "delta_for", "constant_delta"}
    assert {s["dtype"] for s in REF_SEGMENTS} == {"int32", "int64", "uint64"}


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


# ---------------------------------------------------------------- every integral type

INT_DTYPES = [np.int8, np.int16, np.int32, np.int64, np.uint8, np.uint16, np.uint32, np.uint64]
FORCED = ["delta_for", "for", "constant_delta", "constant"]


def bitwidth_tables(bits):
    """The three tables of test/sql/storage/compression/bitpacking/bitpacking_bitwidths.test_slow
    (:19, :43, :67) for one type size: 2**(i//2048) as UINT<bits> and -(2**(i//2048)) as
    INT<bits> over bits·2048 rows, 2**(i//2048) as INT<bits> over (bits-1)·2048 rows."""
    k = np.arange(bits * 2048) // 2048
    unsigned = np.array([1 << int(x) for x in k], dtype=object).astype(f"uint{bits}")
    neg = np.array([-(1 << int(x)) for x in k], dtype=object).astype(f"int{bits}")
    pos = np.array([1 << int(x) for x in k[: (bits - 1) * 2048]], dtype=object).astype(f"int{bits}")
    return {"test_unsigned": unsigned, "test_signed_neg": neg, "test_signed_pos": pos}


@pytest.mark.parametrize("mode", FORCED)
@pytest.mark.parametrize("bits", [8, 16, 32, 64])
def test_bitwidths_reference_case(bits, mode):
    """bitpacking_bitwidths.test_slow under each forced mode: every table reads back bits (or
    bits - 1) distinct values, 2,048 rows each, each distinct value twice the one before
    (`i // lag(i)` = 2). The groups line up with the 2,048-row runs, so each is one value: a
    forced CONSTANT / CONSTANT_DELTA writes it as such, FOR and DELTA_FOR as FOR of width 0
    (DELTA_FOR's delta width 0 is not below the value width 0, bitpacking.cpp:258-261)."""
    for name, v in bitwidth_tables(bits).items():
        c = O.bp_compress(v, None, mode)
        assert c is not None, (name, mode)
        d = O.bp_decode(c)
        assert d.dtype == v.dtype and np.array_equal(d, v), (name, mode)
        vals, counts = np.unique(d, return_counts=True)
        assert len(vals) == (bits - 1 if name == "test_signed_pos" else bits)
        assert set(counts.tolist()) == {2048}
        if name != "test_signed_neg":
            assert all(int(b) // int(a) == 2 for a, b in zip(vals[:-1], vals[1:]))
        # per group: a forced CONSTANT / CONSTANT_DELTA as such — but an unsigned value above T_S's
        # maximum never delta-encodes (bitpacking.cpp:155-160), so that group falls to FOR
        firsts = v[::2048]
        above = (firsts.astype(np.uint64) > np.uint64(2 ** (bits - 1) - 1)) if v.dtype.kind == "u" else \
            np.zeros(len(firsts), bool)
        want = [{"constant": "constant", "constant_delta": "for" if a else "constant_delta"}.get(mode, "for")
                for a in above]
        assert O.bp_group_modes(c) == want, (name, mode)


@pytest.mark.parametrize("mode", FORCED)
@pytest.mark.parametrize("dtype", INT_DTYPES + [np.bool_])
def test_nullpack_reference_case(dtype, mode):
    """bitpacking_bitwidths.test_slow:101-117: CAST((i//3000)%2 AS <integral type> | BOOL) over
    12,000 rows → AVG 0.5 (BOOL is packed as int8_t, bitpacking.cpp:955-957)."""
    v = ((np.arange(12000) // 3000) % 2).astype(np.int8 if dtype is np.bool_ else dtype)
    c = O.bp_compress(v, None, mode)
    assert c is not None
    assert O.bp_decode(c).astype(np.int64).mean() == 0.5


@pytest.mark.parametrize("mode", FORCED)
def test_nulls_reference_case(mode):
    """bitpacking_nulls.test: a BIGINT column of three 10,000-row inserts (1337, i, i//2) with
    every fifth row NULL → sum 70,694,000, min 0, max 9,999, under each forced mode."""
    i = np.arange(10000, dtype=np.int64)
    v = np.concatenate([np.full(10000, 1337, np.int64), i, i // 2])
    valid = np.tile(i % 5 != 0, 3)
    c = O.bp_compress(v, valid.astype(np.uint8), mode)
    assert c is not None
    d = O.bp_decode(c)[valid]
    assert (int(d.sum()), int(d.min()), int(d.max())) == (70694000, 0, 9999)


@pytest.mark.parametrize("mode", FORCED)
def test_delta_full_range_reference_case(mode):
    """bitpacking_delta.test_slow: UBIGINT alternating 0 and 18446744073709551615 over 1 M rows
    stays BITPACKING under every forced mode (no delta above T_S's maximum: FOR of width 64,
    bitpacking.cpp:155-160) and reads back 500,000 of each."""
    v = np.where(np.arange(1_000_000) % 2 == 0, np.uint64(0), np.uint64(2 ** 64 - 1)).astype(np.uint64)
    c = O.bp_compress(v, None, mode)
    assert c is not None
    d = O.bp_decode(c)
    vals, counts = np.unique(d, return_counts=True)
    assert vals.tolist() == [0, 2 ** 64 - 1] and counts.tolist() == [500000, 500000]
    assert set(O.bp_group_modes(c)) == {"for"}


def filter_pushdown_column():
    """bitpacking_filter_pushdown.test:24-30: INTEGER col = range(10000), 1337 × 10,000,
    range(30000, 40000); id = the row's source integer."""
    col = np.concatenate([np.arange(10000), np.full(10000, 1337), np.arange(30000, 40000)]).astype(np.int32)
    ids = np.concatenate([np.arange(10000), np.arange(20000, 30000), np.arange(30000, 40000)]).astype(np.int64)
    return col, ids


@pytest.mark.parametrize("mode", ["auto"] + FORCED)
def test_filter_pushdown_reference_case(mode):
    """bitpacking_filter_pushdown.test: WHERE col = 1337 → SUM 13371337, MIN = MAX = 1337,
    COUNT 10001; WHERE id = 5000 → col 5000, one row; under AUTO and each forced mode."""
    from cubit_amd import filters as F

    col, ids = filter_pushdown_column()
    c = O.bp_compress(col, None, mode)
    assert c is not None
    d = O.bp_decode(c)
    assert np.array_equal(d, col)
    fs = F.TableFilterSet({0: F.ConstantFilter("=", 1337)})
    rows = O.table_scan([O.Column(d)], F.serialize(fs), len(d))
    got = d[rows]
    assert (int(got.sum()), int(got.min()), int(got.max()), len(got)) == (13371337, 1337, 1337, 10001)
    fs = F.TableFilterSet({1: F.ConstantFilter("=", 5000)})
    rows = O.table_scan([O.Column(d), O.Column(ids)], F.serialize(fs), len(d))
    assert d[rows].tolist() == [5000]


def typed_case(dtype, mode, n=2048 * 7 + 1001, below_2_63=False):
    """Values of one integral type — the type's extremes, a run of one value, a constant step, a
    descending sorted stretch (negative deltas: a DELTA_FOR frame below zero, T's wrap-around in
    the unsigned types), values next to the minimum, NULLs, an all-NULL group where the mode
    allows one, a partial last group — and their segments under force_bitpacking_mode `mode`.
    below_2_63: UBIGINT values stay below 2^63 (an INT64 column can hold them)."""
    rng = np.random.default_rng(abs(hash((np.dtype(dtype).name, mode, below_2_63))) % 2 ** 32)
    info = np.iinfo(dtype)
    # random groups over half the type's span (a signed group whose max - min overflows T is
    # not bitpackable at all: the reference picks another compression), the unsigned ones over
    # all of it (width 64 for UBIGINT)
    lo, hi = (info.min // 2, info.max // 2) if info.min < 0 else (info.min, info.max)
    if below_2_63:
        hi = 2 ** 63 - 1
    v = rng.integers(lo, hi, n, dtype=dtype, endpoint=True)
    v[:2048] = hi                                                             # one value
    step = 3 if info.bits >= 16 else 0  # 2,048 distinct 8-bit values do not exist
    v[2048:4096] = (np.arange(2048) * step + 1).astype(dtype)                 # constant delta
    v[4096:6144] = np.sort(rng.integers(lo, min(hi, info.max // 2), 2048, dtype=dtype))[::-1]  # descending
    v[6144:8192] = info.min + rng.integers(0, 7, 2048).astype(dtype)         # next to the minimum
    valid = rng.random(n) > 0.05
    valid[:6144] = True                                                       # the delta groups need all-valid
    if mode in ("auto", "constant"):
        # an all-NULL group is CONSTANT; under the other forced modes it is not bitpackable at
        # all (max - min of an empty group overflows T, bitpacking.cpp:149-151, 231-234)
        valid[10240:12288] = False
    c = O.bp_compress(v, valid.astype(np.uint8), mode)
    assert c is not None, (np.dtype(dtype).name, mode)
    return v, valid, c


@pytest.mark.parametrize("mode", ["auto"] + FORCED)
@pytest.mark.parametrize("dtype", INT_DTYPES)
def test_every_type_round_trips(dtype, mode):
    """Every integral type DuckDB bit-packs through the writer and back (typed_case)."""
    v, valid, c = typed_case(dtype, mode)
    d = O.bp_decode(c)
    assert d.dtype == np.dtype(dtype)
    assert np.array_equal(d[valid], v[valid])
    if mode == "auto":
        assert {"constant", "for"} <= set(O.bp_group_modes(c))


@pytest.mark.parametrize("mode", ["for", "delta_for", "constant_delta"])
def test_all_null_group_is_not_bitpackable_under_forced_modes(mode):
    """A forced FOR / DELTA_FOR / CONSTANT_DELTA cannot write an all-NULL group (its max - min
    overflows T and it has no deltas): Flush fails and the reference picks another compression."""
    v = np.zeros(4096, np.int32)
    valid = np.ones(4096, np.uint8)
    valid[2048:] = 0
    assert O.bp_compress(v, valid, mode) is None
    assert O.bp_compress(v, valid, "auto") is not None


# ---------------------------------------------------------------- FTS index segments (wider FOR groups)

FTS = json.loads((Path(__file__).resolve().parent / "golden" / "bitpacking_reference_segments_fts.json").read_text())
FTS_BP = [s for s in FTS["segments"] if s["compression"] == "bitpacking"]


def fts_segment(s):
    """A fixture segment of bitpacking_reference_segments_fts.json as a one-segment BitpackedColumn."""
    raw = np.frombuffer(bytes.fromhex(s["segment_hex"]), dtype=np.uint8)
    data = np.zeros((len(raw) + 7) // 8 * 8 + 8, dtype=np.uint8)
    data[: len(raw)] = raw
    return O.BitpackedColumn(data, np.array([0], np.uint64), np.array([len(raw)], np.uint64),
                             np.array([s["count"]], np.uint64), np.dtype(s["dtype"]))


def rle_decode(s):
    """An RLE segment of BIGINTs (src/storage/compression/rle.cpp:248-277, RLEScanState: the
    8-byte header is the offset of the uint16 run lengths; the run values start at byte 8)."""
    seg = bytes.fromhex(s["segment_hex"])
    off = int.from_bytes(seg[:8], "little")
    n_runs = (len(seg) - off) // 2
    vals = np.frombuffer(seg[8:8 + 8 * n_runs], dtype="<i8")
    runs = np.frombuffer(seg[off:off + 2 * n_runs], dtype="<u2")
    out = np.repeat(vals, runs)
    assert len(out) == s["count"]
    return out


def fts_decoded():
    """Every FTS column: BITPACKING ones by the restatement, RLE ones by rle_decode."""
    return {s["name"]: (O.bp_decode(fts_segment(s)) if s["compression"] == "bitpacking" else rle_decode(s))
            for s in FTS["segments"]}


def check_fts_invariants(cols):
    """fts_indexing.cpp:83-149 over the decoded columns (see the fixture's `invariants`)."""
    docid, termid = cols["terms.docid"], cols["terms.termid"]
    assert np.array_equal(cols["docs.len"], np.bincount(docid, minlength=153))
    assert np.array_equal(np.unique(termid), np.arange(1558))
    pairs = np.unique(termid.astype(np.int64) * 1024 + docid)
    assert np.array_equal(cols["dict.df"], np.bincount(pairs // 1024, minlength=1558))
    assert abs(cols["docs.len"].sum() / 153 - FTS["stats_avgdl"]) < 1e-9


def test_fts_segments_widths_and_modes():
    """The FTS file adds FOR groups of 7, 8 and 11 bits (the storage_version.db segments are at
    most 3 bits wide) and CONSTANT_DELTA groups, all with an 8-byte T."""
    modes, widths = set(), set()
    for s in FTS_BP:
        seg = bytes.fromhex(s["segment_hex"])
        end = int.from_bytes(seg[:8], "little")
        for g in range((s["count"] + 2047) // 2048):
            meta = int.from_bytes(seg[end - 4 * (g + 1):end - 4 * g], "little")
            mode, off = meta >> 24, meta & 0xFFFFFF
            modes.add(mode)
            if mode == 5:  # FOR: frame of reference, then the width (T-sized fields)
                widths.add(int.from_bytes(seg[off + 8:off + 16], "little", signed=True))
    assert modes == {3, 5}  # CONSTANT_DELTA, FOR (bitpacking.cpp BitpackingMode)
    assert {7, 8, 11} <= widths


@pytest.mark.parametrize("s", FTS_BP, ids=[s["name"] for s in FTS_BP])
def test_fts_segment_decodes_to_its_definition_and_statistics(s):
    """Each segment decodes to the values the FTS definitions give where they fix them
    (CONSTANT_DELTA columns; docs.len from the RLE column terms.docid) and to the minimum and
    maximum its DataPointer stores."""
    got = O.bp_decode(fts_segment(s))
    assert int(got.min()) == s["statistics"]["min"] and int(got.max()) == s["statistics"]["max"]
    vals = s["values"]
    if isinstance(vals, dict):
        vals = list(range(*vals["range"]))
    if vals is not None:
        assert got.tolist() == vals


def test_fts_columns_satisfy_the_index_definitions():
    """docs.len = terms per doc, dict.df = distinct docs per term, every termid present,
    Σ len / 153 = stats.avgdl — over the restatement's decode of the FOR segments."""
    check_fts_invariants(fts_decoded())


@pytest.mark.parametrize("s", FTS_BP, ids=[s["name"] for s in FTS_BP])
def test_fts_compressor_writes_duckdbs_bytes(s):
    """The restatement's writer given the decoded values reproduces DuckDB's segment byte for
    byte, up to the left-over bits past the last value of a 32-value block."""
    got = O.bp_decode(fts_segment(s))
    ours = O.bp_compress(got, None, "auto")
    assert ours is not None and len(ours.seg_off) == 1
    ref = packed_tail_masked(bytes.fromhex(s["segment_hex"]), 8, s["count"])
    mine = packed_tail_masked(bytes(ours.data[: int(ours.seg_size[0])]), 8, s["count"])
    assert mine == ref
