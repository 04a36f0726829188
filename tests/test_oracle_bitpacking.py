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
