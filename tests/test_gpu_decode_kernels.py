"""The three evaluate + decode kernels — pair-claimed (eval_decode_pairs), run-claimed
(eval_decode_runs) and look-back (eval_decode_lookback: one tile per workgroup, offsets from
the earlier tiles' published counts) — against the oracle's CPU bitmap evaluator, forced one at
a time through cubit_ctx_set_decode_kernel and under the automatic policy. At 140 M rows the
look-back grid (1,069 workgroups) exceeds what is co-resident, so its waits span workgroups
that start only after others finish. The look-back runs land in tile order, so its default
output is already the ascending array, and ordered scans take it up to 4,608 tiles.

The run-claimed kernel keeps decoding a workgroup's tiles into one LDS stage until the next
tile does not fit, so its interesting cases need workgroups that walk many tiles: tables of
more than 2 × 512 tiles of 131,072 rows (the production grid is two workgroups per CU), with
tiles of every kind — empty, sparse (many tiles per run, up to the 16-tile cap), around the
8,192-entry stage (runs of one or two tiles, switches on consecutive tiles) and dense (more
hits than a stage: the direct path). Row ids are compared bit-exactly, in tile-run order
through the directory and in the ordered layout, with a row base offset.
"""
import ctypes as C

import numpy as np
import pytest

from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.table import Context, CubitTable, padded_words, runs_in_row_order
from oracle import oracle as O

pytestmark = pytest.mark.gpu

TILE_WORDS = 2048  # 131,072 rows


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.set_decode_kernel(L.DECODE_AUTO)
    c.close()


def rand_words(rng, n, k):
    """AND of k random words: each bit set with probability 2^-k."""
    w = rng.integers(0, 2 ** 64, n, dtype=np.uint64)
    for _ in range(k - 1):
        w &= rng.integers(0, 2 ** 64, n, dtype=np.uint64)
    return w


def shaped_leaf(rng, n_rows):
    """A leaf whose tiles differ: empty, 1/128, 1/16 (≈ one stage), all ones (dense)."""
    nw = (n_rows + 63) // 64
    tiles = (nw + TILE_WORDS - 1) // TILE_WORDS
    kinds = rng.choice(4, size=tiles, p=[0.15, 0.55, 0.2, 0.1])
    w = np.zeros(nw, dtype=np.uint64)
    sparse = rand_words(rng, nw, 7)
    mid = rand_words(rng, nw, 4)
    for t, k in enumerate(kinds):
        sl = slice(t * TILE_WORDS, min(nw, (t + 1) * TILE_WORDS))
        if k == 1:
            w[sl] = sparse[sl]
        elif k == 2:
            w[sl] = mid[sl]
        elif k == 3:
            w[sl] = ~np.uint64(0)
    if n_rows & 63:
        w[-1] &= np.uint64((1 << (n_rows & 63)) - 1)
    return w


def run_program(ctx, dleaves, k, neg, prog, n, base, out, cnt, ordered):
    ptrs = (C.c_void_p * k)(*[d.ptr.value for d in dleaves[:k]])
    p = (C.c_int32 * len(prog))(*prog)
    L.check(ctx.lib.cubit_bitvector_eval(ctx.handle, ptrs, k, neg, p, len(prog), n, base, out.ptr, out.nbytes // 8,
                                         cnt.ptr, None, L.SCAN_ORDERED if ordered else 0))
    ctx.check()
    c = int(cnt.download(np.uint64, 1)[0])
    got = out.download(np.int64, c)
    if not ordered:
        d, _ = ctx.last_tiles()
        assert int(d[:, 1].sum()) == c
        got = runs_in_row_order(got, d)
    return got


@pytest.mark.parametrize("n", [1_000_003, 100_000_000, 140_000_001])
def test_pairs_and_runs_match_oracle(ctx, n):
    rng = np.random.default_rng(n % 1000)
    pw = padded_words(n)
    nw = (n + 63) // 64
    # leaf 0 shapes the tiles, the others are 1/2-density noise (so a CONJ of k leaves keeps
    # ≈ 2^-(k-1) of leaf 0's rows), leaf 5 is sparse everywhere (for ORs)
    host = [shaped_leaf(rng, n)] + [rand_words(rng, nw, 1) for _ in range(4)] + [rand_words(rng, nw, 8)]
    for w in host[1:]:
        if n & 63:
            w[-1] &= np.uint64((1 << (n & 63)) - 1)
    dleaves = [ctx.upload(np.concatenate([w, np.zeros(pw - nw, dtype=np.uint64)])) for w in host]
    out = ctx.alloc(max(n // 2, 1024) * 8)
    cnt = ctx.alloc(16)
    programs = [  # (k, negate mask, postfix program)
        (1, 0, [0]),
        (2, 0, [0, 1, L.OP_AND]),
        (2, 0b10, [0, 1, L.OP_AND]),
        (3, 0b100, [0, 1, L.OP_AND, 2, L.OP_AND]),
        (4, 0, [0, 1, L.OP_AND, 2, L.OP_AND, 3, L.OP_AND]),
        (5, 0b01010, [0, 1, L.OP_AND, 2, L.OP_AND, 3, L.OP_AND, 4, L.OP_AND]),
        (6, 0, [0, 1, L.OP_AND, 2, 3, L.OP_AND, L.OP_AND, 4, 5, L.OP_AND, L.OP_OR]),  # DNF-ish with a sparse OR arm
    ]
    for i, (k, neg, prog) in enumerate(programs):
        ol = [(~host[j] if (neg >> j) & 1 else host[j]) for j in range(k)]
        if neg and n & 63:
            for j in range(k):
                if (neg >> j) & 1:
                    ol[j] = ol[j].copy()
                    ol[j][-1] &= np.uint64((1 << (n & 63)) - 1)
        ref, _ = O.bitmap_eval(ol, prog, n, 1_000_000_007)
        assert len(ref) <= out.nbytes // 8
        for kernel in (L.DECODE_PAIRS, L.DECODE_RUNS, L.DECODE_LOOKBACK, L.DECODE_AUTO):
            ctx.set_decode_kernel(kernel)
            for ordered in (False, True):
                got = run_program(ctx, dleaves, k, neg, prog, n, 1_000_000_007, out, cnt, ordered)
                assert np.array_equal(got, ref), (kernel, ordered, k, neg, prog)
                if ctx.last_decode_kernel() == L.DECODE_LOOKBACK:
                    assert np.array_equal(out.download(np.int64, len(ref)), ref), (kernel, ordered)
    ctx.set_decode_kernel(L.DECODE_AUTO)


def test_auto_policy_large_table_scan(ctx):
    """A 140 M-row table, K = 1..3 filters (the run-claimed kernel under the automatic policy):
    every row id equals numpy's evaluation of the same predicate."""
    rng = np.random.default_rng(4)
    n = 140_000_001
    a = rng.integers(0, 10_000, n, dtype=np.int32)
    b = rng.integers(0, 100, n, dtype=np.int32)
    t = CubitTable(ctx, n, row_base=77)
    t.add_column(0, a)
    t.add_column(1, b)
    t.build_index(0, L.INDEX_RANGE, [50, 100, 5_000])
    t.build_index(1, L.INDEX_RANGE)
    cases = [
        (F.TableFilterSet({0: F.ConstantFilter("<", 100)}), a < 100),
        (F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", 50), F.ConstantFilter("<", 100)])}),
         (a >= 50) & (a < 100)),
        (F.TableFilterSet({0: F.ConstantFilter("<", 5_000), 1: F.ConstantFilter("=", 42)}), (a < 5_000) & (b == 42)),
    ]
    for fs, mask in cases:
        ref = np.flatnonzero(mask).astype(np.int64) + 77
        for ordered in (False, True):
            got = t.scan(fs, ordered=ordered)
            if not ordered:
                d, _ = ctx.last_tiles()
                got = runs_in_row_order(got, d)
            assert np.array_equal(got, ref)
        assert t.count(fs) == len(ref)
    t.close()


def test_repeated_launch_timing_keeps_results(ctx):
    """cubit_ctx_set_repeat (the bench's kernel timing): the next decode is launched `reps` times
    back to back between two stream events; each repeat rewrites the same outputs from the same
    inputs (the look-back under a new epoch each time), so the row ids equal the oracle's."""
    rng = np.random.default_rng(9)
    n = 100_000_000
    pw, nw = padded_words(n), (n + 63) // 64
    host = [shaped_leaf(rng, n), rand_words(rng, nw, 1)]  # n is a multiple of 64: no tail mask
    dleaves = [ctx.upload(np.concatenate([w, np.zeros(pw - nw, dtype=np.uint64)])) for w in host]
    out = ctx.alloc(n // 2 * 8)
    cnt = ctx.alloc(16)
    prog = [0, 1, L.OP_AND]
    ref, _ = O.bitmap_eval(host, prog, n, 5)
    with pytest.raises(L.CubitError):
        ctx.repeat_time()  # nothing repeated yet on this context
    for kernel in (L.DECODE_PAIRS, L.DECODE_RUNS, L.DECODE_LOOKBACK):
        ctx.set_decode_kernel(kernel)
        for ordered in (False, True):
            ctx.set_repeat(7)
            got = run_program(ctx, dleaves, 2, 0, prog, n, 5, out, cnt, ordered)
            assert np.array_equal(got, ref), (kernel, ordered)
            ms, launches = ctx.repeat_time()
            assert launches == 7 and 0 < ms < 10
            # disarmed after one decode: the next call launches once
            assert np.array_equal(run_program(ctx, dleaves, 2, 0, prog, n, 5, out, cnt, ordered), ref)
    ctx.set_decode_kernel(L.DECODE_AUTO)


def test_ordered_scan_past_the_old_lookback_limit(ctx):
    """540 M rows = 4,120 tiles: CUBIT_SCAN_ORDERED under AUTO takes the look-back decode (no
    ordering pass) at a size where the unordered scan takes the run-claimed kernel; both equal
    the oracle."""
    rng = np.random.default_rng(11)
    n = 540_000_001
    pw, nw = padded_words(n), (n + 63) // 64
    host = [shaped_leaf(rng, n), rand_words(rng, nw, 1)]
    host[1][-1] &= np.uint64((1 << (n & 63)) - 1)
    dleaves = [ctx.upload(np.concatenate([w, np.zeros(pw - nw, dtype=np.uint64)])) for w in host]
    prog = [0, 1, L.OP_AND]
    ref, _ = O.bitmap_eval(host, prog, n, 3)
    out = ctx.alloc((len(ref) + 1024) * 8)
    cnt = ctx.alloc(16)
    ctx.set_decode_kernel(L.DECODE_AUTO)
    got = run_program(ctx, dleaves, 2, 0, prog, n, 3, out, cnt, True)
    assert ctx.last_decode_kernel() == L.DECODE_LOOKBACK
    assert np.array_equal(got, ref)
    got = run_program(ctx, dleaves, 2, 0, prog, n, 3, out, cnt, False)
    assert ctx.last_decode_kernel() == L.DECODE_RUNS
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("n", [1_000_003, 100_000_000, 140_000_001])
def test_lookback_expiry_recounts_and_stays_exact(ctx, n):
    """The look-back's bounded wait: with a spin limit of 1 poll almost every workgroup finds some
    earlier flag unpublished and counts that tile from its bitvectors itself. Row ids and count
    must still equal the oracle's, in row order, for plain, negated and OR programs — the kernel
    has no failure exit (it used to write count = ~0 and drop its run)."""
    rng = np.random.default_rng(n % 997)
    pw, nw = padded_words(n), (n + 63) // 64
    host = [shaped_leaf(rng, n), rand_words(rng, nw, 1), rand_words(rng, nw, 8)]
    for w in host[1:]:
        if n & 63:
            w[-1] &= np.uint64((1 << (n & 63)) - 1)
    dleaves = [ctx.upload(np.concatenate([w, np.zeros(pw - nw, dtype=np.uint64)])) for w in host]
    out = ctx.alloc(max(n // 2, 1024) * 8)
    cnt = ctx.alloc(16)
    ctx.set_decode_kernel(L.DECODE_LOOKBACK)
    try:
        for spins in (1, 3):
            ctx.set_lookback_spins(spins)
            for k, neg, prog in [(1, 0, [0]), (2, 0b10, [0, 1, L.OP_AND]),
                                 (3, 0, [0, 1, L.OP_AND, 2, L.OP_OR])]:
                ol = [(~host[j] if (neg >> j) & 1 else host[j]) for j in range(k)]
                if neg and n & 63:
                    for j in range(k):
                        if (neg >> j) & 1:
                            ol[j] = ol[j].copy()
                            ol[j][-1] &= np.uint64((1 << (n & 63)) - 1)
                ref, _ = O.bitmap_eval(ol, prog, n, 11)
                got = run_program(ctx, dleaves, k, neg, prog, n, 11, out, cnt, True)
                assert ctx.last_decode_kernel() == L.DECODE_LOOKBACK
                assert np.array_equal(got, ref), (spins, k, neg, prog)
    finally:
        ctx.set_lookback_spins(0)
        ctx.set_decode_kernel(L.DECODE_AUTO)


def test_lookback_expiry_with_zonemap_skip(ctx):
    """The expiry recount follows the live-tile list (zonemap skip): a clustered column whose
    filter keeps a few zones, scanned ordered with a spin limit of 1, equals numpy."""
    n = 50_000_000
    a = (np.arange(n, dtype=np.int64) // 1000).astype(np.int32)  # ascending: zones skip
    t = CubitTable(ctx, n, row_base=5)
    t.add_column(0, a)
    t.build_index(0, L.INDEX_RANGE, [1000, 20000, 30000, 45000])
    fs = F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", 20000), F.ConstantFilter("<", 30000)])})
    ref = np.flatnonzero((a >= 20000) & (a < 30000)).astype(np.int64) + 5
    ctx.set_lookback_spins(1)
    try:
        got = t.scan(fs, ordered=True)
        assert np.array_equal(got, ref)
        ev, zones = t.last_zones()
        assert ev < zones
    finally:
        ctx.set_lookback_spins(0)
        t.close()


def test_single_index_leaf_decodes_from_tile_counts(ctx):
    """A filter answered by one index bitvector as it stands (v < c on an edge of a range index)
    decodes with its per-tile offsets known up front — the bitvector's per-zone counts, kept
    with its zone map — by the look-back kernel without its walk, at any size (here 1,526 tiles,
    twice the co-resident grid the walk needs). Rows equal numpy in
    tile-run and ordered output, with zones skipped, and stay equal after an append changes the
    bitvector (its counts are dropped with the zone map)."""
    rng = np.random.default_rng(17)
    n = 200_000_003
    a = rng.integers(0, 1_000_000, n).astype(np.int32)
    a[50_000_000:90_000_000] = 999_999  # zones where the leaf is empty: a live-tile list
    t = CubitTable(ctx, n, row_base=9)
    t.add_column(0, a)
    t.build_index(0, L.INDEX_RANGE, [10_000, 500_000])
    fs = F.TableFilterSet({0: F.ConstantFilter("<", 10_000)})
    ctx.set_decode_kernel(L.DECODE_AUTO)

    def check(vals):
        ref = np.flatnonzero(vals < 10_000).astype(np.int64) + 9
        for ordered in (False, True):
            got = t.scan(fs, ordered=ordered)
            assert ctx.last_decode_kernel() == L.DECODE_PREFIXED, ordered
            if not ordered:
                d, _ = ctx.last_tiles()
                got = runs_in_row_order(got, d)
            assert np.array_equal(got, ref), ordered
        assert t.last_zones()[0] < t.last_zones()[1]  # the zonemap skipped zones
        # a complemented leaf (v >= c: NOT L(c) within the valid rows) is not one bitvector as
        # it stands: the decode takes the usual kernels and still equals numpy
        ge = F.TableFilterSet({0: F.ConstantFilter(">=", 10_000)})
        assert t.count(ge) == int((vals >= 10_000).sum())

    check(a)
    extra = rng.integers(0, 20_000, 3_000_000).astype(np.int32)
    t.append({0: extra})
    check(np.concatenate([a, extra]))  # dense tiles at the end: the stage rounds
    t.close()


def test_row_ids_past_2_32(ctx):
    """A partition of 2^32 + 4,097 rows (32,769 tiles, two 537 MB leaves): row ids and tile
    offsets past 32 bits, under every decode kernel (the look-back only where the policy lets
    it run), in tile-run and ordered output, bit-exact against the oracle — the largest
    partition one SF300 GPU holds is 1.8 G rows; this is 2.4× that."""
    n = (1 << 32) + 4097
    rng = np.random.default_rng(32)
    nw = (n + 63) // 64
    pw = padded_words(n)
    host = [rand_words(rng, nw, 8), rand_words(rng, nw, 1)]
    for w in host:
        w[-1] &= np.uint64((1 << (n & 63)) - 1)
    host[0][-TILE_WORDS:] |= rand_words(rng, TILE_WORDS, 2)  # a denser last tile, ending mid-word
    host[0][-1] &= np.uint64((1 << (n & 63)) - 1)
    dleaves = [ctx.upload(np.concatenate([w, np.zeros(pw - nw, dtype=np.uint64)])) for w in host]
    base = 3
    ref, _ = O.bitmap_eval(host, [0, 1, L.OP_AND], n, base)
    assert ref[-1] >= 1 << 32
    out = ctx.alloc(len(ref) * 8 + 1024)
    cnt = ctx.alloc(16)
    for kernel in (L.DECODE_PAIRS, L.DECODE_RUNS, L.DECODE_LOOKBACK, L.DECODE_AUTO):
        ctx.set_decode_kernel(kernel)
        for ordered in (False, True):
            got = run_program(ctx, dleaves, 2, 0, [0, 1, L.OP_AND], n, base, out, cnt, ordered)
            assert np.array_equal(got, ref), (kernel, ordered)
    ctx.set_decode_kernel(L.DECODE_AUTO)
    for d in dleaves + [out, cnt]:
        d.free()
