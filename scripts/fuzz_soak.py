#!/usr/bin/env python3
"""Planner soak (development tool): the GPU planner fuzz of tests/test_gpu_planner_fuzz.py at
a larger size and for a fixed wall-clock budget, with fresh seeds — random pushed
TableFilterSets and residual AND/OR trees over range / equality / edge-keyed range + bins /
unindexed columns with NULLs, deletes visible to a snapshot and, in every other round,
updates from a writer; each scan under a random decode kernel (AUTO, pair-claimed, run-claimed,
look-back); every third table holds the typed columns instead (DOUBLE / FLOAT with NaN and ±0,
VARCHAR dictionary codes, full-range UBIGINT, HUGEINT over 16-byte order keys:
tests/test_gpu_typed_fuzz.py). Every result is
compared with the oracle; every third filter also runs through the
table function (random projection with the row id, 1-4 pipeline tasks, staged or per-window
copies): row ids, values and NULL-ness against the oracle's scan and fetch. Prints one summary
line.

  python scripts/fuzz_soak.py [seconds] [rows] [first seed]
"""
import os
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "duckdb-cubit_amd"), str(ROOT), str(ROOT / "tests")]

from cubit_amd import _lib as L  # noqa: E402
from cubit_amd import filters as F  # noqa: E402
from cubit_amd.datagen import validity_from_mask  # noqa: E402
from cubit_amd.scan_function import ROW_ID, CubitScanFunction  # noqa: E402
from cubit_amd.table import Context, CubitTable  # noqa: E402
from oracle import oracle as O  # noqa: E402
from test_gpu_planner_fuzz import TXN_START, rand_const_filter, rand_residual  # noqa: E402
from test_gpu_typed_fuzz import typed_round  # noqa: E402


def table_function_check(t, rng, fs, residual, txn, ref, ocols, row_base, tx, label):
    """The scan through the table-function callbacks: the emitted storage columns' values and
    NULL-ness and the row ids, against the oracle (row ids: its scan; values: its fetch)."""
    keep = [int(c) for c in rng.permutation(4)[: int(rng.integers(0, 5))]]
    column_ids = [0, 1, 2, 3, ROW_ID]
    projection = [4] + keep
    if rng.random() < 0.5:
        os.environ["CUBIT_SCAN_STAGE_MB"] = "0"  # per-window copies
    else:
        os.environ.pop("CUBIT_SCAN_STAGE_MB", None)
    fn = CubitScanFunction(t, column_ids, projection, fs, residual, txn=txn)
    parts, lock = [], threading.Lock()

    def task():
        local = fn.init_local()
        while True:
            vals, masks = fn.function_validity(local)
            if len(vals[0]) == 0:
                return
            with lock:
                parts.append((vals, masks))

    th = [threading.Thread(target=task) for _ in range(int(rng.integers(1, 5)))]
    for x in th:
        x.start()
    for x in th:
        x.join()
    fn.close()
    os.environ.pop("CUBIT_SCAN_STAGE_MB", None)
    if not parts:
        if len(ref):
            raise AssertionError(f"{label}: table function returned no rows, oracle {len(ref)}")
        return
    ids = np.concatenate([p[0][0] for p in parts])
    o = np.argsort(ids, kind="stable")
    if not np.array_equal(ids[o], ref):
        raise AssertionError(f"{label}: table function rows {len(ids)} vs {len(ref)}")
    for k, c in enumerate(keep, start=1):
        vals = np.concatenate([p[0][k] for p in parts])[o]
        valid = np.concatenate([p[1][k] for p in parts])[o]
        rv, rvalid = O.fetch(ocols[c], ref, row_base=row_base, tx=tx, with_valid=True)
        if not (np.array_equal(valid, rvalid) and np.array_equal(vals[valid], rv[rvalid].astype(np.int64))):
            raise AssertionError(f"{label}: table function column {c} differs from the oracle's fetch")


def round_(ctx, seed, n, with_updates):
    rng = np.random.default_rng(seed)
    row_base = int(rng.integers(0, 1 << 40))
    t = CubitTable(ctx, n, row_base=row_base)
    data = []
    for c in range(4):
        d = rng.integers(0, 50, n).astype(np.int32 if c % 2 == 0 else np.int64)
        valid = rng.random(n) > (0.12 if c != 1 else 0.0)
        vw = validity_from_mask(valid) if c != 1 else None
        if c == 3:
            # any integral type DuckDB holds, registered plain (widened on the device), as
            # BITPACKING segments under a random forced mode (the packed filter on or off), as
            # RLE segments, or as row groups of mixed codecs
            dt = np.dtype(rng.choice(["int8", "int16", "int32", "int64", "uint8", "uint16", "uint32", "uint64"]))
            typed = d.astype(dt)
            codec = rng.random()
            if codec < 0.15:
                # row groups of mixed codecs (UNCOMPRESSED, CONSTANT, RLE, BITPACKING) as DuckDB's
                # checkpoint picks them, through cubit_table_add_segment_column
                from test_gpu_segments import mixed_column

                typed, valid, segs = mixed_column(rng, dt, n // 122_880, n % 122_880)
                vw = validity_from_mask(valid)
                t.add_segment_column(c, segs, dt, vw)
            elif codec < 0.35:
                # RLE segments (the restated compressor over runs of 1-15 rows; runs long enough to
                # matter), expanded on the device
                m = n // 4 + 1
                typed = np.repeat(rng.integers(0, 50, m), rng.integers(1, 16, m))[:n].astype(dt)
                if len(typed) < n:
                    typed = np.concatenate([typed, np.zeros(n - len(typed), dt)])
                data_b, offs, rows = O.rle_compress(typed, valid)
                t.add_rle_column(c, data_b, offs, rows, dt, validity=vw)
            elif codec < 0.6:
                c3 = O.bp_compress(typed, valid.astype(np.uint8), str(rng.choice(["auto", "for", "delta_for"])))
                if c3 is None:
                    c3 = O.bp_compress(typed, valid.astype(np.uint8), "auto")
                t.add_bitpacked_column(c, c3.data, c3.seg_off, c3.seg_count, dt, validity=vw)
                t.use_packed_filter(bool(rng.random() < 0.5))
            else:
                t.add_column(c, typed, vw)
            # the oracle's view of the column: UBIGINT stays unsigned (its constants cross as bits, so
            # a negative constant is a value past 2^63 on both sides); the others as held (INT32 / INT64)
            d = typed if dt == np.uint64 else typed.astype(np.int32 if dt.itemsize <= 2 or dt == np.int32 else np.int64)
        else:
            t.add_column(c, d, vw)
        data.append((d, vw))
    t.build_index(0, L.INDEX_RANGE)
    t.build_index(1, L.INDEX_EQUALITY)
    t.build_index(2, L.INDEX_RANGE, [10, 20, 30, 40])
    t.build_index(2, L.INDEX_BINS, [0, 10, 20, 30, 40, 50])
    writer = TXN_START + 5
    upd = {}
    if with_updates:
        for c in (0, 2, 3):
            rows = np.sort(rng.choice(n, size=n // 100, replace=False)).astype(np.int64)
            vals = rng.integers(0, 50, len(rows)).astype(np.int64)
            vers = np.where(rng.random(len(rows)) < 0.5, np.uint64(3), np.uint64(writer)).astype(np.uint64)
            t.set_updates(c, rows, vals, vers)
            upd[c] = (rows, vals, vers)
    ocols = [O.Column(d, vw, updates=upd.get(c)) for c, (d, vw) in enumerate(data)]
    del_rows = np.sort(rng.choice(n, size=n // 20, replace=False)).astype(np.int64)
    del_ids = np.where(rng.random(len(del_rows)) < 0.5, np.uint64(4), np.uint64(writer)).astype(np.uint64)
    t.set_deletes(del_rows, del_ids)
    deleted = np.full(n, np.uint64(2 ** 64 - 2), dtype=np.uint64)
    deleted[del_rows] = del_ids
    views = [(2, writer), (2, TXN_START + 6), (10, TXN_START + 7)]
    checks = 0
    for i in range(30):
        filters = {int(c): rand_const_filter(rng) for c in rng.choice(4, size=rng.integers(0, 4), replace=False)}
        fs = F.TableFilterSet(filters)
        residual = rand_residual(rng, 4) if rng.random() < 0.5 else None
        plan = F.serialize(fs, residual)
        start, tid = views[i % 3]
        ref = O.table_scan(ocols, plan, n, row_base=row_base, tx=O.Mvcc(start, tid, deleted=deleted))
        # every decode kernel, not only the one AUTO picks at this size (results are identical)
        ctx.set_decode_kernel(int(rng.choice([L.DECODE_AUTO, L.DECODE_PAIRS, L.DECODE_RUNS, L.DECODE_LOOKBACK])))
        got = t.scan(fs, residual, txn=L.Txn(start, tid), ordered=bool(i % 2))
        if i % 2 == 0:
            got = np.sort(got)
        if not np.array_equal(got, ref):
            raise AssertionError(f"seed {seed} case {i}: {len(got)} vs {len(ref)} rows; {fs} {residual}")
        if residual is None:
            c = t.count(fs, txn=L.Txn(start, tid))
            if c != len(ref):
                raise AssertionError(f"seed {seed} case {i}: count {c} vs {len(ref)}")
        if i % 3 == 0:
            table_function_check(t, rng, fs, residual, L.Txn(start, tid), ref, ocols, row_base,
                                 O.Mvcc(start, tid, deleted=deleted), f"seed {seed} case {i}")
        checks += 1
    ctx.set_decode_kernel(L.DECODE_AUTO)
    t.close()
    return checks


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 90.0
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 2_000_003
    seed0 = int(sys.argv[3]) if len(sys.argv) > 3 else 10_000
    ctx = Context(0)
    t_end = time.perf_counter() + budget
    rounds = checks = 0
    seed = seed0
    while time.perf_counter() < t_end:
        if rounds % 3 == 2:  # FLOAT / DOUBLE / VARCHAR / UBIGINT / HUGEINT columns (tests/test_gpu_typed_fuzz.py)
            checks += typed_round(ctx, seed, n, with_updates=bool(rounds % 2), n_cases=30)
        else:
            checks += round_(ctx, seed, n, with_updates=bool(rounds % 2))
        rounds += 1
        seed += 1
        print(f"round {rounds}: {checks} scans match the oracle", flush=True)
    ctx.close()
    print(f"fuzz soak: {rounds} tables of {n} rows (seeds {seed0}..{seed - 1}), {checks} random scans, "
          f"every one equal to the oracle")


if __name__ == "__main__":
    main()
