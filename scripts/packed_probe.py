#!/usr/bin/env python3
"""Packed-filter probe (development tool): an INT32 date-like column of N rows packed as DuckDB
BITPACKING FOR segments (libcubit_datagen, 12 bits per value), no index; times
count(*) WHERE v < c with the filter taken straight from the segments and from the plain
column, `reps` times each (run under rocprofv3 for per-kernel times and counters).

  python scripts/packed_probe.py [rows] [reps]
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "duckdb-cubit_amd"), str(ROOT)]

import numpy as np  # noqa: E402

from cubit_amd import datagen  # noqa: E402
from cubit_amd import filters as F  # noqa: E402
from cubit_amd.table import Context, CubitTable  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 600_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    v = (8035 + (np.arange(n, dtype=np.int64) * 2654435761 % 2526)).astype(np.int32)
    b = datagen.bitpack_for(v)
    ctx = Context(0)
    t = CubitTable(ctx, n)
    t.add_bitpacked_column(0, b.data, b.seg_off, b.seg_count, np.int32)
    fs = F.TableFilterSet({0: F.ConstantFilter("<", F.date(1994, 3, 17))})
    for on in (True, False):
        t.use_packed_filter(on)
        t.count(fs)
        t0 = time.perf_counter()
        for _ in range(reps):
            c = t.count(fs)
        ms = (time.perf_counter() - t0) / reps * 1e3
        print(f"{'segments' if on else 'plain   '}: {ms:.3f} ms per query, count {c}, "
              f"{8 * b.data.nbytes / n:.1f} bits per value", flush=True)
    t.close()
    ctx.close()


if __name__ == "__main__":
    main()
