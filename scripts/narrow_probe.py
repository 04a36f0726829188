#!/usr/bin/env python3
"""Selection-narrowing probe (development tool): N rows, an equality-indexed INT32 column of
`keys` distinct values and an unindexed INT64 column; times count(*) WHERE k = 7 AND v < c with
the unindexed comparison narrowed to the index leaf's rows and read in full, `reps` times each
(run under rocprofv3 for per-kernel times).

  python scripts/narrow_probe.py [rows] [keys] [reps]
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "duckdb-cubit_amd"), str(ROOT)]

import numpy as np  # noqa: E402

from cubit_amd import _lib as L  # noqa: E402
from cubit_amd import filters as F  # noqa: E402
from cubit_amd.table import Context, CubitTable  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300_000_000
    keys = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    i = np.arange(n, dtype=np.int64)
    k = (i * 2654435761 % keys).astype(np.int32)
    v = (i * 40503 % 1_000_003).astype(np.int64)
    ctx = Context(0)
    t = CubitTable(ctx, n)
    t.add_column(0, k)
    t.add_column(1, v)
    del k, v
    t.build_index(0, L.INDEX_EQUALITY)
    fs = F.TableFilterSet({0: F.ConstantFilter("=", 7), 1: F.ConstantFilter("<", 500_000)})
    for on in (True, False):
        t.use_narrowing(on)
        t.count(fs)
        t0 = time.perf_counter()
        for _ in range(reps):
            c = t.count(fs)
        ms = (time.perf_counter() - t0) / reps * 1e3
        print(f"{'narrowed' if on else 'full    '}: {ms:.3f} ms per query, count {c}, "
              f"narrowed leaves {t.last_narrowed()}", flush=True)
    t.close()
    ctx.close()


if __name__ == "__main__":
    main()
