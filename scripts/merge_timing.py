"""Time cubit_table_merge_updates at the bench's scale (612 M rows, 1 % of rows updated, a range
index over 50 values) with CUBIT_MERGE_TIMING set: the phases on stderr."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "duckdb-cubit_amd"))
from cubit_amd import _lib as L  # noqa: E402
from cubit_amd.table import Context, CubitTable  # noqa: E402

n = 612_000_000
rng = np.random.default_rng(5)
col = (rng.integers(1, 51, n) * 100).astype(np.int64)
ctx = Context(0)
t = CubitTable(ctx, n)
t.add_column(2, col)
t.build_index(2, L.INDEX_RANGE)
for rep in range(2):
    rows = np.sort(rng.choice(n, size=n // 100, replace=False)).astype(np.int64)
    vals = (rng.integers(1, 51, len(rows)) * 100).astype(np.int64)
    t.set_updates(2, rows, vals, np.ones(len(rows), dtype=np.uint64))
    t0 = time.perf_counter()
    m = t.merge_updates(2, 2)
    print(f"merge rep {rep}: {m} rows in {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
t.close()
ctx.close()
