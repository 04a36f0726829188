#!/usr/bin/env python3
"""Time the oracle's multi-threaded scan (the bench's cpu_baseline leg) on SF1 lineitem Q6 at
T = 1 and T = 8 in this container, for comparison with the reference DuckDB v1.1.2 timings
recorded in BASELINE.md §2 (same container class: 8 vCPUs)."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "duckdb-cubit_amd"), str(ROOT)]
from cubit_amd import datagen  # noqa: E402
from cubit_amd import filters as F  # noqa: E402
from oracle import oracle as O  # noqa: E402

li = datagen.tpch_lineitem(1.0)
cols = [O.Column(li.l_shipdate), O.Column(li.l_discount), O.Column(li.l_quantity)]
plan = F.serialize(F.q6_filter_set())
for t in (1, 8):
    ts = []
    for _ in range(15):
        t0 = time.perf_counter()
        q, _ = O.table_scan_mt(cols, plan, li.n_rows, t)
        ts.append(time.perf_counter() - t0)
    ms = float(np.median(ts)) * 1e3
    print(f"T={t}: q={q} median {ms:.2f} ms  ({q / ms * 1e3 / 1e6:.1f} M qualifying rows/s, "
          f"{li.n_rows / ms * 1e3 / 1e9:.2f} G input rows/s)")
