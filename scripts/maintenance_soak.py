#!/usr/bin/env python3
"""Maintenance soak (development tool): tests/test_gpu_maintenance_fuzz.py's random sequences
of appends, update lists, merges, delete lists and scans (every scan against the oracle) for
a fixed wall-clock budget with fresh seeds; prints one summary line.

  python scripts/maintenance_soak.py [seconds] [rows] [first seed] [clustered]

clustered = 1: columns 0 and 1 ascend with the row, so scans skip zones (zonemaps) while the
sequence rewrites the bitvectors; odd rounds run clustered, even rounds uniform.
"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "duckdb-cubit_amd"), str(ROOT), str(ROOT / "tests")]

from cubit_amd.table import Context  # noqa: E402
from test_gpu_maintenance_fuzz import run  # noqa: E402


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 120.0
    n0 = int(sys.argv[2]) if len(sys.argv) > 2 else 500_000
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    clustered = len(sys.argv) > 4 and sys.argv[4] == "1"
    ctx = Context(0)
    t0 = time.time()
    total, rounds = {}, 0
    while time.time() - t0 < budget:
        c = run(ctx, seed + rounds, 80, n0, clustered=clustered and rounds % 2 == 1)
        for k, v in c.items():
            total[k] = total.get(k, 0) + v
        rounds += 1
        print(f"round {rounds} seed {seed + rounds - 1}: {c}", flush=True)
    ctx.close()
    print(f"maintenance soak: {rounds} tables, first seed {seed}, {n0} initial rows, {time.time() - t0:.0f} s: "
          f"{total} — every scan equal to the oracle")


if __name__ == "__main__":
    main()
