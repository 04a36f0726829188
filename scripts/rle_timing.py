"""Time rle_expand_kernel on a 600 M-row INT32 column of long runs (a sorted DATE-like column: 2,526
distinct days, as l_shipdate would be after an ORDER BY) given as the RLE segments DuckDB writes
(the oracle's restatement of rle.cpp, row groups of 122,880 rows), and on a column of short runs
(1 … 8 rows). Prints the kernel time (cubit_last_kernel_ms) and the write rate; the column read
back equals the values. Usage: python scripts/rle_timing.py [rows]"""
import ctypes
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "duckdb-cubit_amd"))

from cubit_amd import _lib as L  # noqa: E402
from cubit_amd.table import Context, CubitTable  # noqa: E402
from oracle import oracle as O  # noqa: E402


def run(ctx, v, label):
    t0 = time.perf_counter()
    data, offs, rows = O.rle_compress(v)
    t_c = time.perf_counter() - t0
    t = CubitTable(ctx, len(v))
    L.check(ctx.lib.cubit_ctx_enable_timing(ctx.handle, 1))
    times = []
    for _ in range(5):
        t.add_rle_column(0, data, offs, rows, v.dtype)
        ms = ctypes.c_float()
        L.check(ctx.lib.cubit_last_kernel_ms(ctx.handle, ctypes.byref(ms)))
        times.append(ms.value)
    L.check(ctx.lib.cubit_ctx_enable_timing(ctx.handle, 0))
    ok = np.array_equal(t.download_column(0), v)
    ms = float(np.median(times))
    print(f"{label}: rows {len(v)} segments {len(offs)} segment bytes {data.nbytes} (compress {t_c:.1f} s) "
          f"expand kernel {ms:.3f} ms median of {times} -> {len(v) * v.dtype.itemsize / ms / 1e6:.0f} GB/s written; "
          f"equal {ok}", flush=True)
    t.close()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 600_000_000
    ctx = Context(0)
    days = np.sort(np.random.default_rng(1).integers(8035, 8035 + 2526, n).astype(np.int32))
    run(ctx, days, "sorted days (long runs)")
    del days
    m = min(n, 10_000_000)  # the restated compressor walks runs in Python
    rng = np.random.default_rng(2)
    short = np.repeat(rng.integers(0, 1000, m // 4).astype(np.int32), rng.integers(1, 8, m // 4))[:m]
    run(ctx, short, "short runs (1-7 rows)")
    ctx.close()


if __name__ == "__main__":
    main()
