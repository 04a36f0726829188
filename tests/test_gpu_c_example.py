"""The C ABI from a plain-C host (duckdb-cubit_amd/examples/q6_scan.c, built by
__graft_entry__.build()): TPC-H SF1 Q6 through cubit_table_scan, the fused
cubit_table_sum_product and the seq_scan-shaped callbacks of cubit_scan.h, with no Python or
PyTorch in the process, and the whole query as four pthread pipeline tasks over the callbacks.
Its output must equal the reference's SF1 fingerprint and answer."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "duckdb-cubit_amd" / "lib" / "q6_scan"


def fp_count(golden):
    return golden["tpch"]["fingerprints"]["sf1_q6"]["count"]


@pytest.mark.gpu
def test_q6_from_c(golden):
    if not EXE.exists():
        pytest.fail(f"{EXE} is missing: run __graft_entry__.build()")
    out = subprocess.run([str(EXE), "1", "4"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.splitlines()
    f = lines[0].split()
    got = dict(zip(f[0::2], f[1::2]))
    # the query as four pipeline tasks over the callbacks: every row, the fused revenue
    p = lines[1].split()[1:]  # "pipeline" then name value pairs
    pipe = dict(zip(p[0::2], p[1::2]))
    assert int(pipe["threads"]) == 4 and int(pipe["rows"]) == fp_count(golden)
    assert pipe["revenue_match"] == "1"
    fp = golden["tpch"]["fingerprints"]["sf1_q6"]
    assert int(got["rows"]) == fp["count"]
    assert int(got["table_function_rows"]) == fp["count"]
    assert int(got["sum_rowid"]) == fp["sum_rowid"]
    assert int(got["table_function_sum_rowid"]) == fp["sum_rowid"]
    assert got["revenue"] == golden["tpch"]["q6_revenue"]["1"]["revenue"]


def test_c_example_links_against_the_abi():
    """CPU: the example is built and its dynamic dependencies are the repo's own libraries."""
    if not EXE.exists():
        pytest.fail(f"{EXE} is missing: run __graft_entry__.build()")
    out = subprocess.run(["ldd", str(EXE)], capture_output=True, text=True)
    for lib in ("libcubitgpu.so", "libcubit_scan.so", "libcubit_datagen.so"):
        assert lib in out.stdout, out.stdout


@pytest.mark.gpu
def test_q6_from_c_over_partitions(golden):
    """q6_scan --partitions N: lineitem as N row-range partitions with a context each (spread
    over the visible devices), the pipeline over all of them through one cursor
    (cubit_scan_init_global_multi): every Q6 row, the fused revenue."""
    out = subprocess.run([str(EXE), "1", "4", "--partitions", "3"], capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stderr
    line = [x for x in out.stdout.splitlines() if x.startswith("partitioned_pipeline")][0].split()[1:]
    got = dict(zip(line[0::2], line[1::2]))
    assert int(got["partitions"]) == 3 and int(got["threads"]) == 4
    assert int(got["rows"]) == fp_count(golden) and got["revenue_match"] == "1"
