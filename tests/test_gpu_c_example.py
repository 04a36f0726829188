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


# ---- typed columns from C (examples/typed_scan.c) ---------------------------------------------------
TYPED = ROOT / "duckdb-cubit_amd" / "lib" / "typed_scan"
C_OPS = {"=": "=", "<>": "<>", "!=": "<>", "<": "<", "<=": "<=", ">": ">", ">=": ">="}


def typed_run(spec_lines):
    """Run typed_scan over a spec; [(count, [(rowid, [value tokens])])] per query."""
    if not TYPED.exists():
        pytest.fail(f"{TYPED} is missing: run __graft_entry__.build()")
    out = subprocess.run([str(TYPED)], input="\n".join(spec_lines) + "\n", capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    res, cur = [], None
    for line in out.stdout.splitlines():
        f = line.split()
        if f[0] == "result":
            cur = (int(f[1]), [])
            res.append(cur)
        else:
            cur[1].append((int(f[0]), f[1:]))
    for count, rows in res:
        assert count == len(rows)
    return res


def hexlit(s):
    return "x" + (s.encode() if isinstance(s, str) else bytes(s)).hex()


def test_typed_example_links_against_the_abi():
    """CPU: the typed example is built and links the repo's own libraries."""
    if not TYPED.exists():
        pytest.fail(f"{TYPED} is missing: run __graft_entry__.build()")
    out = subprocess.run(["ldd", str(TYPED)], capture_output=True, text=True)
    for lib in ("libcubitgpu.so", "libcubit_scan.so"):
        assert lib in out.stdout, out.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("index", [None, "range", "equality"])
def test_typed_columns_from_c_match_reference_cases(index):
    """The reference's filter cases on HUGEINT / UHUGEINT (test_*_ops, *_null_value, *_storage),
    FLOAT / DOUBLE (nan_test, infinity_test: each type) and VARCHAR (strtest / strings) columns,
    pushed from C through the table-function callbacks: every query's rows / count as the files
    state them."""
    import json

    g = ROOT / "tests" / "golden"
    # HUGEINT / UHUGEINT
    for case in json.loads((g / "huge_filter_cases.json").read_text())["cases"]:
        h = case["columns"].index("h")
        typ = case["types"][h].lower()
        spec = [f"column {typ}"] + [f"row {r[h] if r[h] is not None else 'NULL'}" for r in case["rows"]]
        if index:
            spec.append(f"index 0 {index}")
        for q in case["queries"]:
            spec.append("query 1 0 " + ("isnull -" if q["cmp"] == "IS NULL" else f"{C_OPS[q['cmp']]} {q['constant']}"))
        for q, (count, rows) in zip(case["queries"], typed_run(spec)):
            vals = [v[0] for _, v in rows]
            if q["select"] == "COUNT(*)":
                got = [str(count)]
            elif q["select"].startswith("id, FIRST(h), LAST(h)"):
                assert all(v == "NULL" for v in vals)
                ids = {case["rows"][r][case["columns"].index("id")] for r, _ in rows}
                got = [f"{i}\tNULL\tNULL" for i in sorted(ids)]
            else:
                got = sorted(vals, key=int) if "ORDER BY" in q["sql"] else vals
            assert got == q["rows"], (case["file"], q["sql"], index)
    # FLOAT / DOUBLE
    for case in json.loads((g / "float_filter_cases.json").read_text())["cases"]:
        for typ in ("float", "double"):
            spec = [f"column {typ}"] + [f"row {v}" for v in case["inserted"]]
            if index:
                spec.append(f"index 0 {index}")
            spec += [f"query 1 0 {C_OPS[q['cmp']]} {q['constant']}" for q in case["queries"]]
            for q, (count, rows) in zip(case["queries"], typed_run(spec)):
                got = [v[0] for _, v in rows]  # in row-id order
                if "ORDER BY" in q["sql"]:  # DuckDB's order: NaN above +inf
                    got = sorted(got, key=lambda x: (x == "nan", float(x) if x != "nan" else 0.0))
                    assert got == q["rows"], (case["file"], typ, q["sql"], index)
                else:
                    assert sorted(got) == sorted(q["rows"]), (case["file"], typ, q["sql"], index)
    # VARCHAR
    for case in json.loads((g / "string_filter_cases.json").read_text())["cases"]:
        rows = case["rows"]
        for q in case["queries"]:
            col = q["column"]
            spec = ["column varchar"] + [f"row {hexlit(r[col]) if r[col] is not None else 'NULL'}" for r in rows]
            if index:
                spec.append(f"index 0 {index}")
            terms = [f"0 {C_OPS[op]} {hexlit(lit)}" for op, lit in q["terms"]]
            spec.append(f"query {len(terms)} " + " ".join(terms))
            (count, got), = typed_run(spec)
            proj = q["project"] if q["project"] is not None else col
            assert [rows[r][proj] for r, _ in got] == q["rows"], (q["sql"], index)


@pytest.mark.gpu
def test_typed_columns_from_c_match_numpy():
    """Random UBIGINT (full range), BIGINT, DOUBLE and HUGEINT columns with NULLs in one table,
    conjunctions across them pushed from C: row ids and every projected value against numpy /
    Python on the same rows."""
    import math

    import numpy as np

    rng = np.random.default_rng(3)
    n = 5000
    ub = rng.integers(0, 2 ** 64 - 1, n, dtype=np.uint64, endpoint=True)
    ub[:4] = [0, 2 ** 63 - 1, 2 ** 63, 2 ** 64 - 1]
    bi = rng.integers(-50, 50, n)
    db = rng.standard_normal(n) * 10
    db[rng.integers(0, n, 40)] = math.nan
    hp = [-(2 ** 127), -(2 ** 64), -1, 0, 1, 2 ** 64, 2 ** 100, 2 ** 127 - 1]
    hg = [hp[i] for i in rng.integers(0, len(hp), n)]
    ok = rng.random((4, n)) > 0.1
    spec = ["column ubigint", "column bigint", "column double", "column hugeint"]
    for r in range(n):
        vals = [str(int(ub[r])), str(int(bi[r])), repr(float(db[r])) if not math.isnan(db[r]) else "nan", str(hg[r])]
        spec.append("row " + " ".join(v if ok[j, r] else "NULL" for j, v in enumerate(vals)))
    spec.append("index 3 equality")
    queries = [
        ("0 >= 9223372036854775808", lambda r: ub[r] >= 2 ** 63),
        ("0 < 9223372036854775808 1 > 10", lambda r: ub[r] < 2 ** 63 and bi[r] > 10),
        ("2 > 5 3 >= 0", lambda r: (db[r] > 5 or math.isnan(db[r])) and hg[r] >= 0),
        ("3 < 18446744073709551616 3 > -18446744073709551616", lambda r: -(2 ** 64) < hg[r] < 2 ** 64),
        ("2 = nan 0 <> 0", lambda r: math.isnan(db[r]) and ub[r] != 0),
    ]
    cols_of = {0: 0, 1: 1, 2: 2, 3: 3}
    for text, _ in queries:
        f = text.split()
        spec.append(f"query {len(f) // 3} {text}")
    for (text, pred), (count, rows) in zip(queries, typed_run(spec)):
        used = {cols_of[int(c)] for c in text.split()[0::3]}
        want = [r for r in range(n) if all(ok[j, r] for j in used) and pred(r)]
        assert [r for r, _ in rows] == want, text
        for r, v in rows[:: max(1, len(rows) // 50)]:
            assert v[0] == (str(int(ub[r])) if ok[0, r] else "NULL")
            assert v[1] == (str(int(bi[r])) if ok[1, r] else "NULL")
            assert v[3] == (str(hg[r]) if ok[3, r] else "NULL")
            if ok[2, r] and not math.isnan(db[r]):
                assert float(v[2]) == float(db[r])
