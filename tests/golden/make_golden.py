"""Regenerate tests/golden/*.json from the reference's own files (run in the build
container, where /root/reference exists). The JSON it writes is data only: expected
outputs quoted from the reference's answer files and tests, plus the fingerprints the
survey measured by running the reference."""
import json
import re
from pathlib import Path

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent


def answer(sf):
    p = REF / f"extension/tpch/dbgen/answers/sf{sf}/q06.csv"
    lines = p.read_text().split()
    assert lines[0] == "revenue"
    return {"revenue": lines[1], "source": str(p.relative_to(REF))}


def sqllogic_script(rel):
    """A .test file as data: its statements and queries in order — connection, SQL text, and
    the outcome the file expects (ok / error, or the result rows with NULL as None) — plus the
    session settings that shape the replay (immediate transaction mode, NULL ordering)."""
    src = (REF / rel).read_text()
    script, flags = [], {"immediate_transaction_mode": False, "nulls_first": False}
    loop = None  # (variable, range, blocks) while inside loop ... endloop

    def value(v):
        if v == "NULL":
            return None
        if re.fullmatch(r"-?\d+", v):
            return int(v)
        if re.fullmatch(r"-?\d+\.\d*", v):
            return int(float(v))  # SUM as DOUBLE: "294912.000000"
        return v  # text (an EXPLAIN's plan line): kept as the file has it

    def emit(lines):
        head = lines[0].split()
        con = head[2] if len(head) > 2 else "default"
        if head[0] == "statement":
            body = " ".join(x.strip() for x in lines[1:] if x.strip() != "----")
            for sql in [s.strip() for s in body.split(";") if s.strip()]:  # one entry per statement
                if sql.upper().startswith("SET IMMEDIATE_TRANSACTION_MODE"):
                    flags["immediate_transaction_mode"] = True
                elif sql.upper().startswith("SET DEFAULT_NULL_ORDER"):
                    flags["nulls_first"] = "nulls_first" in sql
                elif not sql.upper().startswith("PRAGMA"):
                    script.append({"op": "statement", "con": con, "sql": sql, "ok": head[1] == "ok"})
        elif head[0] == "query":
            sep = lines.index("----")
            rows = [[value(v) for v in line.split("\t")] for line in lines[sep + 1:]]
            script.append({"op": "query", "con": con, "sql": " ".join(lines[1:sep]), "rows": rows})
        else:
            assert head[0] in ("require", "load"), head

    for block in re.split(r"\n\s*\n", src):
        lines = [x for x in block.strip().split("\n") if x and not x.startswith("#")]
        if not lines:
            continue
        head = lines[0].split()
        if head[0] == "loop":
            loop = (head[1], range(int(head[2]), int(head[3])), [])
            lines = lines[1:]
            if not lines:
                continue
        if lines[-1].strip() == "endloop":
            var, rng, blocks = loop
            blocks.append(lines[:-1])
            for i in rng:
                for b in blocks:
                    if b:
                        emit([x.replace("${" + var + "}", str(i)) for x in b])
            loop = None
            continue
        if loop is not None:
            loop[2].append(lines)
            continue
        emit(lines)
    return {"source": rel, **flags, "script": script}


def main():
    tpch = {
        "q6_revenue": {sf: answer(sf) for sf in ("0.01", "0.1", "1", "100")},
        # SURVEY.md §8c "Golden vectors / known answers", measured with the reference
        # (DuckDB v1.1.2 built from /root/reference) in the survey container.
        "fingerprints": {
            "sf1_q6": {"count": 114160, "sum_rowid": 341745978685, "min": 55, "max": 6001177,
                       "xor_hash": 9778593094192572261},
            "sf1_shipdate_eq_1995_03_15": {"count": 2528, "sum_rowid": 7563025794,
                                            "xor_hash": 11097155983190906094},
            "sf1_leaf_counts": {"shipdate_1994": 909455, "discount_005_007": 1637557, "quantity_lt_24": 2758822},
            "sf100_q6": {"count": 11421368, "sum_rowid": 3427761320230477, "min": 55, "max": 600037873,
                         "xor_hash": 11990059560084878909},
            "sf100_shipdate_eq_1995_03_15": {"count": 249371},
            "sf001_q6": {"count": 1191},
            "sf001_mvcc": {"writer_view": 1267, "reader_view": 1191,
                           "writer_txn": "UPDATE lineitem SET l_quantity=1 WHERE rowid%7=0; "
                                         "DELETE FROM lineitem WHERE rowid%11=0 (uncommitted)"},
            "source": "SURVEY.md §8c; BASELINE.md §3",
        },
    }
    (OUT / "tpch.json").write_text(json.dumps(tpch, indent=1, sort_keys=True) + "\n")

    # test/sql/filter/test_zonemap_segment.test: blocks of 65,534 rows with values 1..5,
    # SUM(i) WHERE i=k
    zm = {
        "source": "test/sql/filter/test_zonemap_segment.test:13-111",
        "block_rows": 65534,
        "values": [1, 2, 3, 4, 5],
        "expected_sum_eq": {"1": 65534, "2": 131068, "3": 196602, "4": 262136, "5": 327670, "6": None},
    }
    # test/sql/transactions/test_interleaved_versions.test: two rows, interleaved deletes
    iv = {
        "source": "test/sql/transactions/test_interleaved_versions.test:66-120",
        "rows": [1, 2],
        "steps": [
            {"con1_deletes": "i=1", "con2_deletes": "i=2", "expect": {"con1": 2, "con2": 1, "con3": 3}},
            {"after": "con1 COMMIT", "expect": {"con1": 2, "con2": 1}},
        ],
    }
    # test/sql/storage/compression/rle/*.test: tables whose INTEGER columns DuckDB stores as RLE
    # segments after the CHECKPOINT, as (value, repeat) runs in row order (null = NULL), a pushed
    # filter per query ([column, op, constant] or null) and its aggregates as the files state them
    # (sum / min / max / count of the integer column, count_star, min_id / max_id)
    rle = {
        "rle_filter_pushdown": {
            "source": "test/sql/storage/compression/rle/rle_filter_pushdown.test:12-33",
            "id": "VARCHAR", "col": [[1, 5000], [2, 5000]],
            "queries": [{"where": ["col", "=", 2], "expect": {"sum": 10000, "min": 2, "max": 2, "count_star": 5000}},
                        {"where": ["id", "=", "5000"],
                         "expect": {"min_id": "5000", "max_id": "5000", "sum": 2, "min": 2, "max": 2, "count_star": 1}}]},
        "rle_index_fetch": {
            "source": "test/sql/storage/compression/rle/rle_index_fetch.test:12-31",
            "id": "INTEGER", "col": [[1, 5000], [2, 5000]],
            "queries": [{"where": ["id", "=", 5000],
                         "expect": {"min_id": 5000, "max_id": 5000, "sum": 2, "min": 2, "max": 2, "count_star": 1}}]},
        "rle_medium": {
            "source": "test/sql/storage/compression/rle/rle_medium.test:13-33",
            "id": None, "col": [[k, 1000] for k in range(1, 7)],
            "queries": [{"where": None, "expect": {"sum": 21000, "min": 1, "max": 6, "count_star": 6000}}]},
        "rle_nulls_edge_case": {
            "source": "test/sql/storage/compression/rle/rle_nulls_edge_case.test:21-44",
            "id": None, "col": [[None, 65535], [1, 1], [2, 1], [3, 1]],
            "queries": [{"where": None, "expect": {"min": 1, "max": 3, "count_star": 65538, "count": 3}}]},
    }
    # test/optimizer/pushdown/timestamp_to_date_pushdown.test: t1(ts TIMESTAMP, i INT) as runs of
    # (timestamp, i from generate_series(lo, hi)); `ts::date == d` is pushed to the scan as the
    # TIMESTAMP range [d 00:00, d + 1 day) (the file checks the plan keeps a SEQ_SCAN filter and no
    # FILTER above it); each count(*) with its optional bound on i
    tsd = {
        "source": "test/optimizer/pushdown/timestamp_to_date_pushdown.test:14-75",
        "runs": [["2024-05-01 00:00:00", 1, 2000], ["2024-05-02 00:00:00", 1, 1000],
                 ["2024-05-02 00:22:00", 1, 1000], ["2024-05-03 00:00:00", 1, 2000]],
        "queries": [{"date": "2024-05-02", "i": [">", 1000], "count": 0},
                    {"date": "2024-05-02", "i": ["<=", 500], "count": 1000},
                    {"date": "2024-05-01", "i": ["<=", 500], "count": 500},
                    {"date": "2024-05-03", "i": None, "count": 2000}],
    }
    # test/optimizer/pushdown/table_or_pushdown.test: integers(a, b) = (1,1) … (5,5); the
    # integer queries' expected rows (a values). The trees use the repo's residual syntax:
    # ["or"|"and", children…] / [column, cmp, constant], column 0 = a, 1 = b.
    orp = {
        "source": "test/optimizer/pushdown/table_or_pushdown.test:11-57",
        "rows": [1, 2, 3, 4, 5],
        "queries": [
            {"sql": "a=1 OR b=2 AND (a>3 OR b<5)",
             "tree": ["or", [0, "=", 1], ["and", [1, "=", 2], ["or", [0, ">", 3], [1, "<", 5]]]],
             "expect": [1, 2]},
            {"sql": "a=1 OR a=2 AND (a>3 OR b<5)",
             "tree": ["or", [0, "=", 1], ["and", [0, "=", 2], ["or", [0, ">", 3], [1, "<", 5]]]],
             "expect": [1, 2]},
            {"sql": "a=1 OR (a>3 AND a<5)",
             "tree": ["or", [0, "=", 1], ["and", [0, ">", 3], [0, "<", 5]]],
             "expect": [1, 4]},
            {"sql": "a=1 OR a>3 OR a<5",
             "tree": ["or", [0, "=", 1], [0, ">", 3], [0, "<", 5]],
             "expect": [1, 2, 3, 4, 5]},
        ],
    }
    # test/sql/update/test_update.test: one row a=3; con1 updates it to 1 and commits, then
    # updates it to 4 and rolls back. Each check: which connection, the WHERE (None = none),
    # and the rows it sees.
    upd = {
        "source": "test/sql/update/test_update.test:11-104",
        "rows": [3],
        "steps": [
            {"do": "con1 BEGIN; UPDATE test SET a=1",
             "checks": [["con1", None, [1]], ["con1", 1, [1]], ["con2", None, [3]], ["con2", 3, [3]]]},
            {"do": "con1 COMMIT", "checks": [["con1", None, [1]], ["con2", None, [1]]]},
            {"do": "con1 BEGIN; UPDATE test SET a=4", "checks": [["con1", None, [4]], ["con2", None, [1]]]},
            {"do": "con1 ROLLBACK", "checks": [["con1", None, [1]], ["con1", 1, [1]], ["con2", None, [1]]]},
        ],
    }
    # test/optimizer/pushdown/table_filter_pushdown.test. The file asserts that these filters
    # are pushed into the scan (no FILTER operator left); the rows each must return follow from
    # the data it inserts. `types` are the <numeric> types whose physical type is an integer
    # of at most 32 bits, or a signed 64-bit one (sqllogic_test_runner.cpp:180-203), with the
    # physical width the shim uploads them at.
    tfp = {
        "source": "test/optimizer/pushdown/table_filter_pushdown.test:8-195",
        "integers": {"rows": [[5, 5, 5], [10, 10, 10]],
                     "queries": [{"where": [[1, "=", 5]], "k": [5]},
                                 {"where": [[1, "=", 5], [0, "=", 10]], "k": []}]},
        "numbers": {"types": {"tinyint": 32, "smallint": 32, "integer": 32, "bigint": 64,
                              "utinyint": 32, "usmallint": 32, "uinteger": 64},
                    "rows": [[0, 0, 0], [1, 1, 1], [2, 2, 2]],
                    "queries": [{"where": [[1, "=", 1]], "k": [1]}, {"where": [[1, ">", 1]], "k": [2]},
                                {"where": [[1, ">=", 1]], "k": [1, 2]}, {"where": [[1, "<", 1]], "k": [0]},
                                {"where": [[1, "<=", 1]], "k": [0, 1]}]},
        # create temporary table t as select range a, range % 10 b ... from range(100);
        # count(*) where b <= 3 and b >= 0
        "range_mod": {"n": 100, "mod": 10, "where": [[0, "<=", 3], [0, ">=", 0]], "count": 40},
        # TIME as int64 microseconds; the fourth row is NULL
        "time": {"micros": [60000000, 600000000, 3600000000, None], "eq": 60000000, "count": 1},
        # BOOLEAN (i, j): (TRUE,TRUE),(TRUE,FALSE),(FALSE,TRUE),(NULL,NULL); SELECT i WHERE j = TRUE
        "bool": {"i": [1, 1, 0, None], "j": [1, 0, 1, None], "eq": 1, "i_expect": [1, 0]},
        # TIMESTAMP rows NOW() and NOW() - 10 years; ts >= NOW() - 1 year -> COUNT(*) = 1
        "timestamp": {"count": 1},
    }
    # test/sql/transactions/test_multi_version.test: rows 1, 2, 3; con1 updates, updates again,
    # deletes and inserts inside one transaction, then commits; SUM(i) as each connection sees
    # it after each statement. The sums are read from the file (the `query R conX` blocks, in
    # order) and must equal the steps below.
    mv_src = REF / "test/sql/transactions/test_multi_version.test"
    mv_sums = [(c, float(v)) for c, v in re.findall(r"query R (con\d)\nSELECT SUM\(i\) FROM integers\n----\n([0-9.]+)",
                                                    mv_src.read_text())]
    mv = {
        "source": "test/sql/transactions/test_multi_version.test:9-99",
        "rows": [1, 2, 3],
        "steps": [
            {"do": "start", "expect": {"con1": 6, "con2": 6}},
            {"do": "con1 BEGIN; UPDATE integers SET i=5 WHERE i=1", "expect": {"con1": 10, "con2": 6}},
            {"do": "con1 UPDATE integers SET i=10 WHERE i=5", "expect": {"con1": 15, "con2": 6}},
            {"do": "con1 DELETE FROM integers WHERE i>5", "expect": {"con1": 5, "con2": 6}},
            {"do": "con1 INSERT INTO integers VALUES (1), (2)", "expect": {"con1": 8, "con2": 6}},
            {"do": "con1 COMMIT", "expect": {"con2": 8}},
        ],
    }
    assert mv_sums == [(c, float(v)) for st in mv["steps"] for c, v in st["expect"].items()], mv_sums
    # test/sql/parallelism/interquery/concurrent_reads_while_updating.test_slow: integers =
    # range(10000); thread 0 runs UPDATE integers SET i=i+1 20 times while 19 threads run
    # SELECT COUNT(*)==10000, SUM(i) BETWEEN 49995000 AND 50195000 200 times each; afterwards
    # COUNT(*), SUM(i) = 10000, 50195000.
    cr_src = (REF / "test/sql/parallelism/interquery/concurrent_reads_while_updating.test_slow").read_text()
    for needle in ("range(10000)", "concurrentloop threadid 0 20", "loop i 0 20", "UPDATE integers SET i=i+1",
                   "loop i 0 200", "SUM(i)>= 49995000 AND SUM(i) <= 50195000", "10000\t50195000"):
        assert needle in cr_src, needle
    cr = {
        "source": "test/sql/parallelism/interquery/concurrent_reads_while_updating.test_slow",
        "rows": 10000, "threads": 20, "updates": 20, "reads_per_thread": 200,
        "reader_count": 10000, "reader_sum_range": [49995000, 50195000],
        "final": {"count": 10000, "sum": 50195000},
    }
    # test/sql/update/test_update_many_updaters.test: rows 1, 2, 3; an updater commits one
    # update per row between four readers' BEGINs (immediate_transaction_mode), reverts, and
    # again; then three readers update and commit in phases. Every `query I <con>` view, in
    # file order (the conflicting statements fail and change nothing).
    mu_src = (REF / "test/sql/update/test_update_many_updaters.test").read_text()
    assert "SET immediate_transaction_mode=true" in mu_src
    mu_views = [[c, [int(x) for x in v.split()]]
                for c, v in re.findall(r"query I (\w+)\nSELECT \* FROM test ORDER BY a\n----\n((?:-?\d+\n?)+)", mu_src)]
    mu = {"source": "test/sql/update/test_update_many_updaters.test", "rows": [1, 2, 3], "views": mu_views}
    # test/sql/update/block_boundary_update.test_slow: BIGINT range(0, 50000); UPDATE i=i+1
    # twice, INSERT INTO test SELECT * FROM test, UPDATE i=i+1 twice; COUNT(i), SUM(i) after
    # the CREATE and after each statement (read from the file, in order)
    bb_src = (REF / "test/sql/update/block_boundary_update.test_slow").read_text()
    assert "CREATE TABLE test AS SELECT * FROM range (0, 50000, 1) t1(i);" in bb_src
    stmts = re.findall(r"statement ok\n(UPDATE test SET i=i\+1|INSERT INTO test SELECT \* FROM test;)", bb_src)
    counts = [[int(a), int(b)] for a, b in re.findall(r"SELECT COUNT\(i\), SUM\(i\) FROM test\n----\n(\d+)\t(\d+)", bb_src)]
    bb = {"source": "test/sql/update/block_boundary_update.test_slow", "rows": 50000,
          "statements": ["update" if x.startswith("UPDATE") else "insert_select" for x in stmts],
          "count_sum": counts}
    assert len(counts) == len(stmts) + 1
    # test/sql/filter/test_zonemap.test_slow (marked `mode skip` in the reference for memory on
    # 32-bit builds; its expected counts stand): t = range(100000000) as a, length(range) b (the
    # digit count), cross-column OR trees, count(*). The trees use the residual syntax above,
    # column 0 = a, 1 = b.
    zt_src = (REF / "test/sql/filter/test_zonemap.test_slow").read_text()
    zt_counts = [int(x) for x in re.findall(r"query I\nselect count\(\*\) from t where [^\n]*\n----\n(\d+)", zt_src)]
    zt_sql = re.findall(r"query I\nselect count\(\*\) from t where ([^\n]*)\n----", zt_src)
    trees = {
        "a > 500 or a <= 700": ["or", [0, ">", 500], [0, "<=", 700]],
        "(a > 500 and b = 3) or (a > 7000 and b = 2)":
            ["or", ["and", [0, ">", 500], [1, "=", 3]], ["and", [0, ">", 7000], [1, "=", 2]]],
        "(a > 500 AND b = 3) OR (a > 400) OR (a > 300 AND b=4) OR (a > 600 AND a > 300)":
            ["or", ["and", [0, ">", 500], [1, "=", 3]], [0, ">", 400], ["and", [0, ">", 300], [1, "=", 4]],
             ["and", [0, ">", 600], [0, ">", 300]]],
        "(a > 500 AND b = 1) OR b < 2": ["or", ["and", [0, ">", 500], [1, "=", 1]], [1, "<", 2]],
    }
    assert "create temporary table t as select range a, length(range) b" in zt_src and "range(100000000)" in zt_src
    zt = {"source": "test/sql/filter/test_zonemap.test_slow", "rows": 100000000,
          "queries": [{"sql": q, "tree": trees[q], "count": c} for q, c in zip(zt_sql, zt_counts)]}
    assert len(zt["queries"]) == 6
    # test/sql/filter/filter_cache.test: integers(a) = generate_series(0, 9999) x generate_series(0, 9)
    # (each a ten times); the nested subqueries' WHERE clauses reach the scan as one filter: the
    # plain comparisons as the TableFilterSet ("where", ANDed), the OR as a residual tree
    fc_case = sqllogic_script("test/sql/filter/filter_cache.test")
    assert any("generate_series(0, 9999, 1) tbl(a), generate_series(0, 9, 1) tbl2(b)" in st["sql"]
               for st in fc_case["script"])
    fc_counts = [st["rows"][0][0] for st in fc_case["script"] if st["op"] == "query"]
    fc_shapes = [
        {"sql": "a<5", "where": [[0, "<", 5]], "tree": None},
        {"sql": "((a>1 AND a<10) OR a>9995) AND a<5", "where": [[0, "<", 5]],
         "tree": ["or", ["and", [0, ">", 1], [0, "<", 10]], [0, ">", 9995]]},
        {"sql": "((a <> 3 AND a<50) OR (a > 9995)) AND a>1 AND a<20 AND a<5",
         "where": [[0, ">", 1], [0, "<", 20], [0, "<", 5]],
         "tree": ["or", ["and", [0, "!=", 3], [0, "<", 50]], [0, ">", 9995]]},
    ]
    assert len(fc_counts) == len(fc_shapes)
    fc = {"source": "test/sql/filter/filter_cache.test", "values": [0, 10000], "repeat": 10,
          "queries": [dict(q, count=c) for q, c in zip(fc_shapes, fc_counts)]}
    # test/sql/filter/test_obsolete_filters.test: integers(a, b) = (1,10) (2,12) (3,14) (4,16)
    # (5,NULL) (NULL,NULL); every query whose WHERE is an AND of comparisons of a with integer
    # constants — redundant, subsumed and contradictory ones, all pushed into the scan as one
    # column's conjunction — with the rows it returns (the VARCHAR table and the constant-only
    # WHEREs, which the planner folds before any scan, are not taken)
    ob_src = (REF / "test/sql/filter/test_obsolete_filters.test").read_text()
    assert "INSERT INTO integers VALUES (1, 10), (2, 12), (3, 14), (4, 16), (5, NULL), (NULL, NULL)" in ob_src
    term = re.compile(r"^a(<=|>=|<>|<|>|=)(-?\d+)$")
    ob_q = []
    for where, body in re.findall(r"query II\nSELECT \* FROM integers WHERE ([^\n]*?)(?: ORDER BY 1)?\n----\n((?:[^\n]+\n?)*)",
                                  ob_src):
        parts = [x.strip() for x in where.split(" AND ")]
        if not all(term.match(x) for x in parts):
            continue
        rows = [[None if v == "NULL" else int(v) for v in line.split("\t")] for line in body.strip().split("\n") if line]
        ob_q.append({"where": where, "terms": [[term.match(x).group(1), int(term.match(x).group(2))] for x in parts],
                     "rows": rows})
    ob = {"source": "test/sql/filter/test_obsolete_filters.test",
          "a": [1, 2, 3, 4, 5, None], "b": [10, 12, 14, 16, None, None], "queries": ob_q}
    assert len(ob_q) >= 30, len(ob_q)
    # the index variant (ART scans, here the bitmap index) on the reference's ART scan
    # tests: test/sql/index/art/scan/test_art_negative_range_scan.test (range(-500, 500), sums of
    # closed ranges) and test_art_many_matches.test (0, 1 interleaved n times, counts of every
    # comparison), read from the files
    art_dir = REF / "test/sql/index/art/scan"
    neg_src = (art_dir / "test_art_negative_range_scan.test").read_text()
    assert "INSERT INTO integers SELECT * FROM range(-500, 500, 1)" in neg_src
    neg = [{"ge": int(a), "le": int(b), "sum": int(float(v))} for a, b, v in re.findall(
        r"query R\nSELECT sum\(i\) FROM integers WHERE i >= (-?\d+) AND i <= (-?\d+)\n----\n(-?[0-9.]+)", neg_src)]
    mm_src = (art_dir / "test_art_many_matches.test").read_text()
    blocks = []
    for part in mm_src.split("BEGIN TRANSACTION")[1:]:
        m = re.search(r"RANGE\(0, (\d+), 1\) t2\(j\), \(VALUES \(0\), \(1\)\) t1\(i\) ORDER BY j, i", part)
        qs = [[op, int(k), int(v)] for op, k, v in re.findall(
            r"query I\nSELECT COUNT\(\*\) FROM integers WHERE i(<=|>=|<|>|=)(\d+)\n----\n(\d+)", part)]
        blocks.append({"pairs": int(m.group(1)), "counts": qs})
    art = {"negative_range": {"source": "test/sql/index/art/scan/test_art_negative_range_scan.test",
                              "range": [-500, 500], "queries": neg},
           "many_matches": {"source": "test/sql/index/art/scan/test_art_many_matches.test", "blocks": blocks}}
    # test_art_adaptive_scan.test: 42 x 2050 then 43 … 5042 appended, COUNT(i) WHERE i = 42; and
    # test_art_range_scan.test's USMALLINT parts: rows 1 … 19 (resp. 134), x > 20 (resp. 135) empty,
    # then 256 (resp. 256, 257) appended after the index and found. Each step: rows appended (None:
    # the table's first rows), then the query's expected rows / count from the file.
    ad = sqllogic_script("test/sql/index/art/scan/test_art_adaptive_scan.test")
    ad_sql = " ".join(st["sql"] for st in ad["script"])
    assert "SELECT 42 AS i FROM range(2050)" in ad_sql and "SELECT 42 + 1 + range FROM range(5000)" in ad_sql
    ad_count = [st["rows"] for st in ad["script"] if st["op"] == "query" and st["sql"].startswith("SELECT COUNT(i)")]
    rs = sqllogic_script("test/sql/index/art/scan/test_art_range_scan.test")
    rs_q = [st for st in rs["script"] if st["op"] == "query" and "x >" in st["sql"] and "'" not in st["sql"]]
    rs_sql = " ".join(st["sql"] for st in rs["script"])
    assert "SELECT i FROM range(1, 20) tbl(i)" in rs_sql and "SELECT i FROM range(1, 135) tbl(i)" in rs_sql
    assert [q["sql"] for q in rs_q] == ["SELECT x FROM test WHERE x > 20;"] * 2 + ["SELECT x FROM test WHERE x > 135;"] * 2
    art["appended"] = [
        {"source": "test/sql/index/art/scan/test_art_adaptive_scan.test", "type": "int32",
         "steps": [{"append": {"repeat": [42, 2050]}, "then": {"range": [43, 5043]}, "filter": ["=", 42],
                    "count": ad_count[0][0][0]}]},
        {"source": "test/sql/index/art/scan/test_art_range_scan.test (node 48)", "type": "uint16",
         "steps": [{"append": {"range": [1, 20]}, "filter": [">", 20], "rows": [r[0] for r in rs_q[0]["rows"]]},
                   {"append": {"values": [256]}, "filter": [">", 20], "rows": [r[0] for r in rs_q[1]["rows"]]}]},
        {"source": "test/sql/index/art/scan/test_art_range_scan.test (node 256)", "type": "uint16",
         "steps": [{"append": {"range": [1, 135]}, "filter": [">", 135], "rows": [r[0] for r in rs_q[2]["rows"]]},
                   {"append": {"values": [256, 257]}, "filter": [">", 135], "rows": [r[0] for r in rs_q[3]["rows"]]}]},
    ]
    assert len(neg) == 3 and len(blocks) == 2 and all(len(b["counts"]) == 6 for b in blocks)
    # test/sql/filter/test_transitive_filters.test: vals1(i, j) = (i, i), (i, i+1), (i, i-1) for
    # i in 0 … 10; the 40 one-table queries `WHERE <i cmp constant> AND <j cmp i>` with their rows in
    # the order the file lists them. DuckDB pushes the constant comparison into the scan and keeps
    # the column-to-column comparison in a filter above it (the join queries are not taken).
    tf_src = (REF / "test/sql/filter/test_transitive_filters.test").read_text()
    for needle in ("CREATE TABLE vals1 AS SELECT i AS i, i AS j FROM range(0, 11, 1) t1(i)",
                   "INSERT INTO vals1 SELECT i, i+1 FROM vals1",
                   "INSERT INTO vals1 SELECT DISTINCT(i), i-1 FROM vals1 ORDER by i"):
        assert needle in tf_src, needle
    tf_rows = [[i, i] for i in range(11)] + [[i, i + 1] for i in range(11)] + [[i, i - 1] for i in range(11)]
    tf_q = []
    const_re = re.compile(r"^i(<=|>=|<|>|=)(-?\d+)$")
    col_re = re.compile(r"^j(<=|>=|<|>|=)i$")
    for where, body in re.findall(r"query II\nSELECT \* FROM vals1 WHERE ([^\n]*)\n----\n((?:[^\n]+\n?)*)", tf_src):
        terms = [x.strip() for x in where.split(" AND ")]
        c = [const_re.match(x) for x in terms if const_re.match(x)]
        r = [col_re.match(x) for x in terms if col_re.match(x)]
        assert len(c) == 1 and len(r) == 1, where
        rows = [[int(v) for v in line.split("\t")] for line in body.strip().split("\n") if line]
        tf_q.append({"where": where, "constant": [c[0].group(1), int(c[0].group(2))], "residual": r[0].group(1),
                     "rows": rows})
    assert len(tf_q) == 40, len(tf_q)
    tf = {"source": "test/sql/filter/test_transitive_filters.test", "rows": tf_rows, "queries": tf_q}
    # NULL-ness through updates (the validity column's update chain): the reference's NULL-update
    # tests as scripts, replayed against the version model in tests/sql_replay.py
    nu = {name: sqllogic_script(f"test/sql/update/{name}.test")
          for name in ("test_null_update", "null_update_merge", "null_update_merge_transaction",
                       "test_update_many_updaters_nulls", "update_null_integers")}
    # inserts, deletes and updates under concurrent transactions: the reference's MVCC scripts,
    # replayed by tests/sql_replay.py (insert / delete stamps and update records)
    mvcc = {Path(rel).stem: sqllogic_script(rel) for rel in (
        "test/sql/update/test_update_delete_same_tuple.test", "test/sql/update/update_after_commit.test",
        "test/sql/update/test_update_same_value.test", "test/sql/update/test_update.test",
        "test/sql/update/test_update_mix.test", "test/sql/update/test_update_many_updaters.test",
        "test/sql/update/test_cascading_updates.test", "test/sql/delete/test_truncate.test",
        "test/sql/delete/test_large_delete_parallel.test", "test/sql/transactions/test_multi_version.test",
        "test/sql/transactions/test_interleaved_versions.test", "test/sql/delete/test_delete.test",
        "test/sql/delete/test_large_delete.test", "test/sql/delete/large_deletes_transactions.test",
        "test/sql/delete/test_segment_deletes.test", "test/sql/transactions/test_multi_transaction_append.test",
        "test/sql/transactions/test_multi_version_large.test", "test/sql/transactions/test_null_version.test",
        "test/sql/transactions/test_transaction_local_data.test")}
    # VARCHAR update chains under concurrent transactions (replayed on dictionary codes,
    # tests/sql_replay.py encode_strings)
    smvcc = {Path(rel).stem: sqllogic_script(rel) for rel in (
        "test/sql/update/test_string_update.test", "test/sql/update/test_string_update_null.test",
        "test/sql/update/test_string_update_rollback.test", "test/sql/update/test_string_update_rollback_null.test",
        "test/sql/update/test_string_update_many_strings.test", "test/sql/update/test_repeated_string_update.test",
        "test/sql/update/test_update_same_string_value.test")}
    (OUT / "reference_cases.json").write_text(json.dumps({"null_updates": nu, "mvcc_scripts": mvcc, "string_mvcc_scripts": smvcc, "transitive_filters": tf, "zonemap_segment": zm, "interleaved_versions": iv,
                                                          "timestamp_date_pushdown": tsd, "rle_cases": rle,
                                                          "table_or_pushdown": orp, "update": upd,
                                                          "table_filter_pushdown": tfp, "multi_version": mv,
                                                          "concurrent_reads_while_updating": cr,
                                                          "many_updaters": mu, "block_boundary_update": bb,
                                                          "zonemap_or_trees": zt, "obsolete_filters": ob, "filter_cache": fc,
                                                          "art_scans": art},
                                                         indent=1, sort_keys=True) + "\n")


if __name__ == "__main__":
    main()
