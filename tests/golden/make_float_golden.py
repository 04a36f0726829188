"""Extract the reference's table-filter cases on FLOAT / DOUBLE columns — the pushed comparisons
of test/sql/types/float/nan_test.test and infinity_test.test, each run under
`foreach type FLOAT DOUBLE` — into tests/golden/float_filter_cases.json. Run in the build
container (where /root/reference exists); the JSON is data only: the values each file inserts
and, per query, its comparison, constant and expected rows, exactly as the files state them
(values as the files print them: 'nan', 'inf', '-inf', '1').

The semantics these pin (NaN equal to NaN and greater than everything, src/common/
vector_operations/comparison_operators.cpp:17-88) are those of FilterSelectionSwitch<float /
double> (src/storage/table/column_segment.cpp:278-349)."""
import json
import re
from pathlib import Path

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent / "float_filter_cases.json"
FILES = ["test/sql/types/float/nan_test.test", "test/sql/types/float/infinity_test.test"]
QUERY = re.compile(r"SELECT f FROM floats WHERE f\s*(=|<>|>=|<=|>|<)\s*(\S+?)(\s+ORDER BY .*)?$")


def constant(tok):
    m = re.fullmatch(r"'(-?\w+)'::\$\{type\}", tok)
    return m.group(1).lower() if m else tok  # 'nan' / 'inf' / '-inf', or a number as written


def cases(rel):
    src = (REF / rel).read_text()
    inserted, queries = None, []
    for block in re.split(r"\n\s*\n", src):
        lines = [x for x in block.strip().split("\n") if x and not x.startswith("#")]
        if not lines:
            continue
        head = lines[0].split()
        if head[0] == "statement" and lines[1].startswith("INSERT INTO floats VALUES"):
            inserted = [v.strip("()' ").lower() for v in lines[1].split("VALUES", 1)[1].split("),")]
        elif head[0] == "query":
            sql = " ".join(lines[1:lines.index("----")]) if "----" in lines else " ".join(lines[1:])
            m = QUERY.match(sql)
            if not m:
                continue
            sep = lines.index("----") if "----" in lines else len(lines)
            queries.append({"cmp": m.group(1), "constant": constant(m.group(2)),
                            "rows": [x.strip() for x in lines[sep + 1:]], "sql": sql})
    assert inserted and queries, rel
    return {"file": rel, "types": ["FLOAT", "DOUBLE"], "inserted": inserted, "queries": queries}


ORDERING = "test/sql/types/float/nan_ordering.test"


def ordering_case():
    """nan_ordering.test: the rows inserted as [value, repeat] runs in order (the range insert is
    one run of 10,000 zeros), the
    `SELECT f FROM floats ORDER BY f` result (NULLs first) and the filtered counts after the
    range insert, as the file states them."""
    src = (REF / ORDERING).read_text()
    inserts, order, counts = [], None, []
    for block in re.split(r"\n\s*\n", src):
        lines = [x for x in block.strip().split("\n") if x and not x.startswith("#")]
        if not lines:
            continue
        body = " ".join(lines[1:])
        if lines[0].startswith("statement") and body.startswith("INSERT INTO floats VALUES"):
            inserts += [[v.strip("()' ").lower().replace("::${type}", "").strip("'"), 1]
                        for v in body.split("VALUES", 1)[1].split("),")]
        elif lines[0].startswith("statement") and body.startswith("INSERT INTO floats SELECT"):
            m = re.match(r"INSERT INTO floats SELECT '(\S+)'::\$\{type\} FROM range\((\d+)\)", body)
            inserts.append([m.group(1), int(m.group(2))])
        elif lines[0].startswith("query") and "----" in lines:
            sep = lines.index("----")
            sql = " ".join(lines[1:sep])
            rows = [x.strip() for x in lines[sep + 1:]]
            if sql == "SELECT f FROM floats ORDER BY f" and order is None:
                order = rows
            m = re.match(r"SELECT COUNT\(\*\) FROM floats WHERE f (>|<) (\S+)$", sql)
            if m:
                counts.append({"cmp": m.group(1), "constant": m.group(2), "count": int(rows[0]), "sql": sql,
                               "rows_inserted_before": sum(k for _, k in inserts)})
    assert order and counts
    return {"file": ORDERING, "types": ["FLOAT", "DOUBLE"], "inserted": inserts, "order_by_f": order,
            "counts": counts}


def main():
    out = {"what": "table filters on FLOAT / DOUBLE columns holding NaN and ±inf: inserted values and each "
                   "pushed comparison's expected rows, as the reference's tests state them (each test runs "
                   "for both types)",
           "generator": "tests/golden/make_float_golden.py",
           "cases": [cases(f) for f in FILES],
           "ordering": ordering_case()}
    OUT.write_text(json.dumps(out, indent=1) + "\n")
    print(f"wrote {sum(len(c['queries']) for c in out['cases'])} queries to {OUT}")


if __name__ == "__main__":
    main()
