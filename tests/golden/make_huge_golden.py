"""Extract the reference's table-filter cases on HUGEINT / UHUGEINT columns into
tests/golden/huge_filter_cases.json: the pushed comparisons and NULL tests of
test/sql/types/{hugeint,uhugeint}/test_*_ops.test, test_*_null_value.test and
test/sql/storage/types/test_*_storage.test. Run in the build container (where /root/reference
exists); the JSON is data only: each table's column types and inserted rows (values as decimal
strings, NULL as null) and, per query, its SQL, the filtered column's comparison (operator and the
constant as a decimal string, or IS NULL), what the query selects and its expected rows, exactly as
the files state them.

The semantics these pin are FilterSelectionSwitch<hugeint_t / uhugeint_t> (src/storage/table/
column_segment.cpp:468-479) with hugeint_t's / uhugeint_t's comparison operators."""
import json
import re
from pathlib import Path

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent / "huge_filter_cases.json"
FILES = [f"test/sql/types/{t}/test_{t}_ops.test" for t in ("hugeint", "uhugeint")] + \
        [f"test/sql/types/{t}/test_{t}_null_value.test" for t in ("hugeint", "uhugeint")] + \
        [f"test/sql/storage/types/test_{t}_storage.test" for t in ("hugeint", "uhugeint")]
CMP = r"(=|<>|>=|<=|>|<)"
WHERE = re.compile(r"^SELECT (.+?) FROM (\w+) WHERE h\s*(?:" + CMP + r"\s*(\S+?)|(IS NULL))(\s+ORDER BY 1)?(\s+GROUP BY id)?;?$")


def literal(tok):
    """A value as the file writes it: 42, 42::HUGEINT, '1267...'::UHUGEINT, 100::UINTEGER, NULL."""
    tok = tok.strip()
    if tok.upper() == "NULL":
        return None
    tok = re.sub(r"::\w+$", "", tok).strip("'")
    assert re.fullmatch(r"-?\d+", tok), tok
    return tok


def tuples(values_sql):
    return [[literal(v) for v in tup.split(",")] for tup in re.findall(r"\(([^()]*(?:\([^)]*\))?[^()]*)\)", values_sql)]


def cases(rel):
    src = (REF / rel).read_text()
    table, columns, types, rows, queries = None, None, None, [], []
    for block in re.split(r"\n\s*\n", src):
        lines = [x for x in block.strip().split("\n") if x and not x.startswith("#")]
        if not lines:
            continue
        head = lines[0].split()
        body = " ".join(lines[1:])
        if head[0] == "statement":
            m = re.match(r"CREATE TABLE (\w+)\s*\((.*)\);?$", body)
            if m and table is None:
                table = m.group(1)
                columns = [c.split()[0] for c in m.group(2).split(",")]
                types = [c.split()[1] for c in m.group(2).split(",")]
            m = re.match(rf"INSERT INTO {table} VALUES (.*?);?$", body) if table else None
            if m:
                rows += tuples(m.group(1))
        elif head[0] == "query" and table:
            sep = lines.index("----") if "----" in lines else len(lines)
            sql = " ".join(lines[1:sep])
            m = WHERE.match(sql)
            if not m or m.group(2) != table:
                continue
            q = {"sql": sql, "select": m.group(1), "rows": [x.strip() for x in lines[sep + 1:]]}
            if m.group(5):
                q["cmp"], q["constant"] = "IS NULL", None
            else:
                q["cmp"], q["constant"] = m.group(3), literal(m.group(4))
            queries.append(q)
    assert table and rows and queries, rel
    return {"file": rel, "table": table, "columns": columns, "types": types, "rows": rows, "queries": queries}


def main():
    out = {"what": "table filters on HUGEINT / UHUGEINT columns: inserted rows and each pushed comparison's "
                   "expected rows, as the reference's tests state them",
           "generator": "tests/golden/make_huge_golden.py",
           "cases": [cases(f) for f in FILES]}
    OUT.write_text(json.dumps(out, indent=1) + "\n")
    print(f"wrote {sum(len(c['queries']) for c in out['cases'])} queries to {OUT}")


if __name__ == "__main__":
    main()
