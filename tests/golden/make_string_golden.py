"""Extract the reference's table-filter cases on VARCHAR columns into
tests/golden/string_filter_cases.json: the strtest queries of test/sql/projection/
test_complex_expressions.test (one comparison each) and the strings queries of
test/sql/filter/test_obsolete_filters.test (two comparisons on one column, folded by the filter
combiner). Run in the build container (where /root/reference exists); the JSON is data only: each
table's inserted rows (NULL as null) and, per query, the pushed comparisons (operator, string
literal), the projected column and the expected rows, exactly as the files state them.

The semantics these pin are FilterSelectionSwitch<string_t> (src/storage/table/
column_segment.cpp:278-349) with string_t's operators (src/include/duckdb/common/types/
string_type.hpp:143-206)."""
import json
import re
from pathlib import Path

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent / "string_filter_cases.json"
FILES = {"test/sql/projection/test_complex_expressions.test": "strtest",
         "test/sql/filter/test_obsolete_filters.test": "strings"}
CMP = r"(=|<>|>=|<=|>|<)"
TERM = re.compile(r"(\w+)\s*" + CMP + r"\s*'([^']*)'$")
QUERY = re.compile(r"SELECT (\*|\w+) FROM (\w+) WHERE (.+)$")


def tuples(values_sql):
    out = []
    for tup in re.findall(r"\(([^)]*)\)", values_sql):
        row = []
        for v in tup.split(","):
            v = v.strip()
            row.append(None if v.upper() == "NULL" else v.strip("'"))
        out.append(row)
    return out


def cases(rel, table):
    src = (REF / rel).read_text()
    columns, rows, queries = None, [], []
    for block in re.split(r"\n\s*\n", src):
        lines = [x for x in block.strip().split("\n") if x and not x.startswith("#")]
        if not lines:
            continue
        head = lines[0].split()
        body = " ".join(lines[1:])
        if head[0] == "statement":
            m = re.match(rf"CREATE TABLE {table}\s*\((.*)\)$", body)
            if m:
                columns = [c.split()[0] for c in m.group(1).split(",")]
            m = re.match(rf"INSERT INTO {table} VALUES (.*)$", body)
            if m:
                rows += tuples(m.group(1))
        elif head[0] == "query" and columns:
            sep = lines.index("----") if "----" in lines else len(lines)
            sql = " ".join(lines[1:sep])
            m = QUERY.match(sql)
            if not m or m.group(2) != table:
                continue
            terms = [TERM.match(t.strip()) for t in m.group(3).split(" AND ")]
            if not all(terms) or len({t.group(1) for t in terms}) != 1:
                continue
            queries.append({"column": columns.index(terms[0].group(1)),
                            "terms": [[t.group(2), t.group(3)] for t in terms],
                            "project": None if m.group(1) == "*" else columns.index(m.group(1)),
                            "rows": [x.strip() for x in lines[sep + 1:]], "sql": sql})
    assert columns and rows and queries, rel
    return {"file": rel, "table": table, "columns": columns, "rows": rows, "queries": queries}


def main():
    out = {"what": "table filters on VARCHAR columns: each table's inserted rows and each query's pushed "
                   "comparisons (operator, string literal), projected column and expected rows, as the "
                   "reference's tests state them",
           "generator": "tests/golden/make_string_golden.py",
           "cases": [cases(f, t) for f, t in FILES.items()]}
    OUT.write_text(json.dumps(out, indent=1) + "\n")
    print(f"wrote {sum(len(c['queries']) for c in out['cases'])} queries to {OUT}")


if __name__ == "__main__":
    main()
