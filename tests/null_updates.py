"""Replay of the reference's NULL-update tests (tests/golden/reference_cases.json "null_updates":
test/sql/update/test_null_update.test, null_update_merge.test, null_update_merge_transaction.test,
test_update_many_updaters_nulls.test, update_null_integers.test) as version state.

Test infrastructure: this is the SQL layer around the scan — it runs each script's INSERTs into
base columns and turns each UPDATE into update records (row, value, valid, version) the way
DuckDB's UpdateSegment chains them (one record per updated row of the column; the value chain
and the validity chain written together, update_segment.cpp:588-600, 1074-1199): a record carries
its writer's transaction id until COMMIT re-stamps it with a commit id, ROLLBACK removes it, and a
row already updated by a version the writer cannot see is a conflict (the statement fails and
changes nothing, update_segment.cpp CheckForConflicts). It then hands every query of the script
to the caller as (snapshot, columns, records), and the caller answers it with the oracle or with
the GPU. Its own answer (`Query.view`) is checked against the file's expected rows first, so the
record lists it produces are pinned by the reference's outputs.

Transaction timing follows DuckDB: start times and commit ids come from one increasing counter; a
transaction sees a version v when v < start_time or v == its transaction id
(TransactionVersionOperator::UseInsertedVersion, chunk_info.cpp:11-14); BEGIN takes the snapshot
immediately under immediate_transaction_mode, otherwise at its first statement; a statement
outside BEGIN is its own transaction.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

TXN_START = 4611686018427388000  # TRANSACTION_ID_START (src/include/duckdb/common/constants.hpp)


# ------------------------------------------------------------------ a tiny SQL expression evaluator

_TOK = re.compile(r"\s*(<=|>=|<>|!=|=|<|>|\(|\)|,|\d+|[A-Za-z_][A-Za-z_0-9]*)")


def _tokens(s: str) -> List[str]:
    out, i = [], 0
    s = s.strip().rstrip(";")
    while i < len(s):
        m = _TOK.match(s, i)
        if not m:
            raise ValueError(f"cannot tokenize {s[i:]!r}")
        out.append(m.group(1))
        i = m.end()
    return out


class _Parser:
    """expr := CASE WHEN cond THEN expr ELSE expr END | NULL | int | column | ( expr )
    cond := pred (AND pred)*; pred := expr op expr | expr IS [NOT] NULL — SQL three-valued
    logic (None = unknown)."""

    def __init__(self, toks):
        self.t, self.i = toks, 0

    def peek(self, k=0):
        return self.t[self.i + k].upper() if self.i + k < len(self.t) else None

    def take(self, want=None):
        tok = self.t[self.i]
        if want is not None and tok.upper() != want:
            raise ValueError(f"expected {want}, got {tok}")
        self.i += 1
        return tok

    def expr(self):
        p = self.peek()
        if p == "CASE":
            self.take("CASE")
            self.take("WHEN")
            c = self.cond()
            self.take("THEN")
            a = self.expr()
            self.take("ELSE")
            b = self.expr()
            self.take("END")
            return lambda row: a(row) if c(row) is True else b(row)
        if p == "NULL":
            self.take()
            return lambda row: None
        if p == "(":
            self.take("(")
            e = self.expr()
            self.take(")")
            return e
        tok = self.take()
        if tok.isdigit():
            v = int(tok)
            return lambda row: v
        name = tok.lower()
        return lambda row: row[name]

    def pred(self):
        a = self.expr()
        if self.peek() == "IS":
            self.take("IS")
            neg = self.peek() == "NOT"
            if neg:
                self.take("NOT")
            self.take("NULL")
            return lambda row: (a(row) is not None) if neg else (a(row) is None)
        op = self.take()
        b = self.expr()
        f = {"=": lambda x, y: x == y, "!=": lambda x, y: x != y, "<>": lambda x, y: x != y,
             "<": lambda x, y: x < y, "<=": lambda x, y: x <= y, ">": lambda x, y: x > y,
             ">=": lambda x, y: x >= y}[op]

        def ev(row):
            x, y = a(row), b(row)
            return None if x is None or y is None else f(x, y)
        return ev

    def cond(self):
        parts = [self.pred()]
        while self.peek() == "AND":
            self.take("AND")
            parts.append(self.pred())

        def ev(row):
            vals = [p(row) for p in parts]
            if any(v is False for v in vals):
                return False
            return None if any(v is None for v in vals) else True
        return ev


def parse_expr(s: str):
    p = _Parser(_tokens(s))
    e = p.expr()
    assert p.i == len(p.t), s
    return e


def parse_cond(s: str):
    p = _Parser(_tokens(s))
    c = p.cond()
    assert p.i == len(p.t), s
    return c


# ------------------------------------------------------------------ version state

@dataclass
class Txn:
    tid: int
    start: Optional[int] = None  # None until the snapshot is taken
    explicit: bool = False
    commit: Optional[int] = None


@dataclass
class Record:
    col: str
    row: int
    value: int
    valid: bool
    owner: Txn

    @property
    def version(self) -> int:
        return self.owner.commit if self.owner.commit is not None else self.owner.tid


def visible(version: int, txn: Txn) -> bool:
    return version < txn.start or version == txn.tid


@dataclass
class Query:
    """One query of the script: who asks (connection, snapshot), the SQL and the expected rows,
    with the table's base columns and update records at that moment."""
    con: str
    sql: str
    rows: list
    start: int
    tid: int
    columns: List[str]
    base: Dict[str, List[Optional[int]]]
    records: Dict[str, list]  # column -> [(row, value, valid, version)], per row chronological
    view: List[Dict[str, Optional[int]]] = field(default_factory=list)  # the model's rows for the txn
    committed_horizon: int = 0  # every committed version is below it

    def update_arrays(self, col: str):
        """(rows, values, versions, valid) of a column's records, grouped by row (stable)."""
        recs = sorted(self.records.get(col, []), key=lambda r: r[0])
        return (np.array([r[0] for r in recs], np.int64), np.array([r[1] for r in recs], np.int64),
                np.array([r[3] for r in recs], np.uint64), np.array([r[2] for r in recs], bool))


class Replay:
    def __init__(self, case: dict):
        self.case = case
        self.clock = 1
        self.next_tid = TXN_START + 1
        self.cols: List[str] = []
        self.table = ""
        self.base: Dict[str, List[Optional[int]]] = {}
        self.records: List[Record] = []
        self.active: Dict[str, Txn] = {}

    def tick(self) -> int:
        self.clock += 1
        return self.clock

    def new_txn(self, explicit: bool) -> Txn:
        t = Txn(self.next_tid, explicit=explicit)
        self.next_tid += 1
        return t

    def snapshot(self, t: Txn):
        if t.start is None:
            t.start = self.tick()

    def view(self, t: Txn) -> List[Dict[str, Optional[int]]]:
        n = len(self.base[self.cols[0]]) if self.cols else 0
        rows = [{c: self.base[c][r] for c in self.cols} for r in range(n)]
        for rec in self.records:  # chronological: the newest visible record wins
            if visible(rec.version, t):
                rows[rec.row][rec.col] = rec.value if rec.valid else None
        return rows

    # ---- statements
    def create(self, sql):
        m = re.match(r"CREATE TABLE (\w+)\s*\((.*)\)", sql.rstrip(";"), re.I)
        self.table = m.group(1)
        self.cols = [c.strip().split()[0].lower() for c in m.group(2).split(",")]
        self.base = {c: [] for c in self.cols}

    def insert(self, sql):
        m = re.match(r"INSERT INTO \w+ VALUES (.*)$", sql.rstrip(";"), re.I)
        if m:
            for tup in re.findall(r"\(([^)]*)\)", m.group(1)):
                vals = [None if v.strip().upper() == "NULL" else int(v) for v in tup.split(",")]
                for c, v in zip(self.cols, vals):
                    self.base[c].append(v)
            return
        m = re.match(r"INSERT INTO \w+ SELECT (\w+), NULL FROM range\((\d+)\) tbl\((\w+)\)", sql.rstrip(";"), re.I)
        assert m and m.group(1) == m.group(3) and len(self.cols) == 2, sql
        for v in range(int(m.group(2))):
            self.base[self.cols[0]].append(v)
            self.base[self.cols[1]].append(None)

    def update(self, sql, t: Txn):
        m = re.match(r"UPDATE \w+ SET (\w+)\s*=\s*(.*?)(?: WHERE (.*))?$", sql.rstrip(";"), re.I | re.S)
        col, expr, where = m.group(1).lower(), parse_expr(m.group(2)), m.group(3)
        cond = parse_cond(where) if where else (lambda row: True)
        rows = self.view(t)
        new = []
        for r, row in enumerate(rows):
            if cond(row) is not True:
                continue
            for rec in self.records:  # a version the writer cannot see on this row: conflict
                if rec.col == col and rec.row == r and not visible(rec.version, t):
                    return None
            v = expr(row)
            new.append(Record(col, r, 0 if v is None else v, v is not None, t))
        self.records += new
        return len(new)

    def finish(self, t: Txn, commit: bool):
        if commit:
            t.commit = self.tick()
        else:
            self.records = [r for r in self.records if r.owner is not t]

    def query_state(self, con, sql, rows, t: Txn) -> Query:
        recs: Dict[str, list] = {}
        for rec in self.records:
            recs.setdefault(rec.col, []).append((rec.row, rec.value, rec.valid, rec.version))
        return Query(con, sql, rows, t.start, t.tid, list(self.cols), {c: list(v) for c, v in self.base.items()},
                     recs, self.view(t), self.clock + 1)

    def run(self):
        """Yields a Query per `query` of the script (UPDATE-as-query and SELECTs)."""
        imm = self.case["immediate_transaction_mode"]
        for step in self.case["script"]:
            con, sql = step["con"], step["sql"].strip()
            up = sql.upper()
            if up.startswith("CREATE TABLE"):
                self.create(sql)
                continue
            if up.startswith("INSERT"):
                self.insert(sql)
                continue
            if up.startswith("SET ") or up.startswith("CHECKPOINT"):
                continue
            if up.startswith("BEGIN"):
                t = self.new_txn(True)
                if imm:
                    self.snapshot(t)
                self.active[con] = t
                continue
            if up in ("COMMIT", "ROLLBACK"):
                self.finish(self.active.pop(con), up == "COMMIT")
                continue
            t = self.active.get(con) or self.new_txn(False)
            self.snapshot(t)
            if up.startswith("UPDATE"):
                n = self.update(sql, t)
                ok = n is not None
                if step["op"] == "statement":
                    assert ok == step["ok"], (sql, con)
                else:
                    assert ok and [[n]] == step["rows"], (sql, n, step["rows"])
                if not t.explicit:
                    self.finish(t, ok)
                elif not ok:  # a failed statement aborts its transaction
                    self.finish(self.active.pop(con), False)
                continue
            assert step["op"] == "query", sql
            yield self.query_state(con, sql, step["rows"], t)
            if not t.explicit:
                self.finish(t, True)


# ------------------------------------------------------------------ answering a query from a view

def order_key(nulls_first: bool):
    def k(v):
        return (0 if nulls_first else 1, 0) if v is None else (1 if nulls_first else 0, v)
    return k


def answer(q: Query, view: List[Dict[str, Optional[int]]], nulls_first: bool):
    """The rows the query returns over a view (rows as {column: value or None})."""
    sql = q.sql.strip().rstrip(";")
    m = re.match(r"SELECT \* FROM \w+ ORDER BY (\w+)$", sql, re.I)
    if m:
        key = order_key(nulls_first)
        rows = sorted(view, key=lambda r: key(r[m.group(1).lower()]))
        return [[r[c] for c in q.columns] for r in rows]
    m = re.match(r"SELECT COUNT\(\*\) FROM \w+ WHERE (.*)$", sql, re.I)
    if m:
        c = parse_cond(m.group(1))
        return [[sum(1 for r in view if c(r) is True)]]
    m = re.match(r"select COUNT\((\w+)\), MIN\(\w+\), MAX\(\w+\) from \w+$", sql, re.I)
    if m:
        vals = [r[m.group(1).lower()] for r in view if r[m.group(1).lower()] is not None]
        return [[len(vals), min(vals) if vals else None, max(vals) if vals else None]]
    raise ValueError(f"query shape not modelled: {sql}")


def cases(golden):
    return golden["cases"]["null_updates"]


def queries(case: dict):
    return list(Replay(case).run())
