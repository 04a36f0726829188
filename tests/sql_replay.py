"""Replay of the reference's MVCC sqllogictests as version state — the SQL layer around the scan,
as test infrastructure (fixtures: tests/golden/reference_cases.json "null_updates" and "mvcc_scripts",
extracted by tests/golden/make_golden.py).

Files replayed: test/sql/update/{test_null_update, null_update_merge, null_update_merge_transaction,
test_update_many_updaters_nulls, update_null_integers, test_update_delete_same_tuple,
update_after_commit, test_update_same_value, test_update, test_update_mix, test_update_many_updaters,
test_cascading_updates}.test; test/sql/delete/{test_delete, test_large_delete,
large_deletes_transactions, test_segment_deletes, test_truncate, test_large_delete_parallel}.test;
test/sql/transactions/{test_multi_transaction_append, test_multi_version_large, test_null_version,
test_transaction_local_data, test_multi_version, test_interleaved_versions}.test.

The replay records each statement the way DuckDB's version machinery does:
* INSERT appends rows stamped with the inserting transaction's id (ChunkVectorInfo::Append,
  chunk_info.cpp:123-161); COMMIT re-stamps them with the commit id (CommitAppend); ROLLBACK leaves
  them stamped with an id no snapshot sees;
* DELETE stamps each deleted row with the deleter's id (ChunkVectorInfo::Delete,
  chunk_info.cpp:181-202): a row already stamped by another transaction is a conflict;
* UPDATE appends (row, value, valid, version) records per updated row of each assigned column — the
  value chain and the validity chain together (update_segment.cpp:588-600, 1074-1199): a record of
  that row and column the writer cannot see is a conflict. An UPDATE and a DELETE of one row by two
  transactions do not conflict (test_update_delete_same_tuple.test).
Start times and commit ids come from one increasing counter; a transaction sees a version v when
v < start_time or v == its transaction id (TransactionVersionOperator::UseInsertedVersion,
chunk_info.cpp:11-14). BEGIN takes the snapshot at once under immediate_transaction_mode, else at the
transaction's first statement; a statement outside BEGIN is its own transaction. A failed statement
inside BEGIN aborts the transaction (its effects are dropped) and the COMMIT or ROLLBACK that
follows ends it; TRUNCATE is a DELETE of every row; CHECKPOINT is left to the tests (a merge).

Each SELECT is handed to the caller as a `Query`: the snapshot and the whole version state at that
moment (every row ever appended with its insert and delete stamps, and the update records). The
caller answers it with the oracle or the GPU; the replay's own answer (`Query.view`) is checked
against the file's rows first, so the state it hands over is pinned by the reference's outputs.
Columns are numpy (values, valid) pairs throughout — the scripts reach a million rows.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np

TXN_START = 4611686018427388000  # TRANSACTION_ID_START (src/include/duckdb/common/constants.hpp)
NOT_DELETED = 2 ** 64 - 2  # NOT_DELETED_ID (src/common/constants.cpp:16); also a rolled-back insert's stamp

Frame = Dict[str, tuple]  # column -> (int64 values, bool valid); "rowid" -> (int64 ids, all True)


# ------------------------------------------------------------------ a small vectorised SQL evaluator

_TOK = re.compile(r"\s*(<=|>=|<>|!=|=|<|>|\(|\)|,|\+|-|%|\*|\d+|[A-Za-z_][A-Za-z_0-9]*)")


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


def _const(v):
    def ev(f: Frame):
        n = len(f["rowid"][0])
        return np.full(n, 0 if v is None else v, np.int64), np.full(n, v is not None)
    return ev


def _arith(a, b, op):
    def ev(f):
        (x, xo), (y, yo) = a(f), b(f)
        ok = xo & yo
        if op == "+":
            v = x + y
        elif op == "-":
            v = x - y
        elif op == "*":
            v = x * y
        else:  # integer modulo keeps the dividend's sign (C semantics); x % 0 is NULL
            ok = ok & (y != 0)
            v = np.fmod(x, np.where(y == 0, 1, y))
        return np.where(ok, v, 0), ok
    return ev


class _Parser:
    """expr := term (('+'|'-') term)*; term := atom (('*'|'%') atom)*;
    atom := CASE WHEN cond THEN expr ELSE expr END | NULL | int | column | ( expr ) | - atom;
    cond := pred (AND pred)*; pred := expr op expr | expr IS [NOT] NULL.
    An expression evaluates to (values, valid) over a Frame; a condition to (true, unknown) masks —
    SQL's three-valued logic."""

    def __init__(self, toks):
        self.t, self.i = toks, 0

    def peek(self):
        return self.t[self.i].upper() if self.i < len(self.t) else None

    def take(self, want=None):
        tok = self.t[self.i]
        if want is not None and tok.upper() != want:
            raise ValueError(f"expected {want}, got {tok}")
        self.i += 1
        return tok

    def atom(self):
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

            def ev(f):
                t, _ = c(f)
                (x, xo), (y, yo) = a(f), b(f)
                return np.where(t, x, y), np.where(t, xo, yo)
            return ev
        if p == "NULL":
            self.take()
            return _const(None)
        if p == "(":
            self.take("(")
            e = self.expr()
            self.take(")")
            return e
        if p == "-":
            self.take("-")
            return _arith(_const(0), self.atom(), "-")
        tok = self.take()
        if tok.isdigit():
            return _const(int(tok))
        name = tok.lower()
        return lambda f: f[name]

    def term(self):
        a = self.atom()
        while self.peek() in ("*", "%"):
            op = self.take()
            a = _arith(a, self.atom(), op)
        return a

    def expr(self):
        a = self.term()
        while self.peek() in ("+", "-"):
            op = self.take()
            a = _arith(a, self.term(), op)
        return a

    def pred(self):
        a = self.expr()
        if self.peek() == "IS":
            self.take("IS")
            neg = self.peek() == "NOT"
            if neg:
                self.take("NOT")
            self.take("NULL")

            def isnull(f):
                _, ok = a(f)
                return (ok if neg else ~ok), np.zeros(len(ok), bool)
            return isnull
        op = self.take()
        b = self.expr()
        cmp = {"=": np.equal, "!=": np.not_equal, "<>": np.not_equal, "<": np.less, "<=": np.less_equal,
               ">": np.greater, ">=": np.greater_equal}[op]

        def ev(f):
            (x, xo), (y, yo) = a(f), b(f)
            ok = xo & yo
            return ok & cmp(x, y), ~ok
        return ev

    def cond(self):
        parts = [self.pred()]
        while self.peek() == "AND":
            self.take("AND")
            parts.append(self.pred())

        def ev(f):
            res = [p(f) for p in parts]
            false = np.zeros(len(f["rowid"][0]), bool)
            for t, u in res:
                false |= ~t & ~u
            t_all = np.logical_and.reduce([t for t, _ in res])
            return t_all, ~t_all & ~false
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


_SIMPLE = re.compile(r"^\s*(\w+)\s*(<=|>=|<>|!=|=|<|>)\s*(-?\d+)\s*$|^\s*(\w+)\s+IS\s+(NOT\s+)?NULL\s*$", re.I)


def simple_terms(where: Optional[str]):
    """The WHERE as an AND of (column, op, constant) / (column, 'IS NULL' | 'IS NOT NULL', None)
    terms — the shape DuckDB pushes into the scan as a TableFilterSet — or None for another shape."""
    if not where:
        return []
    out = []
    for part in re.split(r"\s+AND\s+", where.strip().rstrip(";"), flags=re.I):
        m = _SIMPLE.match(part)
        if not m:
            return None
        if m.group(1):
            out.append((m.group(1).lower(), m.group(2), int(m.group(3))))
        else:
            out.append((m.group(4).lower(), "IS NOT NULL" if m.group(5) else "IS NULL", None))
    return out


# ------------------------------------------------------------------ frames

def frame_take(f: Frame, mask) -> Frame:
    return {k: (v[mask], ok[mask]) for k, (v, ok) in f.items()}


def frame_equal(a: Frame, b: Frame) -> bool:
    """Same keys, same NULL-ness, same values where valid."""
    return a.keys() == b.keys() and all(
        np.array_equal(a[k][1], b[k][1]) and np.array_equal(np.where(a[k][1], a[k][0], 0), np.where(b[k][1], b[k][0], 0))
        for k in a)


def frame_rows(f: Frame, columns: List[str]) -> List[list]:
    cols = [(f[c][0].tolist(), f[c][1].tolist()) for c in columns]
    n = len(f["rowid"][0])
    return [[(v[i] if ok[i] else None) for v, ok in cols] for i in range(n)]


# ------------------------------------------------------------------ version state

@dataclass(eq=False)
class Txn:
    tid: int
    start: Optional[int] = None  # None until the snapshot is taken
    explicit: bool = False
    commit: Optional[int] = None
    aborted: bool = False

    @property
    def version(self) -> int:
        if self.aborted:
            return NOT_DELETED
        return self.commit if self.commit is not None else self.tid


def visible(version, start: int, tid: int):
    v = np.asarray(version, np.uint64)
    return (v < np.uint64(start)) | (v == np.uint64(tid))


@dataclass
class Query:
    """One SELECT of a script: who asks (connection, snapshot), the SQL and the expected rows, and
    the table at that moment — every row ever appended (base values; insert stamp per row, 0 =
    before every snapshot; delete stamp per row, NOT_DELETED = none) and the update records."""
    con: str
    sql: str
    rows: list
    start: int
    tid: int
    columns: List[str]
    base: Dict[str, tuple]          # column -> (int64 values, bool valid), one per row ever appended
    inserted: np.ndarray            # uint64 per row
    deleted: np.ndarray             # uint64 per row
    records: Dict[str, list]        # column -> [(rows, values, valid, version)] batches, chronological
    view: Frame                     # the replay's own answer: the visible rows, with "rowid"
    horizon: int = 0                # the oldest snapshot still open: a checkpoint may merge below it

    @property
    def n_rows(self) -> int:
        return len(self.inserted)

    def update_arrays(self, col: str):
        """(rows, values, versions, valid) of a column's records, grouped by row, chronological within
        a row (the order cubit_table_set_updates takes)."""
        batches = self.records.get(col, [])
        if not batches:
            return np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.uint64), np.zeros(0, bool)
        rows = np.concatenate([b[0] for b in batches])
        vals = np.concatenate([b[1] for b in batches])
        ok = np.concatenate([b[2] for b in batches])
        vers = np.concatenate([np.full(len(b[0]), b[3], np.uint64) for b in batches])
        o = np.argsort(rows, kind="stable")
        return rows[o], vals[o], vers[o], ok[o]

    def insert_ranges(self):
        """Runs of consecutive rows with one insert stamp other than 0: (begins, ends, ids)."""
        ins = self.inserted
        if len(ins) == 0:
            return np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.uint64)
        cut = np.flatnonzero(ins[1:] != ins[:-1]) + 1
        b = np.concatenate([[0], cut])
        e = np.concatenate([cut, [len(ins)]])
        keep = ins[b] != 0
        return b[keep].astype(np.int64), e[keep].astype(np.int64), ins[b[keep]]

    def delete_arrays(self):
        rows = np.flatnonzero(self.deleted != NOT_DELETED).astype(np.int64)
        return rows, self.deleted[rows]


class Replay:
    def __init__(self, case: dict):
        self.case = case
        self.clock = 1
        self.next_tid = TXN_START + 1
        self.cols: List[str] = []
        self.vals: Dict[str, np.ndarray] = {}
        self.valid: Dict[str, np.ndarray] = {}
        self.txns: List[Txn] = []
        self.ins = np.zeros(0, np.int64)   # per row: owner index into txns, -1 = before every snapshot
        self.dels = np.zeros(0, np.int64)  # per row: deleter index into txns, -1 = none
        self.records: List[tuple] = []     # (col, rows, values, valid, owner index), chronological
        self.active: Dict[str, Txn] = {}
        self.started = False  # a snapshot has been taken: later inserts are versioned

    def tick(self) -> int:
        self.clock += 1
        return self.clock

    def new_txn(self, explicit: bool) -> Txn:
        t = Txn(self.next_tid, explicit=explicit)
        self.next_tid += 1
        self.txns.append(t)
        return t

    def snapshot(self, t: Txn):
        if t.start is None:
            t.start = self.tick()
            self.started = True

    def versions(self, owners: np.ndarray, none_value: int) -> np.ndarray:
        tv = np.array([t.version for t in self.txns] + [none_value], np.uint64)
        return tv[np.where(owners < 0, len(self.txns), owners)]

    def seen(self, owner: int, t: Txn) -> bool:
        return bool(visible(self.txns[owner].version, t.start, t.tid))

    def view(self, t: Txn) -> Frame:
        live = visible(self.versions(self.ins, 0), t.start, t.tid) & \
            ~visible(self.versions(self.dels, NOT_DELETED), t.start, t.tid)
        f = {c: (self.vals[c].copy(), self.valid[c].copy()) for c in self.cols}
        for col, rows, vals, ok, owner in self.records:  # chronological: the newest visible record wins
            if self.seen(owner, t):
                f[col][0][rows] = vals
                f[col][1][rows] = ok
        n = len(self.ins)
        f["rowid"] = (np.arange(n, dtype=np.int64), np.ones(n, bool))
        return frame_take(f, live)

    # ---- statements
    def create(self, sql):
        s = sql.rstrip(";")
        m = re.match(r"CREATE TABLE \w+\s*AS SELECT \* FROM range\((\d+)(?:,\s*(\d+)(?:,\s*1)?)?\)\s*\w+\((\w+)\)", s, re.I)
        if m:
            lo, hi = (0, int(m.group(1))) if m.group(2) is None else (int(m.group(1)), int(m.group(2)))
            self.cols = [m.group(3).lower()]
            self.vals = {self.cols[0]: np.arange(lo, hi, dtype=np.int64)}
            self.valid = {self.cols[0]: np.ones(hi - lo, bool)}
            self.ins = np.full(hi - lo, -1, np.int64)
            self.dels = np.full(hi - lo, -1, np.int64)
            return
        m = re.match(r"CREATE TABLE \w+\s*\((.*)\)", s, re.I)
        self.cols = [c.strip().split()[0].lower() for c in m.group(1).split(",")]
        self.vals = {c: np.zeros(0, np.int64) for c in self.cols}
        self.valid = {c: np.zeros(0, bool) for c in self.cols}

    def append(self, cols: Dict[str, tuple], owner: int):
        n = len(next(iter(cols.values()))[0])
        for c in self.cols:
            self.vals[c] = np.concatenate([self.vals[c], cols[c][0]])
            self.valid[c] = np.concatenate([self.valid[c], cols[c][1]])
        self.ins = np.concatenate([self.ins, np.full(n, owner, np.int64)])
        self.dels = np.concatenate([self.dels, np.full(n, -1, np.int64)])

    def insert(self, sql, t: Optional[Txn]):
        s = sql.rstrip(";")
        owner = -1 if t is None else self.txns.index(t)
        m = re.match(r"INSERT INTO \w+ VALUES (.*)$", s, re.I)
        if m:
            tups = [[None if v.strip().upper() == "NULL" else int(v) for v in tup.split(",")]
                    for tup in re.findall(r"\(([^)]*)\)", m.group(1))]
            cols = {c: (np.array([0 if r[j] is None else r[j] for r in tups], np.int64),
                        np.array([r[j] is not None for r in tups], bool)) for j, c in enumerate(self.cols)}
            self.append(cols, owner)
            return
        m = re.match(r"INSERT INTO \w+ SELECT (.*) FROM range\((\d+)(?:,\s*(\d+)(?:,\s*1)?)?\)(?:\s*\w+\((\w+)\))?$", s, re.I)
        if m:  # SELECT <expressions over the range variable> FROM range(lo, hi[, 1]) alias(var)
            lo, hi = (0, int(m.group(2))) if m.group(3) is None else (int(m.group(2)), int(m.group(3)))
            v = np.arange(lo, hi, dtype=np.int64)
            f = {(m.group(4) or "range").lower(): (v, np.ones(len(v), bool)), "rowid": (v, np.ones(len(v), bool))}
            items = [x.strip() for x in m.group(1).split(",")]
            exprs = [parse_expr(m.group(4) or "range") for _ in self.cols] if items == ["*"] else [parse_expr(x) for x in items]
            assert len(exprs) == len(self.cols), sql
            self.append({c: e(f) for c, e in zip(self.cols, exprs)}, owner)
            return
        m = re.match(r"INSERT INTO (\w+) SELECT \* FROM (\w+)$", s, re.I)
        assert m and m.group(1) == m.group(2), sql
        snap = self.view(t if t is not None else Txn(0, start=self.clock + 1))
        self.append({c: snap[c] for c in self.cols}, owner)

    def update(self, sql, t: Txn):
        m = re.match(r"UPDATE \w+ SET (.*?)(?: WHERE (.*))?$", sql.rstrip(";"), re.I | re.S)
        sets = []
        for a in re.split(r",(?![^(]*\))", m.group(1)):
            col, e = a.split("=", 1)
            sets.append((col.strip().lower(), parse_expr(e)))
        f = self.view(t)
        if m.group(2):
            f = frame_take(f, parse_cond(m.group(2))(f)[0])
        rows = f["rowid"][0]
        for col, _ in sets:  # a record of the row's column the writer cannot see: conflict
            for c, r, _, _, owner in self.records:
                if c == col and not self.seen(owner, t) and np.isin(rows, r).any():
                    return None
        owner = self.txns.index(t)
        self.records += [(col, rows, *e(f), owner) for col, e in sets]  # every SET reads the old row
        return len(rows)

    def delete(self, sql, t: Txn):
        m = re.match(r"DELETE FROM \w+(?: WHERE (.*))?$", sql.rstrip(";"), re.I | re.S)
        f = self.view(t)
        if m.group(1):
            f = frame_take(f, parse_cond(m.group(1))(f)[0])
        rows = f["rowid"][0]
        if (self.dels[rows] >= 0).any():  # stamped by a deleter this snapshot cannot see
            return None
        self.dels[rows] = self.txns.index(t)
        return len(rows)

    def finish(self, t: Txn, commit: bool):
        if commit:
            t.commit = self.tick()
            return
        t.aborted = True
        k = self.txns.index(t)
        self.records = [r for r in self.records if r[4] != k]
        self.dels[self.dels == k] = -1

    def query_state(self, con, sql, rows, t: Txn) -> Query:
        recs: Dict[str, list] = {}
        for col, r, v, ok, owner in self.records:
            recs.setdefault(col, []).append((r, v, ok, self.txns[owner].version))
        return Query(con, sql, rows, t.start, t.tid, list(self.cols),
                     {c: (self.vals[c].copy(), self.valid[c].copy()) for c in self.cols},
                     self.versions(self.ins, 0), self.versions(self.dels, NOT_DELETED), recs, self.view(t),
                     min([t.start] + [a.start for a in self.active.values() if a.start is not None]))

    def run(self):
        """Yields a Query per SELECT of the script (a DML statement's outcome and row count are
        checked here)."""
        imm = self.case["immediate_transaction_mode"]
        for step in self.case["script"]:
            con, sql = step["con"], step["sql"].strip()
            up = sql.upper()
            if up.startswith("CREATE TABLE"):
                self.create(sql)
                continue
            if up.startswith(("SET ", "CHECKPOINT", "DROP TABLE")):
                continue
            if up.startswith("BEGIN"):
                t = self.new_txn(True)
                if imm:
                    self.snapshot(t)
                self.active[con] = t
                continue
            if up.rstrip(";") in ("COMMIT", "ROLLBACK"):
                t = self.active.pop(con)
                if not t.aborted:  # COMMIT of an aborted transaction is its rollback
                    self.finish(t, up.startswith("COMMIT"))
                continue
            if up.startswith("INSERT") and not self.started and con not in self.active:
                self.insert(sql, None)  # setup rows, before any snapshot: visible to all
                continue
            if up.startswith("TRUNCATE"):
                sql, up = "DELETE FROM t", "DELETE FROM T"
            t = self.active.get(con) or self.new_txn(False)
            self.snapshot(t)
            if up.startswith(("UPDATE", "DELETE", "INSERT")):
                if up.startswith("INSERT"):
                    self.insert(sql, t)
                    n = 0
                else:
                    n = (self.update if up.startswith("UPDATE") else self.delete)(sql, t)
                ok = n is not None
                if step["op"] == "statement":
                    assert ok == step["ok"], (sql, con)
                else:
                    assert ok and [[n]] == step["rows"], (sql, n, step["rows"])
                if not t.explicit:
                    self.finish(t, ok)
                elif not ok:  # a failed statement aborts its transaction; ROLLBACK (or COMMIT) ends it
                    self.finish(t, False)
                continue
            assert step["op"] == "query", sql
            yield self.query_state(con, sql, step["rows"], t)
            if not t.explicit:
                self.finish(t, True)


# ------------------------------------------------------------------ answering a query from a frame

def split_query(sql: str):
    """(select list, where or None, order-by column or None) of `SELECT … FROM t [WHERE …] [ORDER BY …]`."""
    s = sql.strip().rstrip(";")
    m = re.match(r"SELECT (.*?) FROM \w+(?: WHERE (.*?))?(?: ORDER BY (\w+))?$", s, re.I | re.S)
    if not m:
        raise ValueError(f"query shape not modelled: {sql}")
    return m.group(1).strip(), m.group(2), m.group(3)


def answer(q: Query, f: Frame, nulls_first: bool, filtered: bool = False):
    """The rows the query returns over a frame of visible rows (already filtered by the WHERE when
    `filtered`)."""
    sel, where, order = split_query(q.sql)
    if where and not filtered:
        f = frame_take(f, parse_cond(where)(f)[0])
    m = re.match(r"DISTINCT (\w+)$", sel, re.I)
    if m:  # SELECT DISTINCT col [ORDER BY col]: each value once, NULL first or last
        v, ok = f[m.group(1).lower()]
        vals = sorted(set(v[ok].tolist()))
        out = [[x] for x in vals]
        if (~ok).any():
            out = [[None]] + out if nulls_first else out + [[None]]
        return out
    if sel == "*":
        if order:
            col = q.columns[int(order) - 1] if order.isdigit() else order.lower()
            v, ok = f[col]
            # NULLs last (or first), ties in row order: a stable sort on (NULL rank, value)
            o = np.lexsort((v, ok if nulls_first else ~ok))
            f = {k: (a[o], b[o]) for k, (a, b) in f.items()}
        return frame_rows(f, q.columns)
    out = []
    for item in [x.strip() for x in sel.split(",")]:
        m = re.match(r"(COUNT|SUM|MIN|MAX)\((DISTINCT )?(\*|\w+)\)$", item, re.I)
        assert m, item
        fn, col = m.group(1).upper(), m.group(3).lower()
        if col == "*":
            vals = f["rowid"][0]
        else:
            v, ok = f[col]
            vals = v[ok]
        if m.group(2):
            vals = np.unique(vals)
        if fn == "COUNT":
            out.append(len(vals))
        elif len(vals) == 0:
            out.append(None)
        else:
            out.append(int({"SUM": np.sum, "MIN": np.min, "MAX": np.max}[fn](vals)))
    return [out]


def cases(golden, group: str):
    return golden["cases"][group]


_LITERAL = re.compile(r"'((?:[^']|'')*)'")


def encode_strings(case: dict):
    """A VARCHAR script as an integer one: every string the script names — its literals and the
    strings of its expected rows — sorted as DuckDB orders strings (string_t: the bytes, then the
    length: Python's bytes order) and replaced by its rank. The ranks order as the strings do, so
    comparisons, ORDER BY and DISTINCT replay on them unchanged, and they are the codes of a
    cubit_dict built from the same strings. Returns (the coded case, the strings by code)."""
    strings = set()
    for step in case["script"]:
        strings.update(m.group(1).replace("''", "'").encode() for m in _LITERAL.finditer(step["sql"]))
        for row in step.get("rows", []):
            strings.update(v.encode() for v in row if isinstance(v, str))
    words = sorted(strings)
    code = {w: i for i, w in enumerate(words)}
    steps = []
    for step in case["script"]:
        st = dict(step)
        st["sql"] = _LITERAL.sub(lambda m: str(code[m.group(1).replace("''", "'").encode()]), step["sql"])
        if "rows" in st:
            st["rows"] = [[code[v.encode()] if isinstance(v, str) else v for v in row] for row in step["rows"]]
        steps.append(st)
    return {**case, "script": steps}, words


def queries(case: dict):
    return list(Replay(case).run())
