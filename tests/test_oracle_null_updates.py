"""The reference's NULL-update tests (test/sql/update/test_null_update.test, null_update_merge.test,
null_update_merge_transaction.test, test_update_many_updaters_nulls.test, update_null_integers.test)
on the oracle: the replay's version state (tests/null_updates.py) is pinned by the files' expected
rows, and the oracle's scan + fetch (cpu_ref.c's restatement of UpdateMergeValidity /
FetchRowValidity) answers every query of every file from the update records alone — the
validity chain's SET NULL records included."""
import numpy as np
import pytest

import null_updates as NU
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from oracle import oracle as O

CASES = ["test_null_update", "null_update_merge", "null_update_merge_transaction", "test_update_many_updaters_nulls",
         "update_null_integers"]


def oracle_columns(q: NU.Query):
    cols = []
    for c in q.columns:
        base = q.base[c]
        data = np.array([0 if v is None else v for v in base], dtype=np.int32)
        valid = np.array([v is not None for v in base], dtype=bool)
        rows, vals, vers, ok = q.update_arrays(c)
        cols.append(O.Column(data, validity_from_mask(valid), (rows, vals, vers, ok) if len(rows) else None))
    return cols


def oracle_view(q: NU.Query, cols):
    n = len(q.base[q.columns[0]])
    tx = O.Mvcc(q.start, q.tid)
    rows = O.table_scan(cols, F.serialize(F.TableFilterSet()), n, tx=tx)
    assert rows.tolist() == list(range(n))  # no deletes in these scripts
    view = [dict() for _ in range(n)]
    for c, col in zip(q.columns, cols):
        vals, valid = O.fetch(col, rows, tx=tx, with_valid=True)
        for r in range(n):
            view[r][c] = int(vals[r]) if valid[r] else None
            assert valid[r] or vals[r] == 0
    return view


def predicates(q: NU.Query, col: str):
    """(TableFilter, python predicate) pairs over one column: NULL tests and comparisons at every
    value the column takes (and around them)."""
    vals = sorted({v for c in [q.base[col]] for v in c if v is not None} |
                  {r[1] for r in q.records.get(col, []) if r[2]} | {0})
    out = [(F.IsNullFilter(), lambda v: v is None), (F.IsNotNullFilter(), lambda v: v is not None)]
    for k in vals[:6] + [vals[-1] + 1]:
        for op, f in (("=", lambda v, k=k: v == k), ("<", lambda v, k=k: v < k), (">=", lambda v, k=k: v >= k),
                      ("!=", lambda v, k=k: v != k)):
            out.append((F.ConstantFilter(op, k), lambda v, f=f: v is not None and f(v)))
    # ranges, on bin edges (the GPU test's binned index: 0, 2, 4, 8, 17, 100) and off them, and a
    # NULL-or-value disjunction
    for lo, hi in ((2, 8), (4, 17), (1, 3), (0, 100)):
        out.append((F.ConjunctionAndFilter([F.ConstantFilter(">=", lo), F.ConstantFilter("<", hi)]),
                    lambda v, lo=lo, hi=hi: v is not None and lo <= v < hi))
    out.append((F.ConjunctionOrFilter([F.IsNullFilter(), F.ConstantFilter("<", 3)]),
                lambda v: v is None or v < 3))
    return out


@pytest.mark.parametrize("name", CASES)
def test_replay_matches_reference_rows(golden, name):
    """The replay's own view of every query equals the file's expected rows (the record lists it
    hands to the oracle and the GPU are the ones the reference's outputs imply)."""
    case = NU.cases(golden)[name]
    qs = NU.queries(case)
    assert qs, name
    for q in qs:
        assert NU.answer(q, q.view, case["nulls_first"]) == q.rows, (name, q.con, q.sql)


@pytest.mark.parametrize("name", CASES)
def test_oracle_answers_null_update_scripts(golden, name):
    case = NU.cases(golden)[name]
    for q in NU.queries(case):
        cols = oracle_columns(q)
        view = oracle_view(q, cols)
        assert NU.answer(q, view, case["nulls_first"]) == q.rows, (name, q.con, q.sql)
        tx = O.Mvcc(q.start, q.tid)
        n = len(view)
        for j, c in enumerate(q.columns):
            for flt, pred in predicates(q, c):
                got = O.table_scan(cols, F.serialize(F.TableFilterSet({j: flt})), n, tx=tx).tolist()
                assert got == [r for r in range(n) if pred(view[r][c])], (name, q.sql, c, flt)


def test_null_records_count_in_the_update_list(golden):
    """The scripts do write SET NULL records (the validity chain), and value records onto NULL
    rows: both directions of the transition are exercised."""
    to_null = from_null = 0
    for name in CASES:
        for q in NU.queries(NU.cases(golden)[name]):
            for c, recs in q.records.items():
                to_null += sum(1 for r in recs if not r[2])
                from_null += sum(1 for r in recs if r[2] and q.base[c][r[0]] is None)
    assert to_null > 0 and from_null > 0

