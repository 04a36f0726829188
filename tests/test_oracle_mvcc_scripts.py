"""The reference's MVCC sqllogictests on the oracle: NULL updates
(test/sql/update/{test_null_update, null_update_merge, null_update_merge_transaction,
test_update_many_updaters_nulls, update_null_integers}.test) and inserts / deletes / updates under
concurrent transactions (test/sql/{update,delete,transactions}/*.test, listed in tests/sql_replay.py).

The replay's version state (tests/sql_replay.py) is pinned by the files' expected rows first; then
the oracle answers every query of every file from that state alone — per-row insert and delete
stamps (cpu_ref.c's ChunkVectorInfo restatement), update records with their validity
(UpdateMergeValidity / FetchRowValidity), the WHERE pushed as a TableFilterSet — and the answer is
compared with the file's rows."""
import numpy as np
import pytest

import sql_replay as R
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from oracle import oracle as O

NULL_CASES = ["test_null_update", "null_update_merge", "null_update_merge_transaction", "test_update_many_updaters_nulls",
              "update_null_integers"]
MVCC_CASES = ["test_update_delete_same_tuple", "update_after_commit", "test_update_same_value", "test_delete",
              "test_large_delete", "large_deletes_transactions", "test_segment_deletes",
              "test_multi_transaction_append", "test_multi_version_large", "test_null_version",
              "test_transaction_local_data", "test_update", "test_update_mix", "test_update_many_updaters",
              "test_cascading_updates", "test_truncate", "test_large_delete_parallel", "test_multi_version",
              "test_interleaved_versions"]
ALL = [("null_updates", n) for n in NULL_CASES] + [("mvcc_scripts", n) for n in MVCC_CASES]


def script(golden, group, name):
    return R.cases(golden, group)[name]


def oracle_columns(q: R.Query):
    cols = []
    for c in q.columns:
        data, valid = q.base[c]
        rows, vals, vers, ok = q.update_arrays(c)
        cols.append(O.Column(data.astype(np.int32), validity_from_mask(valid), (rows, vals, vers, ok) if len(rows) else None))
    return cols


def pushed_filters(q: R.Query, where):
    """The WHERE as DuckDB pushes it into the scan (one TableFilter per column, an AND of its terms),
    or None for a WHERE of another shape."""
    terms = R.simple_terms(where)
    if terms is None:
        return None
    per = {}
    for col, op, k in terms:
        flt = F.IsNullFilter() if op == "IS NULL" else F.IsNotNullFilter() if op == "IS NOT NULL" else F.ConstantFilter(op, k)
        per.setdefault(q.columns.index(col), []).append(flt)
    return F.TableFilterSet({j: (fs[0] if len(fs) == 1 else F.ConjunctionAndFilter(fs)) for j, fs in per.items()})


def oracle_frame(q: R.Query, cols, fs=None) -> R.Frame:
    """The rows the snapshot sees (through the pushed filters), every column fetched with its validity."""
    tx = O.Mvcc(q.start, q.tid, inserted=q.inserted, deleted=q.deleted)
    rows = O.table_scan(cols, F.serialize(fs or F.TableFilterSet()), q.n_rows, tx=tx)
    f = {"rowid": (rows.astype(np.int64), np.ones(len(rows), bool))}
    for c, col in zip(q.columns, cols):
        vals, valid = O.fetch(col, rows, tx=tx, with_valid=True)
        assert (vals[~valid] == 0).all()
        f[c] = (vals.astype(np.int64), valid)
    return f


def predicates(q: R.Query, col: str):
    """(TableFilter, mask function over (values, valid)) pairs on one column: NULL tests, comparisons
    at the first values the column takes (and past the largest), ranges on and off the GPU test's
    bin edges, and a NULL-or-value disjunction."""
    data, valid = q.base[col]
    upd = [b[1][b[2]] for b in q.records.get(col, [])]
    vals = np.unique(np.concatenate([data[valid], *upd, [0]]))
    out = [(F.IsNullFilter(), lambda v, ok: ~ok), (F.IsNotNullFilter(), lambda v, ok: ok)]
    for k in [int(x) for x in vals[:6]] + [int(vals[-1]) + 1]:
        for op, f in (("=", np.equal), ("<", np.less), (">=", np.greater_equal), ("!=", np.not_equal)):
            out.append((F.ConstantFilter(op, k), lambda v, ok, f=f, k=k: ok & f(v, k)))
    for lo, hi in ((2, 8), (4, 17), (1, 3), (0, 100)):
        out.append((F.ConjunctionAndFilter([F.ConstantFilter(">=", lo), F.ConstantFilter("<", hi)]),
                    lambda v, ok, lo=lo, hi=hi: ok & (v >= lo) & (v < hi)))
    out.append((F.ConjunctionOrFilter([F.IsNullFilter(), F.ConstantFilter("<", 3)]), lambda v, ok: ~ok | (ok & (v < 3))))
    return out


@pytest.mark.parametrize("group,name", ALL)
def test_replay_matches_reference_rows(golden, group, name):
    """The replay's own view of every query equals the file's expected rows (the version state it
    hands to the oracle and the GPU is the one the reference's outputs imply)."""
    case = script(golden, group, name)
    qs = R.queries(case)
    assert qs, name
    for q in qs:
        assert R.answer(q, q.view, case["nulls_first"]) == q.rows, (name, q.con, q.sql)


@pytest.mark.parametrize("group,name", ALL)
def test_oracle_answers_scripts(golden, group, name):
    case = script(golden, group, name)
    for q in R.queries(case):
        cols = oracle_columns(q)
        view = oracle_frame(q, cols)
        assert R.frame_equal(view, q.view), (name, q.con, q.sql)
        assert R.answer(q, view, case["nulls_first"]) == q.rows, (name, q.con, q.sql)
        _, where, _ = R.split_query(q.sql)
        fs = pushed_filters(q, where)
        if where and fs is not None:
            got = R.answer(q, oracle_frame(q, cols, fs), case["nulls_first"], filtered=True)
            assert got == q.rows, (name, q.con, q.sql, "pushed")
        if q.n_rows > 4096:
            continue
        tx = O.Mvcc(q.start, q.tid, inserted=q.inserted, deleted=q.deleted)
        for j, c in enumerate(q.columns):
            v, ok = view[c]
            for flt, pred in predicates(q, c):
                got = O.table_scan(cols, F.serialize(F.TableFilterSet({j: flt})), q.n_rows, tx=tx)
                assert got.tolist() == view["rowid"][0][pred(v, ok)].tolist(), (name, q.sql, c, flt)


def test_scripts_exercise_every_kind_of_version(golden):
    """Across the scripts: SET NULL records and value records onto NULL rows (both directions of the
    validity chain), uncommitted and committed insert stamps, uncommitted and committed delete
    stamps all occur in some query's state."""
    seen = set()
    for group, name in ALL:
        for q in R.queries(script(golden, group, name)):
            for c, batches in q.records.items():
                for rows, vals, ok, ver in batches:
                    if (~ok).any():
                        seen.add("to_null")
                    if (ok & ~q.base[c][1][rows]).any():
                        seen.add("from_null")
            ins = q.inserted[q.inserted != 0]
            if ((ins >= R.TXN_START) & (ins < R.NOT_DELETED)).any():
                seen.add("insert_uncommitted")
            if (ins < R.TXN_START).any():
                seen.add("insert_committed")
            dels = q.deleted[q.deleted != R.NOT_DELETED]
            if (dels >= R.TXN_START).any():
                seen.add("delete_uncommitted")
            if (dels < R.TXN_START).any():
                seen.add("delete_committed")
    assert seen == {"to_null", "from_null", "insert_uncommitted", "insert_committed", "delete_uncommitted",
                    "delete_committed"}, seen
