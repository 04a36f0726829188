"""The reference's VARCHAR update sqllogictests on the oracle (SURVEY §8 a9 on string columns):
test/sql/update/{test_string_update, test_string_update_null, test_string_update_rollback,
test_string_update_rollback_null, test_string_update_many_strings, test_repeated_string_update,
test_update_same_string_value}.test — string value chains and their validity under concurrent
transactions, commits and rollbacks.

The replay (tests/sql_replay.py) runs each script on the ranks of the strings it names
(encode_strings: ranks order as the strings do) and is pinned by the files' expected rows; the
oracle then answers every query on the STRINGS — an ostring per row, update records carrying
strings, the WHERE pushed with string constants (FilterSelectionSwitch<string_t>) — and its rows,
mapped back to ranks, must equal the replay's view and the file's rows."""
import numpy as np
import pytest

import sql_replay as R
from cubit_amd import filters as F
from oracle import oracle as O

CASES = ["test_string_update", "test_string_update_null", "test_string_update_rollback",
         "test_string_update_rollback_null", "test_string_update_many_strings", "test_repeated_string_update",
         "test_update_same_string_value"]


def coded(golden, name):
    return R.encode_strings(R.cases(golden, "string_mvcc_scripts")[name])


def string_columns(q: R.Query, words):
    cols = []
    for c in q.columns:
        data, valid = q.base[c]
        rows, vals, vers, ok = q.update_arrays(c)
        strs = [words[int(v)] if k else None for v, k in zip(data, valid)]
        upd = (rows, [words[int(v)] if k else None for v, k in zip(vals, ok)], vers, ok) if len(rows) else None
        cols.append(O.StringColumn(strs, updates=upd))
    return cols


def string_filters(q: R.Query, where, words):
    """The WHERE (an AND of column-op-constant / IS NULL terms, constants as ranks) pushed with the
    strings the ranks stand for, or None for another shape."""
    terms = R.simple_terms(where)
    if terms is None:
        return None
    per = {}
    for col, op, k in terms:
        flt = F.IsNullFilter() if op == "IS NULL" else F.IsNotNullFilter() if op == "IS NOT NULL" else \
            F.ConstantFilter(op, words[k])
        per.setdefault(q.columns.index(col), []).append(flt)
    return F.TableFilterSet({j: (fs[0] if len(fs) == 1 else F.ConjunctionAndFilter(fs)) for j, fs in per.items()})


def string_frame(q: R.Query, cols, words, fs=None) -> R.Frame:
    """The rows the snapshot sees through the pushed filters, each column fetched as strings and
    mapped back to ranks."""
    rank = {w: i for i, w in enumerate(words)}
    tx = O.Mvcc(q.start, q.tid, inserted=q.inserted, deleted=q.deleted)
    rows = O.table_scan(cols, F.serialize(fs or F.TableFilterSet()), q.n_rows, tx=tx)
    f = {"rowid": (rows.astype(np.int64), np.ones(len(rows), bool))}
    for c, col in zip(q.columns, cols):
        addrs, valid = O.fetch(col, rows, tx=tx, with_valid=True)
        strs = col.decode(addrs, valid)
        f[c] = (np.array([rank[s] if s is not None else 0 for s in strs], np.int64), valid)
    return f


def string_predicates(words):
    """Comparisons at every string of the script and at strings between / around them (absent from
    the dictionary), NULL tests and a NULL-or-range disjunction: (filter, mask over ranks)."""
    out = [(F.IsNullFilter(), lambda v, ok: ~ok), (F.IsNotNullFilter(), lambda v, ok: ok)]
    ops = (("=", np.equal), ("<", np.less), ("<=", np.less_equal), (">", np.greater), (">=", np.greater_equal),
           ("!=", np.not_equal))
    for k, w in enumerate(words):
        for op, f in ops:
            out.append((F.ConstantFilter(op, w), lambda v, ok, f=f, k=k: ok & f(v, k)))
    # absent strings: below every word, just past a word, above every word — each as a code bound
    for s, lb in [(b"", 0), (words[0] + b"\x00", 1), (b"\xff", len(words))]:
        for op, f in (("=", None), ("<", np.less), ("<=", np.less), (">", np.greater_equal), (">=", np.greater_equal)):
            if f is None:
                out.append((F.ConstantFilter(op, s), lambda v, ok: np.zeros(len(v), bool)))
            else:
                out.append((F.ConstantFilter(op, s), lambda v, ok, f=f, lb=lb: ok & f(v, lb)))
    out.append((F.ConjunctionOrFilter([F.IsNullFilter(), F.ConstantFilter("<", words[-1])]),
                lambda v, ok: ~ok | (ok & (v < len(words) - 1))))
    return out


@pytest.mark.parametrize("name", CASES)
def test_replay_matches_reference_rows(golden, name):
    case, words = coded(golden, name)
    qs = R.queries(case)
    assert qs and words == sorted(words), name
    for q in qs:
        assert R.answer(q, q.view, case["nulls_first"]) == q.rows, (name, q.con, q.sql)


@pytest.mark.parametrize("name", CASES)
def test_oracle_answers_string_scripts(golden, name):
    case, words = coded(golden, name)
    for q in R.queries(case):
        cols = string_columns(q, words)
        view = string_frame(q, cols, words)
        assert R.frame_equal(view, q.view), (name, q.con, q.sql)
        assert R.answer(q, view, case["nulls_first"]) == q.rows, (name, q.con, q.sql)
        _, where, _ = R.split_query(q.sql)
        fs = string_filters(q, where, words)
        if where and fs is not None:
            got = R.answer(q, string_frame(q, cols, words, fs), case["nulls_first"], filtered=True)
            assert got == q.rows, (name, q.con, q.sql, "pushed")
        tx = O.Mvcc(q.start, q.tid, inserted=q.inserted, deleted=q.deleted)
        for j, c in enumerate(q.columns):
            v, ok = view[c]
            for flt, pred in string_predicates(words):
                got = O.table_scan(cols, F.serialize(F.TableFilterSet({j: flt})), q.n_rows, tx=tx)
                assert got.tolist() == view["rowid"][0][pred(v, ok)].tolist(), (name, q.sql, c, flt)


def test_string_scripts_exercise_string_chains(golden):
    """Across the scripts: string values over string values, SET NULL onto a string and a string
    onto NULL, rolled-back and uncommitted string records all occur in some query's state."""
    seen = set()
    for name in CASES:
        case, _ = coded(golden, name)
        for q in R.queries(case):
            for c, batches in q.records.items():
                for rows, vals, ok, ver in batches:
                    if (~ok).any():
                        seen.add("to_null")
                    if (ok & ~q.base[c][1][rows]).any():
                        seen.add("from_null")
                    if (ok & q.base[c][1][rows]).any():
                        seen.add("string_over_string")
                    if ver >= R.TXN_START:
                        seen.add("uncommitted")
    assert {"to_null", "string_over_string", "uncommitted"} <= seen, seen
