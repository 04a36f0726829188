"""Pin the oracle (oracle/cpu_ref.c) and the lineitem generator against the reference's
own answers: extension/tpch/dbgen/answers/sf*/q06.csv and the fingerprints SURVEY.md §8c
measured by running DuckDB v1.1.2 (tests/golden/tpch.json)."""
import numpy as np
import pytest

from conftest import lineitem, revenue_from_answer
from cubit_amd import filters as F
from oracle import oracle as O


def q6_columns(li):
    return [O.Column(li.l_shipdate), O.Column(li.l_discount), O.Column(li.l_quantity), O.Column(li.l_extendedprice)]


def q6_rows(li, tx=None, cols=None):
    plan = F.serialize(F.q6_filter_set(0, 1, 2))
    return O.table_scan(cols or q6_columns(li), plan, li.n_rows, li.row_base, tx=tx)


@pytest.mark.parametrize("sf", [0.01, 0.1, 1])
def test_q6_revenue_matches_reference_answer(sf, golden):
    li = lineitem(sf)
    rows = q6_rows(li)
    rev = O.sum_product(li.l_extendedprice, li.l_discount, rows)
    key = {0.01: "0.01", 0.1: "0.1", 1: "1"}[sf]
    assert rev == revenue_from_answer(golden["tpch"]["q6_revenue"][key]["revenue"])


def test_sf001_q6_count(li001, golden):
    assert len(q6_rows(li001)) == golden["tpch"]["fingerprints"]["sf001_q6"]["count"]


def test_sf1_q6_fingerprint(li1, golden):
    fp = golden["tpch"]["fingerprints"]["sf1_q6"]
    rows = q6_rows(li1)
    assert len(rows) == fp["count"]
    assert int(rows.sum()) == fp["sum_rowid"]
    assert int(rows.min()) == fp["min"] and int(rows.max()) == fp["max"]
    assert O.xor_hash(rows) == fp["xor_hash"]
    assert np.all(np.diff(rows) > 0)


def test_sf1_shipdate_equality_fingerprint(li1, golden):
    fp = golden["tpch"]["fingerprints"]["sf1_shipdate_eq_1995_03_15"]
    fs = F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter("=", F.date(1995, 3, 15)),
                                                      F.IsNotNullFilter()])})
    rows = O.table_scan(q6_columns(li1), F.serialize(fs), li1.n_rows)
    assert len(rows) == fp["count"]
    assert int(rows.sum()) == fp["sum_rowid"]
    assert O.xor_hash(rows) == fp["xor_hash"]


def test_sf1_leaf_counts(li1, golden):
    fp = golden["tpch"]["fingerprints"]["sf1_leaf_counts"]
    cols = q6_columns(li1)
    ship = F.TableFilterSet()
    ship.push_filter(0, F.ConstantFilter(">=", F.date(1994, 1, 1)))
    ship.push_filter(0, F.ConstantFilter("<", F.date(1995, 1, 1)))
    disc = F.TableFilterSet()
    disc.push_filter(1, F.ConstantFilter(">=", 5))
    disc.push_filter(1, F.ConstantFilter("<=", 7))
    qty = F.TableFilterSet({2: F.ConstantFilter("<", 2400)})
    assert len(O.table_scan(cols, F.serialize(ship), li1.n_rows)) == fp["shipdate_1994"]
    assert len(O.table_scan(cols, F.serialize(disc), li1.n_rows)) == fp["discount_005_007"]
    assert len(O.table_scan(cols, F.serialize(qty), li1.n_rows)) == fp["quantity_lt_24"]


TXN_START = 4611686018427388000  # TRANSACTION_ID_START (src/common/constants.cpp:14)


def mvcc_scenario(li):
    """con1 (uncommitted) UPDATE l_quantity=1 WHERE rowid%7=0 and DELETE WHERE
    rowid%11=0. Writer: start_time 2, transaction_id TXN_START+1; reader con2: start_time 2,
    transaction_id TXN_START+2. Uncommitted versions carry the writer's transaction id."""
    n = li.n_rows
    writer = TXN_START + 1
    upd_rows = np.arange(0, n, 7, dtype=np.int64)
    del_rows = np.arange(0, n, 11, dtype=np.int64)
    deleted = np.full(n, np.uint64(2 ** 64 - 2), dtype=np.uint64)  # NOT_DELETED_ID
    deleted[del_rows] = writer
    return upd_rows, del_rows, deleted, writer


def test_sf001_mvcc_writer_and_reader_views(li001, golden):
    fp = golden["tpch"]["fingerprints"]["sf001_mvcc"]
    upd_rows, _, deleted, writer = mvcc_scenario(li001)
    qty = O.Column(li001.l_quantity, updates=(upd_rows, np.full(len(upd_rows), 100, dtype=np.int64),
                                              np.full(len(upd_rows), writer, dtype=np.uint64)))
    cols = [O.Column(li001.l_shipdate), O.Column(li001.l_discount), qty, O.Column(li001.l_extendedprice)]
    w = O.Mvcc(2, writer, deleted=deleted)
    r = O.Mvcc(2, TXN_START + 2, deleted=deleted)
    assert len(q6_rows(li001, tx=w, cols=cols)) == fp["writer_view"]
    assert len(q6_rows(li001, tx=r, cols=cols)) == fp["reader_view"]


def test_oracle_bitmap_evaluator_agrees_with_scan(li01):
    """The CPU bitmap evaluator over range-encoded bitvectors equals the value scan."""
    n = li01.n_rows
    sd, di, qu = O.Column(li01.l_shipdate), O.Column(li01.l_discount), O.Column(li01.l_quantity)
    leaves = [O.build_bitvector(sd, n, 2, F.date(1995, 1, 1)),   # shipdate < 1995-01-01
              O.build_bitvector(sd, n, 2, F.date(1994, 1, 1)),   # shipdate < 1994-01-01
              O.build_bitvector(di, n, 2, 8),                    # discount < 0.08
              O.build_bitvector(di, n, 2, 5),                    # discount < 0.05
              O.build_bitvector(qu, n, 2, 2400)]                 # quantity < 24
    prog = [0, 1, O.OB_ANDNOT, 2, 3, O.OB_ANDNOT, O.OB_AND, 4, O.OB_AND]
    rows, _ = O.bitmap_eval(leaves, prog, n)
    assert np.array_equal(rows, q6_rows(li01))


def test_per_column_or_is_a_set_union_in_child_order():
    """ConjunctionOrFilter keeps child order (column_segment.cpp:381-409): the raw output is
    not ascending, the canonical set equals the numpy predicate."""
    rng = np.random.default_rng(7)
    n = 10000
    a = rng.integers(0, 100, n).astype(np.int32)
    fs = F.TableFilterSet({0: F.ConjunctionOrFilter([F.ConstantFilter(">", 90), F.ConstantFilter("<", 5)])})
    plan = F.serialize(fs)
    raw = O.table_scan([O.Column(a)], plan, n, canonical=False)
    canon = O.table_scan([O.Column(a)], plan, n, canonical=True)
    expect = np.nonzero((a > 90) | (a < 5))[0]
    assert np.array_equal(np.sort(raw), expect)
    assert np.array_equal(canon, expect)
    assert not np.all(np.diff(raw) > 0)


def test_residual_or_tree_with_nulls():
    rng = np.random.default_rng(11)
    n = 5000
    cols = [rng.integers(0, 100, n).astype(np.int32) for _ in range(4)]
    valid = [rng.random(n) > 0.1 for _ in range(4)]
    from cubit_amd.datagen import validity_from_mask

    ocols = [O.Column(c, validity_from_mask(v)) for c, v in zip(cols, valid)]
    tree = F.Or(F.And(F.Cmp(0, "<", 10), F.Cmp(1, "<", 10)), F.And(F.Cmp(2, "<", 10), F.Cmp(3, "<", 10)))
    rows = O.table_scan(ocols, F.serialize(None, tree), n)
    m = ((cols[0] < 10) & valid[0] & (cols[1] < 10) & valid[1]) | ((cols[2] < 10) & valid[2] & (cols[3] < 10) & valid[3])
    assert np.array_equal(rows, np.nonzero(m)[0])


def test_zonemap_segment_reference_case(golden):
    """test/sql/filter/test_zonemap_segment.test: SUM(i) WHERE i=k over 5 blocks of 65,534."""
    c = golden["cases"]["zonemap_segment"]
    data = np.repeat(np.array(c["values"], dtype=np.int32), c["block_rows"])
    for k, want in c["expected_sum_eq"].items():
        fs = F.TableFilterSet({0: F.ConstantFilter("=", int(k))})
        rows = O.table_scan([O.Column(data)], F.serialize(fs), len(data))
        got = int(data[rows].astype(np.int64).sum()) if len(rows) else None
        assert got == want


def timestamp_table(c):
    """t1(ts TIMESTAMP as int64 microseconds since the epoch, i INTEGER) from the case's runs."""
    from datetime import datetime, timezone

    def us(text):
        return int(datetime.fromisoformat(text).replace(tzinfo=timezone.utc).timestamp()) * 1_000_000

    ts = np.concatenate([np.full(hi - lo + 1, us(t), dtype=np.int64) for t, lo, hi in c["runs"]])
    i = np.concatenate([np.arange(lo, hi + 1, dtype=np.int32) for _, lo, hi in c["runs"]])
    return ts, i, us


def timestamp_filter_sets(c, us):
    """Each query's pushed filters: ts in [d 00:00, d + 1 day), and the bound on i."""
    out = []
    for q in c["queries"]:
        lo = us(q["date"] + " 00:00:00")
        f = {0: F.ConjunctionAndFilter([F.ConstantFilter(">=", lo), F.ConstantFilter("<", lo + 86_400_000_000)])}
        if q["i"]:
            f[1] = F.ConstantFilter(q["i"][0], q["i"][1])
        out.append((F.TableFilterSet(f), q["count"]))
    return out


def test_timestamp_date_pushdown_reference_case(golden):
    """test/optimizer/pushdown/timestamp_to_date_pushdown.test: ts::date = d pushed as a TIMESTAMP
    range, beside a bound on i: the file's counts."""
    c = golden["cases"]["timestamp_date_pushdown"]
    ts, i, us = timestamp_table(c)
    for fs, want in timestamp_filter_sets(c, us):
        assert len(O.table_scan([O.Column(ts), O.Column(i)], F.serialize(fs), len(ts))) == want


def test_interleaved_versions_reference_case(golden):
    """test/sql/transactions/test_interleaved_versions.test:66-120 (deletes by two txns)."""
    data = np.array([1, 2], dtype=np.int32)
    t1, t2 = TXN_START + 10, TXN_START + 11
    deleted = np.array([t1, t2], dtype=np.uint64)  # con1 deletes i=1, con2 deletes i=2
    plan = F.serialize(F.TableFilterSet())

    def s(tx):
        r = O.table_scan([O.Column(data)], plan, 2, tx=tx)
        return int(data[r].sum()) if len(r) else None

    exp = golden["cases"]["interleaved_versions"]["steps"]
    assert s(O.Mvcc(5, t1, deleted=deleted)) == exp[0]["expect"]["con1"]
    assert s(O.Mvcc(5, t2, deleted=deleted)) == exp[0]["expect"]["con2"]
    assert s(O.Mvcc(5, TXN_START + 12, deleted=deleted)) == exp[0]["expect"]["con3"]
    # con1 commits with commit id 6: the delete of i=1 now carries id 6; con2 (start 5) still sees it
    deleted_c = np.array([6, t2], dtype=np.uint64)
    assert s(O.Mvcc(5, t2, deleted=deleted_c)) == exp[1]["expect"]["con2"]
    assert s(O.Mvcc(7, TXN_START + 13, deleted=deleted_c)) == 2


def residual_from_json(node):
    """["or"|"and", children…] / [column, cmp, constant] → residual filter tree."""
    if node[0] in ("or", "and"):
        kids = [residual_from_json(c) for c in node[1:]]
        return F.Or(*kids) if node[0] == "or" else F.And(*kids)
    col, cmp, c = node
    return F.Cmp(col, cmp, c)


def test_table_or_pushdown_reference_case(golden):
    """test/optimizer/pushdown/table_or_pushdown.test: cross-column OR/AND trees on (a, b)."""
    c = golden["cases"]["table_or_pushdown"]
    data = np.array(c["rows"], dtype=np.int32)
    cols = [O.Column(data), O.Column(data.copy())]
    for q in c["queries"]:
        rows = O.table_scan(cols, F.serialize(None, residual_from_json(q["tree"])), len(data))
        assert data[rows].tolist() == q["expect"], q["sql"]


def where_filters(where):
    """[[column, cmp, constant], …] (AND) → TableFilterSet; two filters on one column AND."""
    per = {}
    for col, cmp, c in where:
        per.setdefault(col, []).append(F.ConstantFilter(cmp, c))
    return F.TableFilterSet({c: fs[0] if len(fs) == 1 else F.ConjunctionAndFilter(fs) for c, fs in per.items()})


def update_case_views(golden):
    """test/sql/update/test_update.test as update lists and snapshots: yields (step, update
    list, {connection: (start, transaction id)}). con1's update is uncommitted (its
    transaction id) until COMMIT gives it commit id 6; the rolled-back update leaves the list."""
    steps = golden["cases"]["update"]["steps"]
    t1, t2, t3, t4, t5 = (TXN_START + k for k in range(1, 6))
    u = lambda vals, vers: (np.zeros(len(vals), np.int64), np.array(vals, np.int64), np.array(vers, np.uint64))
    yield steps[0], u([1], [t1]), {"con1": (5, t1), "con2": (5, t2)}
    yield steps[1], u([1], [6]), {"con1": (7, t3), "con2": (7, t4)}
    yield steps[2], u([1, 4], [6, t5]), {"con1": (7, t5), "con2": (7, t4)}
    yield steps[3], u([1], [6]), {"con1": (8, TXN_START + 6), "con2": (8, TXN_START + 7)}


def test_update_reference_case(golden):
    """test/sql/update/test_update.test:11-104: an update seen by its writer only, then by all
    after COMMIT; a rolled-back update seen by no one afterwards."""
    data = np.array(golden["cases"]["update"]["rows"], dtype=np.int32)
    for step, upd, conns in update_case_views(golden):
        for con, eq, expect in step["checks"]:
            fs = F.TableFilterSet({0: F.ConstantFilter("=", eq)}) if eq is not None else F.TableFilterSet()
            start, tid = conns[con]
            col = O.Column(data, updates=upd)
            rows = O.table_scan([col], F.serialize(fs), 1, tx=O.Mvcc(start, tid))
            seen = O.fetch(col, rows, tx=O.Mvcc(start, tid)).tolist() if len(rows) else []
            assert list(seen) == expect, (step["do"], con, eq)


NOT_DELETED = 2 ** 64 - 2  # NOT_DELETED_ID, src/common/constants.cpp:16


def multi_version_views(golden):
    """test/sql/transactions/test_multi_version.test as version state per step: yields (step,
    update list of column 0, per-row delete ids, rows inserted by con1 (appended after the three
    base rows) with their insert id, {connection: (start, transaction id)}). con1's statements
    carry its transaction id until COMMIT gives them commit id 6; con2's snapshot starts at 5,
    and after the commit a new one at 7."""
    t1, t2 = TXN_START + 1, TXN_START + 2
    u = lambda vals, vers: (np.zeros(len(vals), np.int64), np.array(vals, np.int64), np.array(vers, np.uint64))
    none = u([], [])
    steps = golden["cases"]["multi_version"]["steps"]
    conns = {"con1": (5, t1), "con2": (5, t2)}
    yield steps[0], none, [NOT_DELETED] * 3, ([], 0), conns
    yield steps[1], u([5], [t1]), [NOT_DELETED] * 3, ([], 0), conns
    yield steps[2], u([5, 10], [t1, t1]), [NOT_DELETED] * 3, ([], 0), conns
    yield steps[3], u([5, 10], [t1, t1]), [t1, NOT_DELETED, NOT_DELETED], ([], 0), conns
    yield steps[4], u([5, 10], [t1, t1]), [t1, NOT_DELETED, NOT_DELETED], ([1, 2], t1), conns
    yield steps[5], u([5, 10], [6, 6]), [6, NOT_DELETED, NOT_DELETED], ([1, 2], 6), {"con2": (7, TXN_START + 3)}


def test_multi_version_reference_case(golden):
    """test/sql/transactions/test_multi_version.test:9-99: a writer's update, second update,
    delete and insert seen by the writer only; by every later snapshot after COMMIT."""
    base = [1, 2, 3]
    for step, upd, deleted, (ins, ins_id), conns in multi_version_views(golden):
        data = np.array(base + ins, dtype=np.int32)
        n = len(data)
        inserted = np.array([0] * 3 + [ins_id] * len(ins), dtype=np.uint64)
        dele = np.array(deleted + [NOT_DELETED] * len(ins), dtype=np.uint64)
        col = O.Column(data, updates=upd)
        for con, want in step["expect"].items():
            tx = O.Mvcc(*conns[con], inserted=inserted, deleted=dele)
            rows = O.table_scan([col], F.serialize(F.TableFilterSet()), n, tx=tx)
            assert int(O.fetch(col, rows, tx=tx).sum()) == want, (step["do"], con)


def test_concurrent_reads_while_updating_reference_case(golden):
    """concurrent_reads_while_updating.test_slow, serially: after k of the 20 committed
    UPDATE i=i+1, a snapshot sees 10,000 rows summing to 49,995,000 + 10,000·k — inside the
    reader's bounds — and the last one the final 10,000 / 50,195,000."""
    c = golden["cases"]["concurrent_reads_while_updating"]
    n = c["rows"]
    data = np.arange(n, dtype=np.int32)
    rows = np.tile(np.arange(n, dtype=np.int64), c["updates"])
    vals = np.concatenate([np.arange(n, dtype=np.int64) + k for k in range(1, c["updates"] + 1)])
    vers = np.repeat(np.arange(1, c["updates"] + 1, dtype=np.uint64) * 10, n)
    order = np.argsort(rows, kind="stable")  # chronological per row
    col = O.Column(data, updates=(rows[order], vals[order], vers[order]))
    lo, hi = c["reader_sum_range"]
    for k in (0, 1, 7, c["updates"]):
        tx = O.Mvcc(10 * k + 1, TXN_START + 100 + k)
        r = O.table_scan([col], F.serialize(F.TableFilterSet()), n, tx=tx)
        total = int(O.fetch(col, r, tx=tx).sum())
        assert len(r) == c["reader_count"] and lo <= total <= hi and total == lo + n * k
    assert (len(r), total) == (c["final"]["count"], c["final"]["sum"])


def many_updaters_reads(golden):
    """test/sql/update/test_update_many_updaters.test as the version state at each read: yields
    (connection, (start, transaction id), update list of column a) in file order, to pair with
    the golden views. Start times and commit ids share one increasing counter; BEGIN takes the
    snapshot (immediate_transaction_mode); a statement outside BEGIN is its own transaction; an
    uncommitted record carries its writer's transaction id until COMMIT re-stamps it."""
    tid = {c: TXN_START + i for i, c in enumerate(("con1", "con2", "con3", "con4", "updater"), 1)}
    recs = []  # [row, value, version or writer connection]
    committed = {}  # connection -> commit id of its records
    snap = {}

    def ulist():
        order = sorted(range(len(recs)), key=lambda i: (recs[i][0], i))  # per row, chronological
        vers = [committed.get(recs[i][2], tid.get(recs[i][2])) if isinstance(recs[i][2], str) else recs[i][2]
                for i in order]
        return (np.array([recs[i][0] for i in order], np.int64), np.array([recs[i][1] for i in order], np.int64),
                np.array(vers, np.uint64))

    def reads(*cons):
        for c in cons:
            yield c, snap[c], ulist()

    for phase_start in (1, 9):  # the process runs twice; phase 1 ends with the revert at 8
        c = phase_start
        snap["con1"] = (c, tid["con1"])
        recs.append([0, 4, c + 1])
        snap["con2"] = (c + 2, tid["con2"])
        recs.append([1, 5, c + 3])
        snap["con3"] = (c + 4, tid["con3"])
        recs.append([2, 6, c + 5])
        snap["con4"] = (c + 6, tid["con4"])
        yield from reads("con1", "con2", "con3", "con4")
        if phase_start == 1:
            recs.extend([[0, 1, 8], [1, 2, 8], [2, 3, 8]])  # updater: a=a-3, committed at 8
    recs.extend([[0, 7, "con2"], [1, 8, "con3"], [2, 9, "con4"]])
    yield from reads("con1", "con2", "con3", "con4")
    snap["updater"] = (16, tid["updater"])
    yield from reads("updater")
    committed["con4"] = 17
    snap["con4"] = (18, TXN_START + 10)
    yield from reads("con1", "con2", "con3", "con4")
    committed["con2"] = 19
    snap["con2"] = snap["con4"] = (20, TXN_START + 11)
    yield from reads("con1", "con2", "con3", "con4")
    committed["con3"] = 21
    snap["con2"] = snap["con3"] = snap["con4"] = (22, TXN_START + 12)
    yield from reads("con1", "con2", "con3", "con4")
    snap["con1"] = (23, TXN_START + 13)
    yield from reads("con1")


def test_many_updaters_reference_case(golden):
    """test/sql/update/test_update_many_updaters.test: the 26 views four snapshots, a writer
    and the committed state take of one 3-row table while updates commit between them."""
    c = golden["cases"]["many_updaters"]
    data = np.array(c["rows"], dtype=np.int32)
    got = list(many_updaters_reads(golden))
    assert [g[0] for g in got] == [v[0] for v in c["views"]]
    for (con, (start, tx_id), upd), (_, want) in zip(got, c["views"]):
        col = O.Column(data, updates=upd)
        tx = O.Mvcc(start, tx_id)
        rows = O.table_scan([col], F.serialize(F.TableFilterSet()), 3, tx=tx)
        assert sorted(O.fetch(col, rows, tx=tx).tolist()) == want, (con, start)


def block_boundary_states(golden):
    """test/sql/update/block_boundary_update.test_slow as version state: yields, after the
    CREATE and after each statement, (statement, rows appended by it or None, update list of
    column i, per-row insert ids, snapshot start, expected (count, sum)). Statement k commits at
    2k; each read starts at 2k + 1. UPDATE i=i+1 adds one record per row (value = the row's
    current value + 1); INSERT INTO test SELECT * FROM test appends a copy of the current values."""
    c = golden["cases"]["block_boundary_update"]
    cur = np.arange(c["rows"], dtype=np.int64)
    ins = np.zeros(c["rows"], np.uint64)
    rows, vals, vers = [], [], []

    def ulist():
        if not rows:
            return (np.zeros(0, np.int64),) * 2 + (np.zeros(0, np.uint64),)
        r, v, w = np.concatenate(rows), np.concatenate(vals), np.concatenate(vers)
        o = np.argsort(r, kind="stable")  # per row, in commit order
        return r[o], v[o], w[o]

    yield "create", None, ulist(), ins, 1, tuple(c["count_sum"][0])
    for k, st in enumerate(c["statements"], 1):
        appended = None
        if st == "update":
            cur = cur + 1
            rows.append(np.arange(len(cur), dtype=np.int64))
            vals.append(cur.copy())
            vers.append(np.full(len(cur), 2 * k, np.uint64))
        else:
            appended = cur.copy()
            ins = np.concatenate([ins, np.full(len(cur), 2 * k, np.uint64)])
            cur = np.concatenate([cur, cur])
        yield st, appended, ulist(), ins, 2 * k + 1, tuple(c["count_sum"][k])


def test_block_boundary_update_reference_case(golden):
    """block_boundary_update.test_slow: COUNT(i), SUM(i) after whole-table updates across
    vector and row-group boundaries and an INSERT … SELECT of the table into itself."""
    base = np.arange(golden["cases"]["block_boundary_update"]["rows"], dtype=np.int64)
    for st, appended, upd, ins, start, (cnt, total) in block_boundary_states(golden):
        if appended is not None:
            base = np.concatenate([base, appended])
        col = O.Column(base, updates=upd)
        tx = O.Mvcc(start, TXN_START + 50, inserted=ins)
        r = O.table_scan([col], F.serialize(F.TableFilterSet()), len(base), tx=tx)
        assert (len(r), int(O.fetch(col, r, tx=tx).sum())) == (cnt, total), st


def zonemap_table(n):
    """test_zonemap.test_slow's t: a = range(n) (BIGINT), b = length(range) — its digit count."""
    a = np.arange(n, dtype=np.int64)
    b = (np.searchsorted(10 ** np.arange(1, 10, dtype=np.int64), a, side="right") + 1).astype(np.int32)
    return a, b


def test_zonemap_or_trees_reference_case(golden):
    """test/sql/filter/test_zonemap.test_slow: count(*) of cross-column OR trees over 1e8 rows
    (a = range, b = digit count) equals the file's counts — the oracle's morsel-parallel scan."""
    c = golden["cases"]["zonemap_or_trees"]
    a, b = zonemap_table(c["rows"])
    cols = [O.Column(a), O.Column(b)]
    for q in c["queries"]:
        n, _ = O.table_scan_mt(cols, F.serialize(None, residual_from_json(q["tree"])), c["rows"], threads=8)
        assert n == q["count"], q["sql"]


def filter_cache_table(golden):
    """filter_cache.test's integers: every a in [0, 10000) ten times (a cross product's rows)."""
    c = golden["cases"]["filter_cache"]
    lo, hi = c["values"]
    return np.repeat(np.arange(lo, hi, dtype=np.int32), c["repeat"])


def filter_cache_filters(q):
    """A filter_cache query as (TableFilterSet of its plain comparisons, residual OR tree or None)."""
    return where_filters(q["where"]), (residual_from_json(q["tree"]) if q["tree"] else None)


def test_filter_cache_reference_case(golden):
    """test/sql/filter/filter_cache.test: nested subqueries' filters combined into one scan —
    comparisons pushed, an OR of ranges as the residual — count the file's rows."""
    a = filter_cache_table(golden)
    for q in golden["cases"]["filter_cache"]["queries"]:
        fs, res = filter_cache_filters(q)
        rows = O.table_scan([O.Column(a)], F.serialize(fs, res), len(a))
        assert len(rows) == q["count"], q["sql"]


def obsolete_filter_sets(golden):
    """test_obsolete_filters.test's integer queries as (WHERE text, TableFilterSet of the AND
    chain on column a, expected (a, b) rows sorted)."""
    c = golden["cases"]["obsolete_filters"]
    op = {"<>": "!="}
    for q in c["queries"]:
        fs = F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(op.get(o, o), k) for o, k in q["terms"]])})
        yield q["where"], fs, sorted(tuple(r) for r in q["rows"])


def obsolete_filter_columns(golden):
    c = golden["cases"]["obsolete_filters"]
    out = []
    for vals in (c["a"], c["b"]):
        valid = np.array([v is not None for v in vals])
        data = np.array([0 if v is None else v for v in vals], dtype=np.int32)
        out.append((data, valid))
    return out


def test_obsolete_filters_reference_case(golden):
    """test/sql/filter/test_obsolete_filters.test: redundant, subsumed and contradictory AND
    chains on one nullable column return the file's rows."""
    from cubit_amd.datagen import validity_from_mask

    (a, av), (b, bv) = obsolete_filter_columns(golden)
    cols = [O.Column(a, validity_from_mask(av)), O.Column(b, validity_from_mask(bv))]
    for where, fs, want in obsolete_filter_sets(golden):
        rows = O.table_scan(cols, F.serialize(fs), len(a))
        got = sorted((int(a[r]) if av[r] else None, int(b[r]) if bv[r] else None) for r in rows)
        assert got == want, where


def art_scan_cases(golden):
    """The reference's ART scan tests as (values, [(TableFilterSet, "sum" | "count", expected)]):
    test_art_negative_range_scan.test (closed ranges over range(-500, 500)) and
    test_art_many_matches.test (0, 1 interleaved, every comparison)."""
    c = golden["cases"]["art_scans"]
    lo, hi = c["negative_range"]["range"]
    yield np.arange(lo, hi, dtype=np.int32), [
        (F.TableFilterSet({0: F.ConjunctionAndFilter([F.ConstantFilter(">=", q["ge"]), F.ConstantFilter("<=", q["le"])])}),
         "sum", q["sum"]) for q in c["negative_range"]["queries"]]
    for b in c["many_matches"]["blocks"]:
        v = np.tile(np.array([0, 1], dtype=np.int32), b["pairs"])
        yield v, [(F.TableFilterSet({0: F.ConstantFilter(op, k)}), "count", want) for op, k, want in b["counts"]]


def test_art_scans_reference_case(golden):
    """test/sql/index/art/scan/test_art_{negative_range_scan,many_matches}.test on the oracle."""
    for v, queries in art_scan_cases(golden):
        for fs, kind, want in queries:
            rows = O.table_scan([O.Column(v)], F.serialize(fs), len(v))
            got = int(v[rows].sum()) if kind == "sum" else len(rows)
            assert got == want, (kind, want)


def art_appended_cases(golden):
    """test_art_adaptive_scan.test and test_art_range_scan.test's integer parts as (source, dtype,
    steps): each step's appended values, its filter as a TableFilterSet, and the file's answer
    ("count" or the rows)."""
    def values(spec):
        if "repeat" in spec:
            v, k = spec["repeat"]
            return np.full(k, v, np.int64)
        if "range" in spec:
            return np.arange(*spec["range"], dtype=np.int64)
        return np.array(spec["values"], np.int64)

    for case in golden["cases"]["art_scans"]["appended"]:
        steps = []
        for st in case["steps"]:
            add = values(st["append"])
            if "then" in st:
                add = np.concatenate([add, values(st["then"])])
            op, k = st["filter"]
            steps.append((add, F.TableFilterSet({0: F.ConstantFilter(op, k)}), st.get("count"), st.get("rows")))
        yield case["source"], case["type"], steps


def test_art_appended_reference_cases(golden):
    """The ART scans over rows inserted after the index (test_art_range_scan.test) or before it
    (test_art_adaptive_scan.test) on the oracle: each step's answer from the file."""
    for source, _, steps in art_appended_cases(golden):
        v = np.zeros(0, np.int64)
        for add, fs, count, rows in steps:
            v = np.concatenate([v, add])
            got = O.table_scan([O.Column(v)], F.serialize(fs), len(v))
            if count is not None:
                assert len(got) == count, source
            else:
                assert v[got].tolist() == rows, source


def filter_pushdown_tables(golden):
    """The tables of test/optimizer/pushdown/table_filter_pushdown.test as (name, columns
    [(values, valid mask or None, physical width)], queries [(TableFilterSet, result column,
    expected values)])."""
    c = golden["cases"]["table_filter_pushdown"]
    out = []
    rows = np.array(c["integers"]["rows"])
    out.append(("integers", [(rows[:, j].astype(np.int32), None) for j in range(3)],
                [(where_filters(q["where"]), 2, q["k"]) for q in c["integers"]["queries"]]))
    nums = np.array(c["numbers"]["rows"])
    for ty, width in c["numbers"]["types"].items():
        dt = np.int32 if width == 32 else np.int64
        out.append((ty, [(nums[:, j].astype(dt), None) for j in range(3)],
                    [(where_filters(q["where"]), 2, q["k"]) for q in c["numbers"]["queries"]]))
    rm = c["range_mod"]
    b = (np.arange(rm["n"]) % rm["mod"]).astype(np.int64)
    out.append(("range_mod", [(b, None)], [(where_filters(rm["where"]), None, rm["count"])]))
    tm = c["time"]
    valid = np.array([v is not None for v in tm["micros"]])
    vals = np.array([v or 0 for v in tm["micros"]], dtype=np.int64)
    out.append(("time", [(vals, valid)], [(where_filters([[0, "=", tm["eq"]]]), None, tm["count"])]))
    bo = c["bool"]
    cols = []
    for name in ("i", "j"):
        valid = np.array([v is not None for v in bo[name]])
        cols.append((np.array([v or 0 for v in bo[name]], dtype=np.int32), valid))
    out.append(("bool", cols, [(where_filters([[1, "=", bo["eq"]]]), 0, bo["i_expect"])]))
    now = 1_760_000_000_000_000                       # a fixed NOW() in microseconds
    year = 365 * 86_400_000_000
    ts = np.array([now, now - 10 * year - 2 * 86_400_000_000], dtype=np.int64)
    out.append(("timestamp", [(ts, None)],
                [(where_filters([[0, ">=", now - year]]), None, c["timestamp"]["count"])]))
    return out


def test_table_filter_pushdown_reference_case(golden):
    """test/optimizer/pushdown/table_filter_pushdown.test: every filter the file expects pushed
    into the scan, over the integer-backed types, answered by the scan itself."""
    from cubit_amd.datagen import validity_from_mask

    for name, cols, queries in filter_pushdown_tables(golden):
        ocols = [O.Column(v, validity_from_mask(m) if m is not None else None) for v, m in cols]
        n = len(cols[0][0])
        for fs, out_col, expect in queries:
            rows = O.table_scan(ocols, F.serialize(fs), n)
            if out_col is None:
                assert len(rows) == expect, name
            else:
                assert cols[out_col][0][rows].tolist() == expect, name
