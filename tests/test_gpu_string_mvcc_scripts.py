"""The reference's VARCHAR update sqllogictests on the GPU (tests/test_oracle_string_mvcc_scripts.py
lists them): the column is registered against a cubit_dict built from the script's strings, so its
codes are the replay's ranks; rows are appended as the script inserts them, insert / delete stamps
and string update records (codes, with SET NULL) re-declared per query; each query is answered
through the table function under its snapshot with the WHERE pushed as string constants and
compared with the file's rows, the replay's view and the oracle's strings; every string comparison
(present and absent strings) against the view; a checkpoint merges the last snapshot's committed
records and the last query is asked again."""
import numpy as np
import pytest

import sql_replay as R
from cubit_amd import _lib as L
from cubit_amd import filters as F
from cubit_amd.datagen import validity_from_mask
from cubit_amd.table import Context, CubitTable, Dictionary
from oracle import oracle as O
from test_gpu_mvcc_scripts import table_function_frame
from test_oracle_string_mvcc_scripts import CASES, coded, string_columns, string_filters, string_predicates

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = Context(0)
    yield c
    c.close()


class DeviceStrings:
    def __init__(self, ctx, words, encoding):
        self.ctx, self.encoding, self.t = ctx, encoding, None
        self.d = Dictionary(words)
        assert self.d.entries() == words  # the dictionary's codes are the replay's ranks

    def sync(self, q: R.Query, since=0):
        n = q.n_rows
        if self.t is None:
            self.t = CubitTable(self.ctx, n)
            for j, c in enumerate(q.columns):
                data, valid = q.base[c]
                codes = np.ascontiguousarray(data, np.int32)  # held: the call reads them
                vw = None if valid.all() else validity_from_mask(valid)
                L.check(self.t.lib.cubit_table_add_dict_column(self.t.handle, j, self.d.handle, codes.ctypes.data,
                                                               None if vw is None else vw.ctypes.data, 0))
                self.t.types[j] = L.TYPE_VARCHAR
                if self.encoding is not None:
                    self.t.build_index(j, self.encoding)
        elif n > self.t.n_rows:
            old = self.t.n_rows
            cols, vmask = {}, {}
            for j, c in enumerate(q.columns):
                data, valid = q.base[c]
                cols[j] = data[old:n].astype(np.int32)
                if not valid[old:n].all():
                    vmask[j] = validity_from_mask(valid[old:n])
            self.t.append(cols, vmask or None)
        self.t.set_inserts(*q.insert_ranges())
        self.t.set_deletes(*q.delete_arrays())
        for j, c in enumerate(q.columns):
            rows, vals, vers, ok = q.update_arrays(c)
            keep = vers >= since
            self.t.set_updates(j, rows[keep], vals[keep], vers[keep], valid=ok[keep])

    def close(self):
        if self.t is not None:
            self.t.close()


def check_query(t, q: R.Query, words, nulls_first, label):
    txn = L.Txn(q.start, q.tid)
    view = table_function_frame(t, q, txn)
    assert R.frame_equal(view, q.view), (label, q.con, q.sql)
    assert R.answer(q, view, nulls_first) == q.rows, (label, q.con, q.sql)
    _, where, _ = R.split_query(q.sql)
    fs = string_filters(q, where, words)
    if where and fs is not None:
        got = table_function_frame(t, q, txn, fs)
        assert R.answer(q, got, nulls_first, filtered=True) == q.rows, (label, q.sql, "pushed")
    ids = view["rowid"][0]
    tx = O.Mvcc(q.start, q.tid, inserted=q.inserted, deleted=q.deleted)
    ocols = string_columns(q, words)
    for j, c in enumerate(q.columns):
        codes, valid = t.fetch(j, ids, txn)
        addrs, rvalid = O.fetch(ocols[j], ids, tx=tx, with_valid=True)
        assert np.array_equal(valid, rvalid), (label, c)
        assert [words[k] if ok else None for k, ok in zip(codes, valid)] == ocols[j].decode(addrs, rvalid), (label, c)
        v, ok = view[c]
        for flt, pred in string_predicates(words):
            fsj = F.TableFilterSet({j: flt})
            want = ids[pred(v, ok)].tolist()
            assert t.scan(fsj, txn=txn).tolist() == want, (label, q.sql, c, flt)


@pytest.mark.parametrize("encoding", [None, L.INDEX_RANGE, L.INDEX_EQUALITY])
@pytest.mark.parametrize("name", CASES)
def test_string_scripts_on_gpu(ctx, golden, name, encoding):
    case, words = coded(golden, name)
    qs = R.queries(case)
    dev = DeviceStrings(ctx, words, encoding)
    for q in qs:
        dev.sync(q)
        check_query(dev.t, q, words, case["nulls_first"], (name, encoding))
    last = qs[-1]
    for j in range(len(last.columns)):
        dev.t.merge_updates(j, last.start)
    check_query(dev.t, last, words, case["nulls_first"], (name, encoding, "merged"))
    dev.close()


@pytest.mark.parametrize("name", CASES)
def test_string_scripts_with_a_checkpoint_after_every_query(ctx, golden, name):
    case, words = coded(golden, name)
    dev = DeviceStrings(ctx, words, L.INDEX_RANGE)
    merged = 0
    for q in R.queries(case):
        dev.sync(q, since=merged)
        check_query(dev.t, q, words, case["nulls_first"], (name, "merge-each"))
        horizon = max(merged, q.horizon)
        for j in range(len(q.columns)):
            dev.t.merge_updates(j, horizon)
        merged = horizon
    dev.close()
