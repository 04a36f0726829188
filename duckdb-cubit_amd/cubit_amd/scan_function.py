"""Python handle on libcubit_scan.so — the TableFunction mirror (include/cubit_scan.h).

CubitScanFunction.init_global / init_local / function / get_batch_index / progress follow
DuckDB's seq_scan callbacks (src/function/table/table_scan.cpp); `function` returns the
next DataChunk as a list of int64 numpy columns, empty when the scan is finished.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

import numpy as np

from . import _lib as L
from .filters import Residual, TableFilterSet, serialize, to_ctypes

ROW_ID = 2 ** 64 - 1  # COLUMN_IDENTIFIER_ROW_ID
VECTOR_SIZE = 2048


def _handles(tables):
    """A partition or a row-ordered list of partitions → (ctypes array of handles, count)."""
    ts = list(tables) if isinstance(tables, (list, tuple)) else [tables]
    return (C.c_void_p * len(ts))(*[t.handle.value if isinstance(t.handle, C.c_void_p) else t.handle for t in ts]), len(ts)


def cardinality(table):
    """TableScanCardinality: (estimated, max) rows of the partition(s) (bind time)."""
    lib = L.scan_lib()
    e, m = C.c_uint64(), C.c_uint64()
    hs, n = _handles(table)
    L.check_scan(lib.cubit_scan_cardinality_multi(hs, n, C.byref(e), C.byref(m)))
    return int(e.value), int(m.value)


def statistics(table, column_id: int):
    """TableScanStatistics: (min, max, has_null, has_no_null) of a storage column over the
    partition(s), or None for the row id (the reference returns no statistics)."""
    lib = L.scan_lib()
    lo, hi = C.c_int64(), C.c_int64()
    hn, hv = C.c_int(), C.c_int()
    hs, n = _handles(table)
    rc = lib.cubit_scan_statistics_multi(hs, n, column_id, C.byref(lo), C.byref(hi), C.byref(hn), C.byref(hv))
    if rc == L.ERR_UNSUPPORTED and column_id == ROW_ID:
        return None
    L.check_scan(rc)
    return int(lo.value), int(hi.value), bool(hn.value), bool(hv.value)


class LocalState:
    def __init__(self, scan: "CubitScanFunction"):
        self.scan = scan
        h = C.c_void_p()
        L.check_scan(scan.lib.cubit_scan_init_local(scan.handle, C.byref(h)))
        self.handle = h
        self.bufs = [np.empty(VECTOR_SIZE, dtype=np.int64) for _ in range(scan.n_out)]
        self.ptrs = (C.c_void_p * max(scan.n_out, 1))(*[b.ctypes.data for b in self.bufs])
        self.vbufs = [np.empty(VECTOR_SIZE // 64, dtype=np.uint64) for _ in range(scan.n_out)]
        self.vptrs = (C.c_void_p * max(scan.n_out, 1))(*[b.ctypes.data for b in self.vbufs])

    def __del__(self):
        try:
            self.scan.lib.cubit_scan_local_destroy(self.handle)
        except Exception:
            pass


class CubitScanFunction:
    """init_global: run the GPU scan (+ probes) for the given column_ids / projection_ids /
    filters; then any number of local states drain it chunk by chunk. `table` is one partition
    or a row-ordered list of them (cubit_scan_init_global_multi: one cursor over all)."""

    def __init__(self, table, column_ids: Sequence[int], projection_ids: Optional[Sequence[int]] = None,
                 filter_set: Optional[TableFilterSet] = None, residual: Optional[Residual] = None,
                 txn: Optional[L.Txn] = None):
        self.lib = L.scan_lib()
        self.table = table
        cols = (C.c_uint64 * max(len(column_ids), 1))(*column_ids)
        proj = list(projection_ids or [])
        projc = (C.c_uint64 * max(len(proj), 1))(*proj)
        nodes = serialize(filter_set, residual).nodes if (filter_set or residual) else []
        arr = to_ctypes(nodes)
        h = C.c_void_p()
        hs, n = _handles(table)
        L.check_scan(self.lib.cubit_scan_init_global_multi(hs, n, cols, len(column_ids), projc if proj else None,
                                                            len(proj), arr if nodes else None, len(nodes),
                                                            C.byref(txn) if txn is not None else None, C.byref(h)))
        self.handle = h
        self.n_out = len(proj) if proj else len(column_ids)

    def max_threads(self) -> int:
        v = C.c_uint64()
        L.check_scan(self.lib.cubit_scan_max_threads(self.handle, C.byref(v)))
        return int(v.value)

    def init_local(self) -> LocalState:
        return LocalState(self)

    def function(self, local: LocalState) -> List[np.ndarray]:
        n = C.c_uint64()
        L.check_scan(self.lib.cubit_scan_function(self.handle, local.handle, local.ptrs, C.byref(n)))
        return [b[: n.value].copy() for b in local.bufs]

    def function_validity(self, local: LocalState):
        """The next chunk with each column's validity (cubit_scan_function_validity):
        (columns, valid) — int64 values (0 at NULL rows) and bool masks, empty at the end."""
        n = C.c_uint64()
        L.check_scan(self.lib.cubit_scan_function_validity(self.handle, local.handle, local.ptrs, local.vptrs,
                                                           C.byref(n)))
        k = n.value
        valid = [np.unpackbits(w.view(np.uint8), bitorder="little")[:k].astype(bool) for w in local.vbufs]
        return [b[:k].copy() for b in local.bufs], valid

    def get_batch_index(self, local: LocalState) -> int:
        v = C.c_uint64()
        L.check_scan(self.lib.cubit_scan_batch_index(self.handle, local.handle, C.byref(v)))
        return int(v.value)

    def decodes(self) -> int:
        """Decode launches init_global made (cubit_scan_decodes): one per partition unless the
        filter kept more than twice the estimated rows."""
        v = C.c_uint32()
        L.check_scan(self.lib.cubit_scan_decodes(self.handle, C.byref(v)))
        return int(v.value)

    def progress(self) -> float:
        v = C.c_double()
        L.check_scan(self.lib.cubit_scan_progress(self.handle, C.byref(v)))
        return float(v.value)

    def close(self):
        if self.handle:
            self.lib.cubit_scan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
