"""ORACLE — test infrastructure only.

ctypes handle on oracle/lib/libcubit_oracle.so (cpu_ref.c, the C restatement of the
reference CPU scan path). Imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker or the reported CPU baseline — never on the
product path.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "lib" / "libcubit_oracle.so"

OMAX_COLS = 16
OTYPE_INT32, OTYPE_INT64, OTYPE_FLOAT, OTYPE_DOUBLE, OTYPE_VARCHAR, OTYPE_UINT64 = 0, 1, 2, 3, 4, 5
OTYPE_INT128, OTYPE_UINT128 = 6, 7
OB_AND, OB_OR, OB_ANDNOT, OB_NOT = -1, -2, -3, -4


class OCol(C.Structure):
    _fields_ = [("type", C.c_int32), ("pad", C.c_int32), ("data", C.c_void_p), ("validity", C.c_void_p),
                ("n_updates", C.c_uint64), ("upd_rows", C.c_void_p), ("upd_values", C.c_void_p),
                ("upd_version", C.c_void_p), ("upd_valid", C.c_void_p)]


class OMvcc(C.Structure):
    _fields_ = [("inserted", C.c_void_p), ("deleted", C.c_void_p), ("start_time", C.c_uint64),
                ("transaction_id", C.c_uint64)]


class OFilter(C.Structure):
    _fields_ = [("kind", C.c_int32), ("cmp", C.c_int32), ("column", C.c_int32), ("n_children", C.c_int32),
                ("constant", C.c_int64)]


class OPushed(C.Structure):
    _fields_ = [("column", C.c_int32), ("root", C.c_int32)]


class OScan(C.Structure):
    _fields_ = [("cols", C.POINTER(OCol)), ("n_cols", C.c_int32), ("n_pushed", C.c_int32),
                ("pushed", C.POINTER(OPushed)), ("nodes", C.POINTER(OFilter)), ("residual_root", C.c_int32),
                ("canonical", C.c_int32), ("n_rows", C.c_uint64), ("row_base", C.c_int64),
                ("tx", C.POINTER(OMvcc))]


_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        l = C.CDLL(str(LIB))
        l.oracle_table_scan.restype = C.c_int64
        l.oracle_table_scan.argtypes = [C.POINTER(OScan), C.c_void_p, C.c_uint64]
        l.oracle_table_scan_mt.restype = C.c_int64
        l.oracle_table_scan_mt.argtypes = [C.POINTER(OScan), C.c_int, C.POINTER(C.c_uint64)]
        l.oracle_fetch.restype = C.c_int
        l.oracle_fetch.argtypes = [C.POINTER(OCol), C.POINTER(OMvcc), C.c_void_p, C.c_uint64, C.c_int64, C.c_void_p,
                                   C.c_void_p]
        l.oracle_sum_product.restype = None
        l.oracle_sum_product.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_int64,
                                         C.POINTER(C.c_uint64), C.POINTER(C.c_int64)]
        l.oracle_bitmap_eval.restype = C.c_int64
        l.oracle_bitmap_eval.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_int32), C.c_int, C.c_uint64, C.c_int64,
                                         C.c_void_p, C.c_uint64, C.c_void_p]
        l.oracle_build_bitvector.restype = None
        l.oracle_build_bitvector.argtypes = [C.POINTER(OCol), C.c_uint64, C.c_int, C.c_int64, C.c_void_p]
        l.oracle_xor_hash.restype = C.c_uint64
        l.oracle_xor_hash.argtypes = [C.c_void_p, C.c_uint64]
        l.oracle_bp_compress.restype = C.c_int
        l.oracle_bp_compress.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_uint64, C.c_int, C.c_uint64, C.c_void_p,
                                         C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                         C.POINTER(C.c_uint32)]
        l.oracle_bp_decode.restype = C.c_int
        l.oracle_bp_decode.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_int, C.c_void_p]
        l.oracle_bp_group_modes.restype = C.c_int
        l.oracle_bp_group_modes.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint64]
        _lib = l
    return _lib


def fp_bits(values, dtype) -> np.ndarray:
    """FLOAT / DOUBLE values as the int64 bit patterns the oracle and the C ABI carry (FLOAT:
    the 32-bit pattern, zero-extended)."""
    if np.dtype(dtype) == np.float32:
        return np.ascontiguousarray(np.asarray(values, dtype=np.float32)).view(np.uint32).astype(np.int64)
    return np.ascontiguousarray(np.asarray(values, dtype=np.float64)).view(np.int64)


class Column:
    """A column as the oracle sees it: base values, optional validity words and a
    chronological update list (rows, values, version ids[, valid flags: False = SET NULL]).
    FLOAT / DOUBLE columns (float32 / float64 data): update values given as floats are carried
    as their bit patterns (fp_bits)."""

    def __init__(self, data: np.ndarray, validity: Optional[np.ndarray] = None, updates=None):
        self.data = np.ascontiguousarray(data)
        assert self.data.dtype in (np.int32, np.int64, np.float32, np.float64, np.uint64)
        self.validity = None if validity is None else np.ascontiguousarray(validity, dtype=np.uint64)
        self.upd_valid = None
        if updates is None:
            self.upd = None
        else:
            r, v, ver = updates[:3]
            if self.data.dtype.kind == "f" and np.asarray(v).dtype.kind == "f":
                v = fp_bits(v, self.data.dtype)
            if np.asarray(v).dtype == np.uint64:  # UBIGINT values as their bits
                v = np.ascontiguousarray(v, dtype=np.uint64).view(np.int64)
            self.upd = (np.ascontiguousarray(r, dtype=np.int64), np.ascontiguousarray(v, dtype=np.int64),
                        np.ascontiguousarray(ver, dtype=np.uint64))
            if len(updates) > 3 and updates[3] is not None:
                self.upd_valid = np.ascontiguousarray(updates[3], dtype=np.uint8)

    def ocol(self) -> OCol:
        c = OCol()
        c.type = {np.dtype(np.int32): OTYPE_INT32, np.dtype(np.int64): OTYPE_INT64, np.dtype(np.float32): OTYPE_FLOAT,
                  np.dtype(np.float64): OTYPE_DOUBLE, np.dtype(np.uint64): OTYPE_UINT64}[self.data.dtype]
        c.data = self.data.ctypes.data
        c.validity = self.validity.ctypes.data if self.validity is not None else None
        if self.upd is not None:
            c.n_updates = len(self.upd[0])
            c.upd_rows, c.upd_values, c.upd_version = (a.ctypes.data for a in self.upd)
            c.upd_valid = self.upd_valid.ctypes.data if self.upd_valid is not None else None
        return c


class OString(C.Structure):
    _fields_ = [("data", C.c_void_p), ("size", C.c_uint64)]


class StringColumn(Column):
    """A VARCHAR column as the oracle sees it: an ostring per row (string_t: data + size), NULL
    rows from None. Update values are strings too (carried as addresses, filters.string_ref);
    fetch hands back addresses — decode() turns them into bytes."""

    def __init__(self, values, updates=None):
        from cubit_amd.datagen import validity_from_mask
        from cubit_amd.filters import string_ref

        self.values = [None if v is None else (v.encode() if isinstance(v, str) else bytes(v)) for v in values]
        n = len(self.values)
        self._bufs = [C.create_string_buffer(v or b"", max(len(v or b""), 1)) for v in self.values]
        self.arr = (OString * max(n, 1))()
        for i, (v, b) in enumerate(zip(self.values, self._bufs)):
            self.arr[i] = OString(C.cast(b, C.c_void_p).value, len(v or b""))
        valid = np.array([v is not None for v in self.values], dtype=bool)
        self.validity = None if valid.all() else validity_from_mask(valid)
        self.data = np.zeros(0, dtype=np.int8)  # unused (the ostrings are in self.arr)
        self.upd = None
        self.upd_valid = None
        if updates is not None:
            r, v, ver = updates[:3]
            vals = np.array([0 if x is None else string_ref(x) for x in v], dtype=np.int64)
            self.upd = (np.ascontiguousarray(r, dtype=np.int64), vals, np.ascontiguousarray(ver, dtype=np.uint64))
            ok = updates[3] if len(updates) > 3 and updates[3] is not None else np.array([x is not None for x in v])
            self.upd_valid = np.ascontiguousarray(ok, dtype=np.uint8)

    def ocol(self) -> OCol:
        c = OCol()
        c.type = OTYPE_VARCHAR
        c.data = C.addressof(self.arr)
        c.validity = self.validity.ctypes.data if self.validity is not None else None
        if self.upd is not None:
            c.n_updates = len(self.upd[0])
            c.upd_rows, c.upd_values, c.upd_version = (a.ctypes.data for a in self.upd)
            c.upd_valid = self.upd_valid.ctypes.data
        return c

    def decode(self, addrs, valid=None):
        """Fetched values (ostring addresses) → bytes (None where not valid)."""
        from cubit_amd.filters import string_at

        base, size = C.addressof(self.arr), C.sizeof(OString)
        out = []
        for i, a in enumerate(np.asarray(addrs, dtype=np.int64).tolist()):
            if valid is not None and not valid[i]:
                out.append(None)
            elif base <= a < base + size * len(self.values):
                out.append(self.values[(a - base) // size])
            else:
                out.append(string_at(a))
        return out


class OHuge(C.Structure):
    """hugeint_t / uhugeint_t: {lower, upper} (hugeint.hpp)."""

    _fields_ = [("lower", C.c_uint64), ("upper", C.c_uint64)]


_HUGES = {}  # int -> OHuge, kept for the life of the process
_HUGE_AT = {}  # address -> int


def huge_ref(v: int) -> int:
    """The address of a persistent ohuge holding the 128-bit integer v (negative: two's
    complement): how a HUGEINT / UHUGEINT constant or update value reaches the oracle."""
    v = int(v)
    if v not in _HUGES:
        u = v & ((1 << 128) - 1)
        h = OHuge(u & (2 ** 64 - 1), u >> 64)
        _HUGES[v] = h
        _HUGE_AT[C.addressof(h)] = v
    return C.addressof(_HUGES[v])


class HugeColumn(Column):
    """A HUGEINT (signed=True) / UHUGEINT column as the oracle sees it: an ohuge per row from
    Python ints, NULL rows from None; update values are ints (or None) carried as ohuge
    addresses; fetch hands back addresses — decode() turns them into ints."""

    def __init__(self, values, signed=True, updates=None):
        from cubit_amd.datagen import validity_from_mask

        self.signed = signed
        self.values = [None if v is None else int(v) for v in values]
        lo, hi = (-(1 << 127), (1 << 127) - 1) if signed else (0, (1 << 128) - 1)
        assert all(v is None or lo <= v <= hi for v in self.values)
        n = len(self.values)
        self.arr = (OHuge * max(n, 1))()
        for i, v in enumerate(self.values):
            u = (v or 0) & ((1 << 128) - 1)
            self.arr[i] = OHuge(u & (2 ** 64 - 1), u >> 64)
        valid = np.array([v is not None for v in self.values], dtype=bool)
        self.validity = None if valid.all() else validity_from_mask(valid)
        self.data = np.zeros(0, dtype=np.int8)  # unused (the ohuges are in self.arr)
        self.upd = None
        self.upd_valid = None
        if updates is not None:
            r, v, ver = updates[:3]
            vals = np.array([0 if x is None else huge_ref(x) for x in v], dtype=np.int64)
            self.upd = (np.ascontiguousarray(r, dtype=np.int64), vals, np.ascontiguousarray(ver, dtype=np.uint64))
            ok = updates[3] if len(updates) > 3 and updates[3] is not None else np.array([x is not None for x in v])
            self.upd_valid = np.ascontiguousarray(ok, dtype=np.uint8)

    def ocol(self) -> OCol:
        c = OCol()
        c.type = OTYPE_INT128 if self.signed else OTYPE_UINT128
        c.data = C.addressof(self.arr)
        c.validity = self.validity.ctypes.data if self.validity is not None else None
        if self.upd is not None:
            c.n_updates = len(self.upd[0])
            c.upd_rows, c.upd_values, c.upd_version = (a.ctypes.data for a in self.upd)
            c.upd_valid = self.upd_valid.ctypes.data
        return c

    def decode(self, addrs, valid=None):
        """Fetched values (ohuge addresses) → ints (None where not valid)."""
        base, size = C.addressof(self.arr), C.sizeof(OHuge)
        out = []
        for i, a in enumerate(np.asarray(addrs, dtype=np.int64).tolist()):
            if valid is not None and not valid[i]:
                out.append(None)
            elif base <= a < base + size * len(self.values):
                out.append(self.values[(a - base) // size])
            else:
                out.append(_HUGE_AT[a])
        return out


class Mvcc:
    def __init__(self, start_time: int, transaction_id: int, inserted: Optional[np.ndarray] = None,
                 deleted: Optional[np.ndarray] = None):
        self.inserted = None if inserted is None else np.ascontiguousarray(inserted, dtype=np.uint64)
        self.deleted = None if deleted is None else np.ascontiguousarray(deleted, dtype=np.uint64)
        self.s = OMvcc(self.inserted.ctypes.data if self.inserted is not None else None,
                       self.deleted.ctypes.data if self.deleted is not None else None, start_time, transaction_id)


def _scan_struct(columns: Sequence[Column], plan, n_rows: int, row_base: int, tx: Optional[Mvcc], canonical: bool):
    ocols = (OCol * len(columns))(*[c.ocol() for c in columns])
    nodes = (OFilter * max(len(plan.nodes), 1))()
    for i, (k, cmp, col, nc, const) in enumerate(plan.nodes):
        nodes[i] = OFilter(k, cmp, col, nc, const)
    pushed = (OPushed * max(len(plan.pushed), 1))(*[OPushed(c, r) for c, r in plan.pushed])
    s = OScan()
    s.cols = ocols
    s.n_cols = len(columns)
    s.n_pushed = len(plan.pushed)
    s.pushed = pushed
    s.nodes = nodes
    s.residual_root = plan.residual_root
    s.canonical = 1 if canonical else 0
    s.n_rows = n_rows
    s.row_base = row_base
    s.tx = C.pointer(tx.s) if tx is not None else None
    keep = (ocols, nodes, pushed, columns, tx)
    return s, keep


def table_scan(columns: Sequence[Column], plan, n_rows: int, row_base: int = 0, tx: Optional[Mvcc] = None,
               canonical: bool = True) -> np.ndarray:
    """RowGroup::TemplatedScan restatement → qualifying row ids (per-vector sel order; with
    canonical=True each vector's ids are sorted, so the whole output is ascending)."""
    s, keep = _scan_struct(columns, plan, n_rows, row_base, tx, canonical)
    out = np.empty(max(n_rows, 1), dtype=np.int64)
    n = lib().oracle_table_scan(C.byref(s), out.ctypes.data, n_rows)
    assert n >= 0
    return out[:n].copy()


def table_scan_mt(columns: Sequence[Column], plan, n_rows: int, threads: int, row_base: int = 0,
                  tx: Optional[Mvcc] = None) -> Tuple[int, int]:
    """Morsel-driven multi-threaded scan (timing leg): returns (count, sum of row ids)."""
    s, keep = _scan_struct(columns, plan, n_rows, row_base, tx, False)
    sm = C.c_uint64()
    n = lib().oracle_table_scan_mt(C.byref(s), threads, C.byref(sm))
    return int(n), int(sm.value)


def fetch(column: Column, rowids: np.ndarray, row_base: int = 0, tx: Optional[Mvcc] = None,
          with_valid: bool = False):
    """ColumnData::FetchRow per row id: values (0 at NULL rows), and with_valid=True also the
    validity (bool per row) — (values, valid)."""
    rowids = np.ascontiguousarray(rowids, dtype=np.int64)
    out = np.empty(max(len(rowids), 1), dtype=np.int64)
    valid = np.empty(max(len(rowids), 1), dtype=np.uint8)
    c = column.ocol()
    rc = lib().oracle_fetch(C.byref(c), C.pointer(tx.s) if tx is not None else None, rowids.ctypes.data,
                            len(rowids), row_base, out.ctypes.data, valid.ctypes.data)
    assert rc == 0
    if with_valid:
        return out[: len(rowids)], valid[: len(rowids)].astype(bool)
    return out[: len(rowids)]


def sum_product(a: np.ndarray, b: np.ndarray, rowids: np.ndarray, row_base: int = 0) -> int:
    rowids = np.ascontiguousarray(rowids, dtype=np.int64)
    lo = C.c_uint64()
    hi = C.c_int64()
    lib().oracle_sum_product(a.ctypes.data, b.ctypes.data, rowids.ctypes.data, len(rowids), row_base, C.byref(lo),
                             C.byref(hi))
    return (int(hi.value) << 64) + int(lo.value)


def bitmap_eval(leaves: Sequence[np.ndarray], prog: Sequence[int], n_rows: int, row_base: int = 0):
    """CPU bitmap evaluator: returns (row ids, result words)."""
    arrs = [np.ascontiguousarray(x, dtype=np.uint64) for x in leaves]
    ptrs = (C.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])
    p = (C.c_int32 * len(prog))(*prog)
    nw = (n_rows + 63) // 64
    words = np.empty(nw, dtype=np.uint64)
    out = np.empty(max(n_rows, 1), dtype=np.int64)
    n = lib().oracle_bitmap_eval(ptrs, p, len(prog), n_rows, row_base, out.ctypes.data, n_rows, words.ctypes.data)
    return out[:n].copy(), words


def build_bitvector(column: Column, n_rows: int, cmp: int, constant: int) -> np.ndarray:
    words = np.empty((n_rows + 63) // 64, dtype=np.uint64)
    c = column.ocol()
    lib().oracle_build_bitvector(C.byref(c), n_rows, cmp, constant, words.ctypes.data)
    return words


def xor_hash(rowids: np.ndarray) -> int:
    rowids = np.ascontiguousarray(rowids, dtype=np.int64)
    return int(lib().oracle_xor_hash(rowids.ctypes.data, len(rowids)))


# ---------------------------------------------------------------- DuckDB BITPACKING (bitpacking_ref.c)

BP_MODES = {"auto": 1, "constant": 2, "constant_delta": 3, "delta_for": 4, "for": 5}
BP_MODE_NAMES = {v: k for k, v in BP_MODES.items()}
DUCKDB_BLOCK_SIZE = 262144 - 8  # Storage::BLOCK_SIZE (storage_info.hpp:40-45)


class BitpackedColumn:
    """Segments of one column in DuckDB's BITPACKING format: all segment images concatenated
    in `data`, with per-segment byte offsets / sizes / row counts."""

    def __init__(self, data, seg_off, seg_size, seg_count, dtype):
        self.data, self.seg_off, self.seg_size, self.seg_count, self.dtype = data, seg_off, seg_size, seg_count, dtype

    @property
    def n_rows(self) -> int:
        return int(self.seg_count.sum())


BP_DTYPES = tuple(np.dtype(d) for d in (np.int8, np.int16, np.int32, np.int64,
                                           np.uint8, np.uint16, np.uint32, np.uint64))


def bp_ttype(dtype) -> int:
    """The restatement's value type code: byte size | 0x100 when unsigned."""
    dt = np.dtype(dtype)
    assert dt in BP_DTYPES, dt
    return dt.itemsize | (0x100 if dt.kind == "u" else 0)


def bp_compress(values: np.ndarray, valid: Optional[np.ndarray] = None, mode: str = "auto",
                block_size: int = DUCKDB_BLOCK_SIZE) -> Optional[BitpackedColumn]:
    """Compress like DuckDB's checkpoint would with force_bitpacking_mode=`mode` (None when
    the column is not bitpackable, e.g. a group whose max - min overflows). `values` may be
    any integral type DuckDB bit-packs (TINYINT … BIGINT, UTINYINT … UBIGINT)."""
    values = np.ascontiguousarray(values)
    ttype = bp_ttype(values.dtype)
    n = len(values)
    vb = None if valid is None else np.ascontiguousarray(valid, dtype=np.uint8)
    cap = n * values.itemsize * 2 + (n // 2048 + 8) * 64 + 4 * block_size
    out = np.zeros(cap, dtype=np.uint8)
    max_segs = cap // 64 + 16
    so = np.zeros(max_segs, dtype=np.uint64)
    ss = np.zeros(max_segs, dtype=np.uint64)
    sc = np.zeros(max_segs, dtype=np.uint64)
    ns = C.c_uint32()
    rc = lib().oracle_bp_compress(values.ctypes.data, ttype, vb.ctypes.data if vb is not None else None, n,
                                  BP_MODES[mode], block_size, out.ctypes.data, cap, so.ctypes.data, ss.ctypes.data,
                                  sc.ctypes.data, max_segs, C.byref(ns))
    if rc == 1:
        return None
    assert rc == 0, rc
    k = ns.value
    used = int(so[k - 1] + ss[k - 1]) if k else 0
    return BitpackedColumn(out[:used].copy(), so[:k].copy(), ss[:k].copy(), sc[:k].copy(), values.dtype)


def bp_decode(col: BitpackedColumn) -> np.ndarray:
    out = np.zeros(max(col.n_rows, 1), dtype=col.dtype)
    rc = lib().oracle_bp_decode(col.data.ctypes.data, col.seg_off.ctypes.data, col.seg_count.ctypes.data,
                                len(col.seg_off), bp_ttype(col.dtype), out.ctypes.data)
    assert rc == 0
    return out[:col.n_rows]


def bp_group_modes(col: BitpackedColumn):
    cap = col.n_rows // 2048 + len(col.seg_off) + 1
    m = np.zeros(cap, dtype=np.uint8)
    k = lib().oracle_bp_group_modes(col.data.ctypes.data, col.seg_off.ctypes.data, col.seg_count.ctypes.data,
                                    len(col.seg_off), m.ctypes.data, cap)
    return [BP_MODE_NAMES.get(int(x), "invalid") for x in m[:k]]


# ------------------------------------------------------------------ RLE segments (rle.cpp)
RLE_MAX_COUNT = 65535  # NumericLimits<rle_count_t>::Maximum(), rle_count_t = uint16_t (rle.cpp:13)


def rle_compress(values, valid=None, block_size: int = 262144, row_group: int = 122880):
    """DuckDB's RLE compressor restated (src/storage/compression/rle.cpp): one RLECompressState per
    row group (a column checkpoint), RLEState::Update (:45-78) — a NULL row only lengthens the
    current run (leading NULLs join the first valid value's run), a run reaching 65,535 rows is
    written and the next entry starts at 0, so a run of a multiple of 65,535 rows leaves a
    zero-length entry behind; NULL-only runs carry NullValue<T> (numeric_limits<T>::min) —
    WriteValue (:166-188: a segment holds at most (block_size - 8) / (sizeof(T) + 2) entries) and
    FlushSegment (:190-205: the run lengths moved next to the values at AlignValue(8 + n·sizeof(T)),
    that offset in the 8-byte header). Returns (bytes uint8, segment offsets, segment row counts),
    segments 8-aligned and back to back."""
    v = np.ascontiguousarray(values)
    dt = v.dtype
    assert dt.kind in "iu", dt
    n = len(v)
    ok = np.ones(n, bool) if valid is None else np.asarray(valid, bool)
    null_value = np.iinfo(dt).min
    max_entries = (block_size - 8) // (dt.itemsize + 2)
    segs = []
    for g0 in range(0, n, row_group):
        gv, gok = v[g0:g0 + row_group], ok[g0:g0 + row_group]
        m = len(gv)
        entries = []  # (value, count) in write order
        first = int(np.argmax(gok)) if gok.any() else m
        for _ in range(first // RLE_MAX_COUNT):  # leading NULLs reaching the limit: written as NullValue
            entries.append((null_value, RLE_MAX_COUNT))
        lead = first % RLE_MAX_COUNT
        if first == m:
            entries.append((null_value, lead))  # Finalize flushes the NULL-only run, even when empty
        else:
            # the value each row's run carries: the last valid value at or before it
            idx = np.where(gok, np.arange(m), 0)
            np.maximum.accumulate(idx, out=idx)
            filled = gv[idx[first:]]
            starts = np.flatnonzero(np.concatenate([[True], filled[1:] != filled[:-1]]))
            lens = np.diff(np.concatenate([starts, [len(filled)]]))
            lens[0] += lead
            for s0, L in zip(starts.tolist(), lens.tolist()):
                val = filled[s0]
                entries += [(val, RLE_MAX_COUNT)] * (L // RLE_MAX_COUNT)
                entries.append((val, L % RLE_MAX_COUNT))  # 0 after a multiple of the limit
        for c0 in range(0, len(entries), max_entries):
            chunk = entries[c0:c0 + max_entries]
            k = len(chunk)
            off = (8 + dt.itemsize * k + 7) // 8 * 8
            seg = bytearray(off + 2 * k)
            seg[:8] = int(off).to_bytes(8, "little")
            seg[8:8 + dt.itemsize * k] = np.array([e[0] for e in chunk], dtype=dt.newbyteorder("<")).tobytes()
            seg[off:] = np.array([e[1] for e in chunk], dtype="<u2").tobytes()
            segs.append((bytes(seg), sum(e[1] for e in chunk)))
    offs, data = [], bytearray()
    for seg, _ in segs:
        data += bytes((-len(data)) % 8)
        offs.append(len(data))
        data += seg
    return (np.frombuffer(bytes(data) or b"\0", dtype=np.uint8).copy(), np.array(offs, np.uint64),
            np.array([r for _, r in segs], np.uint64))


def rle_decode(data, seg_offsets, seg_rows, dtype) -> np.ndarray:
    """RLEScanState restated (rle.cpp:248-277, RLEScanPartial :335-380): from each segment's
    header offset, run lengths are read until they cover the segment's rows, each run's value
    repeated; the values as T."""
    dt = np.dtype(dtype)
    b = np.asarray(data, np.uint8).tobytes()
    out = []
    for o, rows in zip(np.asarray(seg_offsets).tolist(), np.asarray(seg_rows).tolist()):
        off = int.from_bytes(b[o:o + 8], "little")
        vals, lens, covered, k = [], [], 0, 0
        while covered < rows:
            L = int.from_bytes(b[o + off + 2 * k:o + off + 2 * k + 2], "little")
            vals.append(np.frombuffer(b, dtype=dt.newbyteorder("<"), count=1, offset=o + 8 + k * dt.itemsize)[0])
            lens.append(L)
            covered += L
            k += 1
        assert covered == rows
        out.append(np.repeat(np.array(vals, dtype=dt), lens))
    return np.concatenate(out) if out else np.zeros(0, dt)
