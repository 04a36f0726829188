"""Python handle over the C ABI: device context, device buffers, table partitions.

Everything here is a thin ctypes wrapper; the work happens in libcubitgpu.so.
"""
from __future__ import annotations

import ctypes as C
import weakref
from typing import Dict, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .filters import Plan, Residual, TableFilterSet, serialize, to_ctypes


class Context:
    """cubit_ctx: one per device; optionally bound to an external HIP stream."""

    def __init__(self, device: int = 0, stream: Optional[int] = None):
        self.lib = L.gpu_lib()
        h = C.c_void_p()
        L.check(self.lib.cubit_ctx_create(device, C.byref(h)))
        self.handle = h
        self.device = device
        self._tables = weakref.WeakSet()  # partitions to destroy before the context
        if stream is not None:
            L.check(self.lib.cubit_ctx_set_stream(h, C.c_void_p(stream)))

    def set_stream(self, stream: Optional[int]) -> None:
        L.check(self.lib.cubit_ctx_set_stream(self.handle, C.c_void_p(stream or 0)))

    def set_decode_kernel(self, kernel: int) -> None:
        """L.DECODE_AUTO (measured policy), L.DECODE_PAIRS or L.DECODE_RUNS."""
        L.check(self.lib.cubit_ctx_set_decode_kernel(self.handle, kernel))

    def set_lookback_spins(self, spins: int) -> None:
        """Polls of an earlier tile's flag before the look-back decode counts that tile itself
        (0 = library default); a small value forces the expiry path."""
        L.check(self.lib.cubit_ctx_set_lookback_spins(self.handle, spins))

    def last_decode_kernel(self) -> int:
        k = C.c_int()
        L.check(self.lib.cubit_ctx_last_decode_kernel(self.handle, C.byref(k)))
        return int(k.value)

    def enable_timing(self, on: bool = True) -> None:
        L.check(self.lib.cubit_ctx_enable_timing(self.handle, 1 if on else 0))

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        L.check(self.lib.cubit_last_kernel_ms(self.handle, C.byref(ms)))
        return float(ms.value)

    def timing_reset(self) -> None:
        L.check(self.lib.cubit_ctx_timing_reset(self.handle))

    def kernel_times_ms(self, cap: int = 4096):
        arr = (C.c_float * cap)()
        n = C.c_uint32()
        L.check(self.lib.cubit_ctx_kernel_times(self.handle, arr, cap, C.byref(n)))
        return [float(arr[i]) for i in range(min(cap, n.value))]

    def set_repeat(self, reps: int) -> None:
        """Issue the next decode launch `reps` times back to back between two stream events."""
        L.check(self.lib.cubit_ctx_set_repeat(self.handle, int(reps)))

    def repeat_time(self):
        """(mean ms per launch, launches) of the last repeated decode."""
        ms = C.c_double()
        n = C.c_uint32()
        L.check(self.lib.cubit_ctx_repeat_time(self.handle, C.byref(ms), C.byref(n)))
        return float(ms.value), int(n.value)

    def sync(self) -> None:
        L.check(self.lib.cubit_sync(self.handle))

    def last_tiles(self):
        """Tile directory of the last row-id materialisation: (int64 [n_tiles, 2] of
        {run start, run length}, rows per tile)."""
        d = C.c_void_p()
        n = C.c_uint32()
        rpt = C.c_uint64()
        L.check(self.lib.cubit_ctx_last_tiles(self.handle, C.byref(d), C.byref(n), C.byref(rpt)))
        out = np.empty(2 * n.value, dtype=np.uint64)
        if n.value:
            L.check(self.lib.cubit_memcpy_d2h(self.handle, out.ctypes.data, d, out.nbytes))
        return out.reshape(-1, 2), int(rpt.value)

    def check(self) -> None:
        L.check(self.lib.cubit_ctx_check(self.handle))

    def alloc(self, nbytes: int) -> "DeviceBuffer":
        return DeviceBuffer(self, nbytes)

    def upload(self, arr: np.ndarray) -> "DeviceBuffer":
        arr = np.ascontiguousarray(arr)
        buf = DeviceBuffer(self, max(arr.nbytes, 16))
        if arr.nbytes:
            L.check(self.lib.cubit_memcpy_h2d(self.handle, buf.ptr, arr.ctypes.data, arr.nbytes))
        return buf

    def close(self) -> None:
        if self.handle:
            for t in list(self._tables):
                t.close()
            self.lib.cubit_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceBuffer:
    def __init__(self, ctx: Context, nbytes: int):
        self.ctx = ctx
        self.nbytes = nbytes
        p = C.c_void_p()
        L.check(ctx.lib.cubit_dev_alloc(ctx.handle, nbytes, C.byref(p)))
        self.ptr = p

    @property
    def addr(self) -> int:
        return int(self.ptr.value or 0)

    def download(self, dtype, count: int) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        if count:
            L.check(self.ctx.lib.cubit_memcpy_d2h(self.ctx.handle, out.ctypes.data, self.ptr, out.nbytes))
        return out

    def zero(self) -> None:
        L.check(self.ctx.lib.cubit_memset_d(self.ctx.handle, self.ptr, 0, self.nbytes))

    def free(self) -> None:
        if self.ptr:
            self.ctx.lib.cubit_dev_free(self.ctx.handle, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            if self.ctx.handle:
                self.free()
        except Exception:
            pass


def runs_in_row_order(ids: np.ndarray, directory: np.ndarray) -> np.ndarray:
    """Concatenate the per-tile runs of a tile-run-order output in tile order (what a
    consumer iterating the directory sees)."""
    parts = [ids[int(s): int(s) + int(n)] for s, n in directory if n]
    return np.concatenate(parts) if parts else np.empty(0, dtype=np.int64)


def padded_words(n_rows: int) -> int:
    return int(L.gpu_lib().cubit_padded_words(n_rows))


def pack_strings(values):
    """A list of str / bytes / None as (bytes buffer, uint64 offsets[n + 1], valid bool[n]) — the
    layout cubit_dict_create / cubit_dict_encode take (None: a NULL row, an empty slot)."""
    parts = [b"" if v is None else (v.encode() if isinstance(v, str) else bytes(v)) for v in values]
    offs = np.zeros(len(parts) + 1, dtype=np.uint64)
    if parts:
        offs[1:] = np.cumsum([len(p) for p in parts], dtype=np.uint64)
    buf = np.frombuffer(b"".join(parts) or b"\0", dtype=np.uint8).copy()
    valid = np.array([v is not None for v in values], dtype=bool)
    return buf, offs, valid


class Dictionary:
    """cubit_dict: a VARCHAR column's order-preserving dictionary (the distinct strings in DuckDB's
    order; code = rank)."""

    def __init__(self, strings, lib=None):
        self.lib = lib or L.gpu_lib()
        buf, offs, valid = pack_strings([s for s in strings if s is not None])
        h = C.c_void_p()
        L.check(self.lib.cubit_dict_create(buf.ctypes.data, offs.ctypes.data, len(offs) - 1, C.byref(h)))
        self.handle = h

    def __len__(self):
        n = C.c_uint64()
        L.check(self.lib.cubit_dict_size(self.handle, C.byref(n)))
        return int(n.value)

    def entry(self, code: int) -> bytes:
        p, n = C.c_void_p(), C.c_uint64()
        L.check(self.lib.cubit_dict_entry(self.handle, int(code), C.byref(p), C.byref(n)))
        return C.string_at(p.value, n.value) if n.value else b""

    def entries(self):
        return [self.entry(i) for i in range(len(self))]

    def encode(self, values) -> Tuple[np.ndarray, np.ndarray]:
        """(int32 codes, bool valid) of a list of str / bytes / None."""
        from cubit_amd.datagen import validity_from_mask

        buf, offs, valid = pack_strings(values)
        codes = np.zeros(max(len(values), 1), dtype=np.int32)
        vw = validity_from_mask(valid)
        L.check(self.lib.cubit_dict_encode(self.handle, buf.ctypes.data, offs.ctypes.data, len(values),
                                           vw.ctypes.data, codes.ctypes.data))
        return codes[: len(values)], valid

    def lookup(self, s):
        b = s.encode() if isinstance(s, str) else bytes(s)
        buf = C.create_string_buffer(b, max(len(b), 1))
        lb, present = C.c_uint64(), C.c_int()
        L.check(self.lib.cubit_dict_lookup(self.handle, buf, len(b), C.byref(lb), C.byref(present)))
        return int(lb.value), bool(present.value)

    def close(self):
        if self.handle:
            self.lib.cubit_dict_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class CubitTable:
    """A row-range partition [row_base, row_base + n_rows) resident on one device."""

    def __init__(self, ctx: Context, n_rows: int, row_base: int = 0):
        self.ctx = ctx
        self.lib = ctx.lib
        self.n_rows = int(n_rows)
        self.row_base = int(row_base)
        h = C.c_void_p()
        L.check(self.lib.cubit_table_create(ctx.handle, self.n_rows, self.row_base, C.byref(h)))
        self.handle = h
        ctx._tables.add(self)
        self.types: Dict[int, int] = {}
        self.huge: Dict[int, bool] = {}  # HUGEINT (True) / UHUGEINT (False) dictionary columns
        self._keep = []

    def add_column(self, col: int, data: np.ndarray, validity: Optional[np.ndarray] = None) -> None:
        """Register a column of any integral dtype: int32 / int64 as they are, the narrower and
        unsigned ones widened by the library into an INT32 / INT64 column (uint64 below 2^63);
        float32 / float64 as a FLOAT / DOUBLE column (DuckDB's floating-point comparisons)."""
        data = np.ascontiguousarray(data)
        if data.dtype.name not in L.COLUMN_TYPES:
            raise TypeError(f"unsupported dtype {data.dtype}")
        t = L.COLUMN_TYPES[data.dtype.name]
        assert data.shape[0] == self.n_rows
        vptr = None
        if validity is not None:
            validity = np.ascontiguousarray(validity, dtype=np.uint64)
            vptr = validity.ctypes.data
        L.check(self.lib.cubit_table_add_column(self.handle, col, t, data.ctypes.data, vptr, 0))
        self.types[col] = self.column_data(col)[1]

    def add_bitpacked_column(self, col: int, data: np.ndarray, seg_offsets: np.ndarray, seg_rows: np.ndarray,
                             dtype, validity: Optional[np.ndarray] = None) -> None:
        """A column given as DuckDB BITPACKING segment images (uint8 bytes, per-segment byte
        offsets and row counts); unpacked on the GPU (K5). `dtype` is the segments' T (any
        integral type DuckDB bit-packs); the column holds the values as INT32 (8-, 16- and
        32-bit signed T, 8- and 16-bit unsigned) or INT64 (UINT32, INT64, UINT64 below 2^63)."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        so = np.ascontiguousarray(seg_offsets, dtype=np.uint64)
        sr = np.ascontiguousarray(seg_rows, dtype=np.uint64)
        vw = None if validity is None else np.ascontiguousarray(validity, dtype=np.uint64)
        typ = L.SEGMENT_TYPES[np.dtype(dtype).name]
        L.check(self.lib.cubit_table_add_bitpacked_column(self.handle, col, typ, data.ctypes.data, data.nbytes,
                                                          so.ctypes.data, sr.ctypes.data, len(so),
                                                          vw.ctypes.data if vw is not None else None))
        self.types[col] = self.column_data(col)[1]

    def add_rle_column(self, col: int, data: np.ndarray, seg_offsets: np.ndarray, seg_rows: np.ndarray,
                       dtype, validity: Optional[np.ndarray] = None) -> None:
        """A column given as DuckDB RLE segment images (uint8 bytes, per-segment byte offsets and
        row counts); the runs are read on the host and expanded on the GPU. `dtype` and the column
        held as for add_bitpacked_column."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        so = np.ascontiguousarray(seg_offsets, dtype=np.uint64)
        sr = np.ascontiguousarray(seg_rows, dtype=np.uint64)
        vw = None if validity is None else np.ascontiguousarray(validity, dtype=np.uint64)
        typ = L.SEGMENT_TYPES[np.dtype(dtype).name]
        L.check(self.lib.cubit_table_add_rle_column(self.handle, col, typ, data.ctypes.data if data.size else None,
                                                    data.nbytes, so.ctypes.data, sr.ctypes.data, len(so),
                                                    vw.ctypes.data if vw is not None else None))
        self.types[col] = self.column_data(col)[1]

    def add_segment_column(self, col: int, segments, dtype, validity: Optional[np.ndarray] = None) -> None:
        """A column given as DuckDB segments of mixed codecs, in row order: a list of
        (codec, payload, rows) — CODEC_CONSTANT with the value as payload, the other codecs with the
        segment's bytes (UNCOMPRESSED: rows x T)."""
        buf = bytearray()
        offs, rows, codecs, consts = [], [], [], []
        for codec, payload, n in segments:
            buf += bytes((-len(buf)) % 16)
            offs.append(len(buf))
            if codec == L.CODEC_CONSTANT:
                consts.append(int(payload))
            else:
                consts.append(0)
                buf += bytes(np.asarray(payload, dtype=np.uint8) if not isinstance(payload, (bytes, bytearray))
                             else payload)
            rows.append(n)
            codecs.append(codec)
        data = np.frombuffer(bytes(buf) or b"\0", dtype=np.uint8).copy()
        so = np.array(offs, np.uint64)
        sr = np.array(rows, np.uint64)
        sc = np.array(codecs, np.int32)
        cv = np.array([c - (1 << 64) if c >= 1 << 63 else c for c in consts], np.int64)
        vw = None if validity is None else np.ascontiguousarray(validity, dtype=np.uint64)
        typ = L.SEGMENT_TYPES[np.dtype(dtype).name]
        L.check(self.lib.cubit_table_add_segment_column(self.handle, col, typ, data.ctypes.data, len(buf), so.ctypes.data,
                                                        sr.ctypes.data, sc.ctypes.data, cv.ctypes.data, len(so),
                                                        vw.ctypes.data if vw is not None else None))
        self.types[col] = self.column_data(col)[1]

    def add_string_column(self, col: int, values, dictionary: Optional[Dictionary] = None) -> Dictionary:
        """Register a VARCHAR column from a list of str / bytes / None (NULL): encoded against
        `dictionary` (default: one built from the values) and held as int32 codes."""
        from cubit_amd.datagen import validity_from_mask

        d = dictionary or Dictionary(values, self.lib)
        codes, valid = d.encode(values)
        assert len(codes) == self.n_rows
        vw = validity_from_mask(valid) if not valid.all() else None
        L.check(self.lib.cubit_table_add_dict_column(self.handle, col, d.handle, codes.ctypes.data,
                                                     vw.ctypes.data if vw is not None else None, 0))
        self.types[col] = L.TYPE_VARCHAR
        self._keep.append(d)
        return d

    def add_huge_column(self, col: int, values, signed: bool = True,
                        dictionary: Optional[Dictionary] = None) -> Dictionary:
        """Register a HUGEINT (signed) / UHUGEINT column from a list of Python ints / None (NULL):
        a dictionary column over the values' 16-byte order keys (filters.key128), its codes the
        values' ranks. Constants and index keys on it are key128(...) bytes; probed codes map back
        through dictionary.entry + filters.value128."""
        from cubit_amd.filters import key128

        keys = [None if v is None else key128(v, signed) for v in values]
        d = self.add_string_column(col, keys, dictionary)
        self.huge[col] = signed  # a dictionary column (types: VARCHAR) whose keys are 128-bit values
        return d

    def column_data(self, col: int):
        """(device pointer, CUBIT type) of a registered column's values."""
        ptr, typ = C.c_void_p(), C.c_int()
        L.check(self.lib.cubit_table_column_data(self.handle, col, C.byref(ptr), C.byref(typ)))
        return int(ptr.value or 0), int(typ.value)

    def download_column(self, col: int) -> np.ndarray:
        ptr, typ = self.column_data(col)
        dt = {L.TYPE_INT32: np.int32, L.TYPE_FLOAT: np.float32, L.TYPE_DOUBLE: np.float64, L.TYPE_UINT64: np.uint64,
              L.TYPE_VARCHAR: np.int32}.get(typ, np.int64)
        out = np.empty(self.n_rows, dtype=dt)
        if self.n_rows:
            L.check(self.lib.cubit_memcpy_d2h(self.ctx.handle, out.ctypes.data, C.c_void_p(ptr), out.nbytes))
        return out

    def add_device_column(self, col: int, dptr: int, type_: int, validity_dptr: Optional[int] = None) -> None:
        L.check(self.lib.cubit_table_add_column(self.handle, col, type_, C.c_void_p(dptr),
                                                C.c_void_p(validity_dptr) if validity_dptr else None, 1))
        self.types[col] = type_

    def build_index(self, col: int, encoding: int = L.INDEX_RANGE, keys: Optional[Sequence[int]] = None) -> None:
        if keys is not None and len(keys):
            # FLOAT / DOUBLE columns: keys given as floats cross as their bit patterns
            typ = self.types.get(col)
            if typ == L.TYPE_VARCHAR:  # string keys cross as addresses of cubit_strings
                from cubit_amd.filters import key128, string_ref

                if col in self.huge:  # HUGEINT / UHUGEINT keys given as ints: their order keys
                    keys = [key128(x, self.huge[col]) for x in keys]
                k = np.array([string_ref(x) for x in keys], dtype=np.int64)
            elif typ == L.TYPE_UINT64:  # UBIGINT keys as their bits
                k = np.ascontiguousarray(np.asarray(keys, dtype=np.uint64)).view(np.int64)
            else:
                is_fp = typ in (L.TYPE_FLOAT, L.TYPE_DOUBLE) and np.asarray(keys).dtype.kind == "f"
                k = L.fp_bits(keys, typ) if is_fp else np.ascontiguousarray(np.asarray(keys, dtype=np.int64))
            L.check(self.lib.cubit_table_build_index(self.handle, col, encoding, k.ctypes.data, len(k)))
        else:
            L.check(self.lib.cubit_table_build_index(self.handle, col, encoding, None, 0))

    def save_index(self, col: int, encoding: int, path) -> None:
        L.check(self.lib.cubit_table_save_index(self.handle, col, encoding, str(path).encode()))

    def load_index(self, col: int, path) -> None:
        L.check(self.lib.cubit_table_load_index(self.handle, col, str(path).encode()))

    def index_info(self, col: int):
        n = C.c_uint32()
        b = C.c_uint64()
        L.check(self.lib.cubit_table_index_info(self.handle, col, C.byref(n), C.byref(b)))
        return int(n.value), int(b.value)

    def set_deletes(self, rows: np.ndarray, ids: np.ndarray) -> None:
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        ids = np.ascontiguousarray(ids, dtype=np.uint64)
        L.check(self.lib.cubit_table_set_deletes(self.handle, rows.ctypes.data, ids.ctypes.data, len(rows)))

    def set_inserts(self, row_begin: np.ndarray, row_end: np.ndarray, ids: np.ndarray) -> None:
        """Insert versions: disjoint row ranges [begin, end) with the inserting transaction's id."""
        b = np.ascontiguousarray(row_begin, dtype=np.int64)
        e = np.ascontiguousarray(row_end, dtype=np.int64)
        i = np.ascontiguousarray(ids, dtype=np.uint64)
        L.check(self.lib.cubit_table_set_inserts(self.handle, b.ctypes.data, e.ctypes.data, i.ctypes.data, len(b)))

    def set_updates(self, col: int, rows: np.ndarray, values: np.ndarray, versions: np.ndarray,
                    valid: Optional[np.ndarray] = None) -> None:
        """Update records (row, value, version), chronological. valid (bool per record, optional):
        False = the record sets the row NULL (cubit_table_set_updates_nullable)."""
        rows = np.ascontiguousarray(rows, dtype=np.int64)
        typ = self.types.get(col)
        if typ in (L.TYPE_FLOAT, L.TYPE_DOUBLE) and np.asarray(values).dtype.kind == "f":
            values = L.fp_bits(values, typ)  # FLOAT / DOUBLE values cross as their bit patterns
        if np.asarray(values).dtype == np.uint64:
            values = np.ascontiguousarray(values).view(np.int64)  # UBIGINT values as their bits
        values = np.ascontiguousarray(values, dtype=np.int64)
        versions = np.ascontiguousarray(versions, dtype=np.uint64)
        if valid is None:
            L.check(self.lib.cubit_table_set_updates(self.handle, col, rows.ctypes.data, values.ctypes.data,
                                                     versions.ctypes.data, len(rows)))
            return
        v = np.ascontiguousarray(valid, dtype=np.uint8)
        L.check(self.lib.cubit_table_set_updates_nullable(self.handle, col, rows.ctypes.data, values.ctypes.data,
                                                          v.ctypes.data, versions.ctypes.data, len(rows)))

    # ------------------------------------------------------------------ index maintenance
    def append(self, columns: Dict[int, np.ndarray], validity: Optional[Dict[int, np.ndarray]] = None,
               insert_id: int = 0) -> None:
        """Append rows (RowGroupCollection::Append + BoundIndex::Append): one array per
        registered column, of the column's dtype; validity = LSB-first words per column (bit 0
        = the first appended row), absent = all valid. insert_id != 0 hides the rows from
        snapshots that predate it (an insert range)."""
        cols = sorted(columns)
        n_new = len(columns[cols[0]]) if cols else 0
        keep = []
        for c in cols:
            a = np.ascontiguousarray(columns[c])
            want = {L.TYPE_INT32: np.int32, L.TYPE_FLOAT: np.float32, L.TYPE_DOUBLE: np.float64,
                    L.TYPE_VARCHAR: np.int32, L.TYPE_UINT64: np.uint64}.get(self.types.get(c), np.int64)
            if a.dtype != want or len(a) != n_new:
                raise ValueError(f"column {c}: {len(a)} values of {a.dtype}, want {n_new} of {np.dtype(want)}")
            keep.append(a)
        vkeep = []
        for c in cols:
            v = None if validity is None else validity.get(c)
            vkeep.append(None if v is None else np.ascontiguousarray(v, dtype=np.uint64))
        cid = (C.c_int * max(len(cols), 1))(*cols)
        dptr = (C.c_void_p * max(len(cols), 1))(*[a.ctypes.data for a in keep])
        vptr = (C.c_void_p * max(len(cols), 1))(*[(v.ctypes.data if v is not None else None) for v in vkeep])
        L.check(self.lib.cubit_table_append(self.handle, n_new, cid, dptr, vptr, len(cols), int(insert_id)))
        self.n_rows += n_new

    def merge_updates(self, col: int, horizon: int) -> int:
        """Fold the update records of `col` below `horizon` into the base and its indexes."""
        n = C.c_uint64()
        L.check(self.lib.cubit_table_merge_updates(self.handle, col, int(horizon), C.byref(n)))
        return int(n.value)

    # ------------------------------------------------------------------ scan
    def scan_into(self, plan_nodes, rowids_dptr: int, capacity: int, count_dptr: int,
                  txn: Optional[L.Txn] = None, count_only: bool = False, ordered: bool = False,
                  zonemap: bool = True) -> None:
        """Asynchronous scan into caller-owned device buffers (the bench path)."""
        arr = plan_nodes if isinstance(plan_nodes, C.Array) else to_ctypes(plan_nodes)
        n = len(plan_nodes) if not isinstance(plan_nodes, C.Array) else len(arr)
        flags = (L.SCAN_COUNT_ONLY if count_only else 0) | (L.SCAN_ORDERED if ordered else 0)
        flags |= 0 if zonemap else L.SCAN_NO_ZONEMAP
        L.check(self.lib.cubit_table_scan(self.handle, arr, n, C.byref(txn) if txn is not None else None,
                                          C.c_void_p(rowids_dptr) if rowids_dptr else None, capacity,
                                          C.c_void_p(count_dptr), flags))

    def scan(self, filter_set: Optional[TableFilterSet] = None, residual: Optional[Residual] = None,
             txn: Optional[L.Txn] = None, capacity: Optional[int] = None, ordered: bool = True,
             zonemap: bool = True) -> np.ndarray:
        """Synchronous scan returning the global row ids as numpy int64: ascending with
        ordered=True (device ordered pass), else in tile-run order (see last_tiles())."""
        plan = serialize(filter_set, residual)
        cap = self.n_rows if capacity is None else capacity
        out = self.ctx.alloc(max(cap, 1) * 8)
        cnt = self.ctx.alloc(16)
        self.scan_into(plan.nodes, out.addr, cap, cnt.addr, txn, ordered=ordered, zonemap=zonemap)
        self.ctx.check()
        n = int(cnt.download(np.uint64, 1)[0])
        if n > cap:
            raise L.CubitError(L.ERR_CAPACITY, f"{n} rows qualify, capacity {cap}")
        return out.download(np.int64, n)

    def estimate_rows(self, filter_set: Optional[TableFilterSet] = None, residual: Optional[Residual] = None) -> int:
        """The planner's estimate of the qualifying rows (cubit_table_estimate_rows: zone
        statistics, no scan)."""
        plan = serialize(filter_set, residual)
        nodes = to_ctypes(plan.nodes)
        v = C.c_uint64()
        L.check(self.lib.cubit_table_estimate_rows(self.handle, nodes, len(plan.nodes), C.byref(v)))
        return int(v.value)

    def count(self, filter_set: Optional[TableFilterSet] = None, residual: Optional[Residual] = None,
              txn: Optional[L.Txn] = None, zonemap: bool = True) -> int:
        plan = serialize(filter_set, residual)
        cnt = self.ctx.alloc(16)
        self.scan_into(plan.nodes, 0, 0, cnt.addr, txn, count_only=True, zonemap=zonemap)
        self.ctx.check()
        return int(cnt.download(np.uint64, 1)[0])

    def probe(self, col: int, rowids_dptr: int, count_dptr: int, max_n: int, out_dptr: int,
              txn: Optional[L.Txn] = None) -> None:
        L.check(self.lib.cubit_table_probe(self.handle, col, C.byref(txn) if txn is not None else None,
                                           C.c_void_p(rowids_dptr), C.c_void_p(count_dptr), max_n,
                                           C.c_void_p(out_dptr)))

    def probe_validity(self, col: int, rowids_dptr: int, count_dptr: int, max_n: int, out_dptr: int,
                       valid_dptr: int, txn: Optional[L.Txn] = None) -> None:
        """The probe with NULL-ness: values (0 at NULL rows) and LSB-first validity words."""
        L.check(self.lib.cubit_table_probe_validity(self.handle, col, C.byref(txn) if txn is not None else None,
                                                    C.c_void_p(rowids_dptr), C.c_void_p(count_dptr), max_n,
                                                    C.c_void_p(out_dptr), C.c_void_p(valid_dptr)))

    def fetch(self, col: int, rowids: np.ndarray, txn: Optional[L.Txn] = None):
        """Synchronous probe of host row ids → (values, valid bool array), as the oracle's fetch."""
        ids = np.ascontiguousarray(rowids, dtype=np.int64)
        n = len(ids)
        d_ids, d_cnt = self.ctx.upload(ids), self.ctx.upload(np.array([n], dtype=np.uint64))
        d_out, d_val = self.ctx.alloc(max(n, 1) * 8), self.ctx.alloc(((n + 63) // 64 + 1) * 8)
        self.probe_validity(col, d_ids.addr, d_cnt.addr, n, d_out.addr, d_val.addr, txn)
        self.ctx.check()
        vals = d_out.download(np.int64, n)
        words = d_val.download(np.uint64, (n + 63) // 64)
        valid = np.unpackbits(words.view(np.uint8), bitorder="little")[:n].astype(bool)
        return vals, valid

    def sum_product(self, col_a: int, col_b: int, filter_set: Optional[TableFilterSet] = None,
                    residual: Optional[Residual] = None, txn: Optional[L.Txn] = None,
                    gather_b: bool = False, zonemap: bool = True, packed_a: bool = True) -> Tuple[int, int]:
        """SELECT sum(a*b), count(*) WHERE <filter> in one fused pass → (sum as a Python int
        of the 128-bit DECIMAL storage, qualifying rows)."""
        plan = serialize(filter_set, residual)
        arr = to_ctypes(plan.nodes)
        out = self.ctx.alloc(16)
        cnt = self.ctx.alloc(16)
        L.check(self.lib.cubit_table_sum_product(self.handle, arr, len(plan.nodes),
                                                 C.byref(txn) if txn is not None else None, col_a, col_b,
                                                 C.c_void_p(out.addr), C.c_void_p(cnt.addr),
                                                 (L.SUM_GATHER_B if gather_b else 0)
                                                 | (0 if zonemap else L.SUM_NO_ZONEMAP)
                                                 | (0 if packed_a else L.SUM_PLAIN_A)))
        self.ctx.check()
        lo, hi = (int(x) for x in out.download(np.int64, 2))
        n = int(cnt.download(np.uint64, 1)[0])
        out.free()
        cnt.free()
        return (hi << 64) + (lo & (2 ** 64 - 1)), n

    def last_sum_packed(self) -> bool:
        v = C.c_int()
        L.check(self.lib.cubit_table_last_sum_packed(self.handle, C.byref(v)))
        return bool(v.value)

    def last_sum_decode(self) -> int:
        v = C.c_uint32()
        L.check(self.lib.cubit_table_last_sum_decode(self.handle, C.byref(v)))
        return int(v.value)

    def column_statistics(self, col: int):
        """(min, max, has_null, has_no_null) of a column — DataTable::GetStatistics, widened by
        the column's update records; min = max = 0 when no row is valid."""
        lo, hi = C.c_int64(), C.c_int64()
        hn, hv = C.c_int(), C.c_int()
        L.check(self.lib.cubit_table_column_statistics(self.handle, col, C.byref(lo), C.byref(hi), C.byref(hn),
                                                       C.byref(hv)))
        return int(lo.value), int(hi.value), bool(hn.value), bool(hv.value)

    def use_packed_filter(self, on: bool = True) -> None:
        """Filter bitpacked columns straight from their segments, or from the plain column
        (the default: faster on MI355X)."""
        L.check(self.lib.cubit_table_use_packed_filter(self.handle, 1 if on else 0))

    def last_packed(self) -> int:
        v = C.c_uint32()
        L.check(self.lib.cubit_table_last_packed(self.handle, C.byref(v)))
        return int(v.value)

    def use_narrowing(self, on: bool = True) -> None:
        """Read unindexed (K0) comparison columns of a conjunction only at the rows its other
        filters keep, when they keep few (the default), or always in full."""
        L.check(self.lib.cubit_table_use_narrowing(self.handle, 1 if on else 0))

    def last_narrowed(self) -> int:
        v = C.c_uint32()
        L.check(self.lib.cubit_table_last_narrowed(self.handle, C.byref(v)))
        return int(v.value)

    def last_k0_order(self):
        """Columns of the K0 comparisons the last scan built, in build order (most selective
        first when narrowed)."""
        cap = 64
        arr = (C.c_int32 * cap)()
        n = C.c_uint32()
        L.check(self.lib.cubit_table_last_k0_order(self.handle, arr, cap, C.byref(n)))
        return [int(arr[i]) for i in range(min(cap, n.value))]

    def column_changed(self, col: int) -> None:
        """A caller-owned (device) column's values were rewritten: drop the statistics and zone
        classes the table derived from them."""
        L.check(self.lib.cubit_table_column_changed(self.handle, col))

    def last_zones(self):
        """(zones the last scan / sum_product evaluated, zones of the partition): fewer
        evaluated when the zonemaps skipped zones its filter is false on."""
        ev = C.c_uint32()
        nz = C.c_uint32()
        L.check(self.lib.cubit_table_last_zones(self.handle, C.byref(ev), C.byref(nz)))
        return int(ev.value), int(nz.value)

    def last_plan(self):
        k = C.c_uint32()
        p = C.c_uint32()
        L.check(self.lib.cubit_table_last_plan(self.handle, C.byref(k), C.byref(p)))
        return int(k.value), int(p.value)

    def close(self) -> None:
        # a partition never outlives its context (Context.close destroys it first)
        if self.handle and self.ctx.handle:
            self.lib.cubit_table_destroy(self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
