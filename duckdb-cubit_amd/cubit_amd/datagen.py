"""Input data for tests and the bench (numpy arrays, host memory).

* TPC-H lineitem Q6 columns: libcubit_datagen's restatement of the reference dbgen
  (csrc/tpch_lineitem_gen.cpp) — rows and row ids identical to DuckDB `CALL dbgen(sf=…)`.
* Synthetic uniform INT32 columns: splitmix64(seed, row) mod modulus.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib as L


@dataclass
class Lineitem:
    sf: float
    order_begin: int
    order_end: int
    row_base: int            # global row id of the first row
    l_shipdate: np.ndarray   # int32 DATE (days since epoch)
    l_discount: np.ndarray   # int64 DECIMAL(15,2)
    l_quantity: np.ndarray   # int64 DECIMAL(15,2)
    l_extendedprice: np.ndarray  # int64 DECIMAL(15,2)

    @property
    def n_rows(self) -> int:
        return int(self.l_shipdate.shape[0])


def tpch_orders(sf: float) -> int:
    return int(L.gen_lib().cubit_tpch_orders(sf))


def tpch_rows(sf: float, order_begin: int = 0, order_end: int | None = None, threads: int = 0) -> int:
    if order_end is None:
        order_end = tpch_orders(sf)
    return int(L.gen_lib().cubit_tpch_lineitem_rows(sf, order_begin, order_end, threads))


def tpch_lineitem(sf: float, order_begin: int = 0, order_end: int | None = None, threads: int = 0,
                  columns=("l_shipdate", "l_discount", "l_quantity", "l_extendedprice")) -> Lineitem:
    """lineitem rows of orders [order_begin, order_end) at scale factor sf."""
    g = L.gen_lib()
    if order_end is None:
        order_end = tpch_orders(sf)
    n = tpch_rows(sf, order_begin, order_end, threads)
    base = tpch_rows(sf, 0, order_begin, threads) if order_begin else 0
    want = set(columns)
    sd = np.empty(n if "l_shipdate" in want else 0, dtype=np.int32)
    di = np.empty(n if "l_discount" in want else 0, dtype=np.int64)
    qu = np.empty(n if "l_quantity" in want else 0, dtype=np.int64)
    ep = np.empty(n if "l_extendedprice" in want else 0, dtype=np.int64)

    def ptr(a):
        return a.ctypes.data if a.size else None

    w = g.cubit_tpch_lineitem_gen(sf, order_begin, order_end, ptr(sd), ptr(di), ptr(qu), ptr(ep), threads)
    assert w == n, (w, n)
    return Lineitem(sf, order_begin, order_end, base, sd, di, qu, ep)


def uniform_i32(seed: int, n: int, modulus: int, row_begin: int = 0, threads: int = 0) -> np.ndarray:
    out = np.empty(n, dtype=np.int32)
    rc = L.gen_lib().cubit_synth_uniform_i32(seed, row_begin, n, modulus, out.ctypes.data, threads)
    assert rc == 0
    return out


@dataclass
class Bitpacked:
    """DuckDB BITPACKING segment images of one column (cubit_table_add_bitpacked_column input)."""
    data: np.ndarray       # uint8 segment images, segment i at seg_off[i]
    seg_off: np.ndarray    # uint64
    seg_count: np.ndarray  # uint64 rows per segment


def bitpack_for(values: np.ndarray, block_size: int = 262144, threads: int = 0) -> Bitpacked:
    """Bench input: CONSTANT / FOR groups in 256 KiB segments, one row group per segment run
    (csrc/bitpack_gen.cpp). Test parity uses the oracle's restatement of the reference
    compressor instead."""
    v = np.ascontiguousarray(values)
    if v.dtype not in (np.int32, np.int64):
        raise TypeError(v.dtype)
    n = int(v.shape[0])
    ngroups = (n + 2047) // 2048
    cap = n * v.itemsize + ngroups * 64 + 4096
    max_segs = ngroups + (n + 122879) // 122880 + 1
    out = np.empty(cap, dtype=np.uint8)
    off = np.empty(max_segs, dtype=np.uint64)
    rows = np.empty(max_segs, dtype=np.uint64)
    used = ctypes.c_uint64(0)
    ns = L.gen_lib().cubit_bitpack_for(v.ctypes.data, v.itemsize, n, block_size, out.ctypes.data, cap,
                                       off.ctypes.data, rows.ctypes.data, max_segs, ctypes.byref(used), threads)
    if ns == 0:
        raise RuntimeError("cubit_bitpack_for failed")
    return Bitpacked(out[: used.value], off[:ns].copy(), rows[:ns].copy())


def validity_from_mask(valid: np.ndarray) -> np.ndarray:
    """bool[n] → LSB-first uint64 validity words (DuckDB ValidityMask layout)."""
    n = valid.shape[0]
    nw = (n + 63) // 64
    packed = np.packbits(np.asarray(valid, dtype=bool), bitorder="little")
    buf = np.zeros(nw * 8, dtype=np.uint8)
    buf[: packed.size] = packed
    return buf.view("<u8").astype(np.uint64)


def mask_from_words(words: np.ndarray, n: int) -> np.ndarray:
    """LSB-first uint64 words → bool[n]."""
    b = np.ascontiguousarray(words, dtype="<u8").view(np.uint8)
    return np.unpackbits(b, bitorder="little")[:n].astype(bool)
