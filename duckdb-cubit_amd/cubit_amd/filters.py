"""Predicate IR mirroring DuckDB's TableFilter classes.

Reference (DuckDB v1.1.2):
  TableFilterType / TableFilter / TableFilterSet   src/include/duckdb/planner/table_filter.hpp:20-101
  TableFilterSet::PushFilter (AND-combine per column) src/planner/table_filter.cpp:8-25
  ConstantFilter                                     src/include/duckdb/planner/filter/constant_filter.hpp
  ConjunctionAndFilter / ConjunctionOrFilter          src/include/duckdb/planner/filter/conjunction_filter.hpp
  IsNullFilter / IsNotNullFilter                     src/include/duckdb/planner/filter/null_filter.hpp

A TableFilterSet holds one filter per scanned column, ANDed across columns. Cross-column
OR predicates are not pushed into the scan in this snapshot (filter_combiner.cpp:624); they
run as a residual PhysicalFilter above it (physical_filter.cpp:42-53). `Residual` trees
model that part. Both serialise to the same prefix-order node array, consumed by the HIP
library (cubit_filter_node) and by the CPU oracle (ofilter).
"""
from __future__ import annotations

import ctypes as C
import datetime as _dt
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

from . import _lib as L

_CMP = {"=": L.CMP_EQ, "==": L.CMP_EQ, "!=": L.CMP_NE, "<>": L.CMP_NE, "<": L.CMP_LT, "<=": L.CMP_LE,
        ">": L.CMP_GT, ">=": L.CMP_GE}

EPOCH = _dt.date(1970, 1, 1)


def date(y: int, m: int, d: int) -> int:
    """DATE physical value: int32 days since 1970-01-01."""
    return (_dt.date(y, m, d) - EPOCH).days


class _CString(C.Structure):
    """cubit_string / the oracle's ostring: {const char *data; uint64_t size}."""

    _fields_ = [("data", C.c_void_p), ("size", C.c_uint64)]


_STRINGS = {}  # bytes -> (buffer, _CString): kept for the life of the process
_STRING_AT = {}  # address of a _CString -> bytes


def string_ref(b) -> int:
    """The address of a persistent {data, size} struct holding `b` (str is UTF-8 encoded): how a
    VARCHAR constant, index key or (oracle) update value crosses the ABI."""
    if isinstance(b, str):
        b = b.encode()
    b = bytes(b)
    if b not in _STRINGS:
        buf = C.create_string_buffer(b, max(len(b), 1))
        cs = _CString(C.cast(buf, C.c_void_p).value, len(b))
        _STRINGS[b] = (buf, cs)
        _STRING_AT[C.addressof(cs)] = b
    return C.addressof(_STRINGS[b][1])


def string_at(addr: int) -> bytes:
    """The bytes of a struct made by string_ref."""
    return _STRING_AT[int(addr)]


def key128(v: int, signed: bool = True) -> bytes:
    """A HUGEINT (signed) / UHUGEINT value's 16-byte order key, as cubit_key128 writes it: the
    128 bits big-endian, HUGEINT's sign bit flipped — unsigned byte order = the values' order. A
    HUGEINT / UHUGEINT column's constants and index keys are these keys (as str / bytes constants)."""
    v = int(v)
    if signed:
        assert -(1 << 127) <= v < (1 << 127), v
        v += 1 << 127
    else:
        assert 0 <= v < (1 << 128), v
    return v.to_bytes(16, "big")


def value128(key: bytes, signed: bool = True) -> int:
    """cubit_value128: the value of a 16-byte order key."""
    v = int.from_bytes(bytes(key), "big")
    return v - (1 << 127) if signed else v


def constant_bits(c) -> int:
    """A filter constant as the int64 a cubit_filter_node carries: integers as they are; a
    np.float32 as its 32-bit IEEE pattern (a FLOAT column's constant), any other float as its
    64-bit pattern (DOUBLE) — the C ABI compares FLOAT / DOUBLE columns with DuckDB's semantics
    on those patterns; str / bytes as the address of a cubit_string (a VARCHAR column's constant)."""
    import numpy as np

    if isinstance(c, (str, bytes)):
        return string_ref(c)
    if isinstance(c, np.float32):
        return int(np.array([c], dtype=np.float32).view(np.uint32)[0])
    if isinstance(c, (float, np.floating)):
        return int(np.array([c], dtype=np.float64).view(np.int64)[0])
    c = int(c)
    return c - (1 << 64) if c >= 1 << 63 else c  # a UBIGINT constant past 2^63: its bits as an int64


def decimal(text: str, scale: int = 2) -> int:
    """DECIMAL(p, scale) physical value (scaled integer), e.g. decimal('0.05') == 5."""
    neg = text.startswith("-")
    t = text.lstrip("+-")
    whole, _, frac = t.partition(".")
    frac = (frac + "0" * scale)[:scale]
    v = int(whole or "0") * 10 ** scale + int(frac or "0")
    return -v if neg else v


class TableFilter:
    kind: int

    def nodes(self, column: int) -> List[Tuple[int, int, int, int, int]]:
        raise NotImplementedError


@dataclass
class ConstantFilter(TableFilter):
    comparison: str
    constant: int
    kind = L.FILTER_CONSTANT

    def nodes(self, column):
        return [(L.FILTER_CONSTANT, _CMP[self.comparison], column, 0, constant_bits(self.constant))]


@dataclass
class IsNullFilter(TableFilter):
    kind = L.FILTER_IS_NULL

    def nodes(self, column):
        return [(L.FILTER_IS_NULL, 0, column, 0, 0)]


@dataclass
class IsNotNullFilter(TableFilter):
    kind = L.FILTER_IS_NOT_NULL

    def nodes(self, column):
        return [(L.FILTER_IS_NOT_NULL, 0, column, 0, 0)]


@dataclass
class ConjunctionAndFilter(TableFilter):
    child_filters: List[TableFilter] = field(default_factory=list)
    kind = L.FILTER_AND

    def nodes(self, column):
        out = [(L.FILTER_AND, 0, column, len(self.child_filters), 0)]
        for c in self.child_filters:
            out += c.nodes(column)
        return out


@dataclass
class ConjunctionOrFilter(TableFilter):
    child_filters: List[TableFilter] = field(default_factory=list)
    kind = L.FILTER_OR

    def nodes(self, column):
        out = [(L.FILTER_OR, 0, column, len(self.child_filters), 0)]
        for c in self.child_filters:
            out += c.nodes(column)
        return out


class TableFilterSet:
    """Per-column filters, ANDed across columns (table_filter.hpp:67-101)."""

    def __init__(self, filters: Optional[Dict[int, TableFilter]] = None):
        self.filters: Dict[int, TableFilter] = {}
        for col, f in (filters or {}).items():
            self.push_filter(col, f)

    def push_filter(self, column: int, f: TableFilter) -> None:
        """TableFilterSet::PushFilter: a second filter on a column is AND-combined."""
        cur = self.filters.get(column)
        if cur is None:
            self.filters[column] = f
        elif isinstance(cur, ConjunctionAndFilter):
            cur.child_filters.append(f)
        else:
            self.filters[column] = ConjunctionAndFilter([cur, f])


# --------------------------------------------------------------------- residual (cross-column) trees

class Residual:
    def nodes(self) -> List[Tuple[int, int, int, int, int]]:
        raise NotImplementedError


@dataclass
class Cmp(Residual):
    column: int
    comparison: str
    constant: int

    def nodes(self):
        return [(L.FILTER_CONSTANT, _CMP[self.comparison], self.column, 0, constant_bits(self.constant))]


@dataclass
class IsNull(Residual):
    column: int

    def nodes(self):
        return [(L.FILTER_IS_NULL, 0, self.column, 0, 0)]


@dataclass
class IsNotNull(Residual):
    column: int

    def nodes(self):
        return [(L.FILTER_IS_NOT_NULL, 0, self.column, 0, 0)]


class And(Residual):
    def __init__(self, *children: Residual):
        self.children = list(children)

    def nodes(self):
        out = [(L.FILTER_AND, 0, -1, len(self.children), 0)]
        for c in self.children:
            out += c.nodes()
        return out


class Or(Residual):
    def __init__(self, *children: Residual):
        self.children = list(children)

    def nodes(self):
        out = [(L.FILTER_OR, 0, -1, len(self.children), 0)]
        for c in self.children:
            out += c.nodes()
        return out


# --------------------------------------------------------------------- serialisation

@dataclass
class Plan:
    """Prefix node array + where each part starts.

    nodes[0] is an AND root over (one subtree per pushed column, then the residual tree).
    `pushed` lists (column, root index) in evaluation order; `residual_root` is -1 when
    there is no residual part.
    """

    nodes: List[Tuple[int, int, int, int, int]]
    pushed: List[Tuple[int, int]]
    residual_root: int


def serialize(filter_set: Optional[TableFilterSet] = None, residual: Optional[Residual] = None,
              order: Optional[Sequence[int]] = None) -> Plan:
    filter_set = filter_set or TableFilterSet()
    cols = list(order) if order is not None else list(filter_set.filters.keys())
    n_children = len(cols) + (1 if residual is not None else 0)
    nodes = [(L.FILTER_AND, 0, -1, n_children, 0)]
    pushed = []
    for col in cols:
        pushed.append((col, len(nodes)))
        nodes += filter_set.filters[col].nodes(col)
    rroot = -1
    if residual is not None:
        rroot = len(nodes)
        nodes += residual.nodes()
    return Plan(nodes, pushed, rroot)


def to_ctypes(nodes) -> "C.Array":
    import ctypes as C

    arr = (L.FilterNode * max(len(nodes), 1))()
    for i, (k, cmp, col, nc, const) in enumerate(nodes):
        arr[i].kind, arr[i].cmp, arr[i].column, arr[i].n_children, arr[i].constant = k, cmp, col, nc, const
    return arr


def q6_filter_set(col_shipdate: int = 0, col_discount: int = 1, col_quantity: int = 2) -> TableFilterSet:
    """The TableFilterSet DuckDB pushes into SEQ_SCAN lineitem for TPC-H Q6:
    l_shipdate>='1994-01-01' AND <'1995-01-01' AND IS NOT NULL; l_discount>=0.05 AND <=0.07
    AND IS NOT NULL; l_quantity<24.00 AND IS NOT NULL (filter_combiner.cpp:473-480 adds the
    IS NOT NULL)."""
    fs = TableFilterSet()
    fs.push_filter(col_shipdate, ConstantFilter(">=", date(1994, 1, 1)))
    fs.push_filter(col_shipdate, ConstantFilter("<", date(1995, 1, 1)))
    fs.push_filter(col_shipdate, IsNotNullFilter())
    fs.push_filter(col_discount, ConstantFilter(">=", decimal("0.05")))
    fs.push_filter(col_discount, ConstantFilter("<=", decimal("0.07")))
    fs.push_filter(col_discount, IsNotNullFilter())
    fs.push_filter(col_quantity, ConstantFilter("<", decimal("24.00")))
    fs.push_filter(col_quantity, IsNotNullFilter())
    return fs
