"""cubit_amd — MI355X-native bitmap-indexed table-scan filter (DuckDB-CUBIT hot path).

The scan path is libcubitgpu.so (HIP, gfx950) behind include/cubit_gpu.h; this package is
its Python handle (ctypes) plus the TableFilter mirror used to describe predicates.
"""
from . import _lib
from ._lib import CubitError, Txn
from .filters import (And, Cmp, ConjunctionAndFilter, ConjunctionOrFilter, ConstantFilter, IsNotNull,
                      IsNotNullFilter, IsNull, IsNullFilter, Or, TableFilterSet, date, decimal, q6_filter_set,
                      serialize)
from .table import Context, CubitTable, DeviceBuffer, padded_words

__all__ = [
    "_lib", "CubitError", "Txn", "And", "Cmp", "ConjunctionAndFilter", "ConjunctionOrFilter", "ConstantFilter",
    "IsNotNull", "IsNotNullFilter", "IsNull", "IsNullFilter", "Or", "TableFilterSet", "date", "decimal",
    "q6_filter_set", "serialize", "Context", "CubitTable", "DeviceBuffer", "padded_words",
]
