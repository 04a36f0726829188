"""The order key behind FLOAT / DOUBLE columns (cubit_fp_key / cubit_fp_value, include/cubit_gpu.h;
the device copy in csrc/cubit_internal.hpp): comparing keys as integers must give exactly DuckDB's
floating-point operators (src/common/vector_operations/comparison_operators.cpp:17-88 — NaN equals
NaN and is greater than everything, -0.0 == +0.0), as the oracle restates them. No GPU: the header
helpers are compiled into a small shared object here."""
import ctypes as C
import subprocess

import numpy as np
import pytest

from oracle import oracle as O
from test_abi import ROOT

SRC = r"""
#include "cubit_gpu.h"
int64_t fp_key(int type, int64_t bits) { return cubit_fp_key(type, bits); }
int64_t fp_value(int type, int64_t key) { return cubit_fp_value(type, key); }
"""

TYPE = {np.float32: 8, np.float64: 9}


@pytest.fixture(scope="module")
def keylib(tmp_path_factory):
    d = tmp_path_factory.mktemp("fpkey")
    (d / "k.c").write_text(SRC)
    so = d / "k.so"
    subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-Werror", "-shared", "-fPIC", "-I", str(ROOT / "include"),
                    str(d / "k.c"), "-o", str(so)], check=True)
    lib = C.CDLL(str(so))
    for f in (lib.fp_key, lib.fp_value):
        f.restype = C.c_int64
        f.argtypes = [C.c_int, C.c_int64]
    return lib


def values(dt, rng):
    b = np.uint32 if dt == np.float32 else np.uint64
    fi = np.finfo(dt)
    nans = [0x7FC00000, 0x7FC00001, 0xFFC00000, 0x7F800001, 0xFFFFFFFF] if dt == np.float32 else \
        [0x7FF8000000000000, 0x7FF8000000000001, 0xFFF8000000000000, 0x7FF0000000000001, 0xFFFFFFFFFFFFFFFF]
    v = [0.0, -0.0, np.inf, -np.inf, fi.max, -fi.max, fi.tiny, -fi.tiny, fi.tiny / 8, -fi.tiny / 8, 1.0, -1.0,
         np.nextafter(dt(1.0), dt(2.0)), np.nextafter(dt(-1.0), dt(-2.0))]
    v = list(np.array(v, dtype=dt)) + list(np.array(nans, dtype=b).view(dt))
    v += list((rng.standard_normal(200) * 10.0 ** rng.integers(-30, 30, 200)).astype(dt))
    return np.array(v, dtype=dt)


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_key_order_is_duckdb_comparison(keylib, dt):
    rng = np.random.default_rng(1)
    vals = values(dt, rng)
    bits = O.fp_bits(vals, dt)
    keys = np.array([keylib.fp_key(TYPE[dt], int(b)) for b in bits], dtype=np.int64)
    col = O.Column(vals)
    n = len(vals)
    idx = np.arange(n)
    for j, c in enumerate(bits):
        for cmp, op in enumerate([np.equal, np.not_equal, np.less, np.less_equal, np.greater, np.greater_equal]):
            words = O.build_bitvector(col, n, cmp, int(c))
            want = ((words[idx >> 6] >> (idx & 63).astype(np.uint64)) & np.uint64(1)).astype(bool)
            assert np.array_equal(op(keys, keys[j]), want), (cmp, vals[j])


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_value_inverts_key(keylib, dt):
    rng = np.random.default_rng(2)
    vals = values(dt, rng)
    for v, b in zip(vals, O.fp_bits(vals, dt)):
        k = keylib.fp_key(TYPE[dt], int(b))
        back = keylib.fp_value(TYPE[dt], k)
        if np.isnan(v):
            assert np.isnan(np.array([back], dtype=np.int64).astype(np.uint32 if dt == np.float32 else np.uint64)
                            .view(dt)[0])
        elif v == 0:
            assert back == 0  # both zeros → +0.0
        else:
            assert back == int(b)
    # integer types pass through
    assert keylib.fp_key(1, -5) == -5 and keylib.fp_value(0, 7) == 7
