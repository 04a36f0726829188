"""The C-ABI library loads and exports every entry point include/*.h declares (no GPU)."""
import re
from pathlib import Path

import numpy as np

from cubit_amd import _lib as L

ROOT = Path(__file__).resolve().parent.parent


def declared(header):
    text = header.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    # header-only helpers (static inline) are not library symbols
    inline = set(re.findall(r"^static\s+inline\b[\w\s\*]*?\b(cubit_\w+)\s*\(", text, flags=re.M))
    return set(re.findall(r"^[A-Za-z_][\w\s\*]*?\b(cubit_\w+)\s*\(", text, flags=re.M)) - inline


def test_every_declared_symbol_is_exported():
    headers = sorted((ROOT / "include").glob("*.h"))
    assert headers
    names = set()
    for h in headers:
        names |= declared(h)
    assert "cubit_table_scan" in names and "cubit_bitvector_eval" in names
    exported = L.exported_symbols(L.GPU_LIB) | L.exported_symbols(L.GEN_LIB) | L.exported_symbols(L.SCAN_LIB)
    missing = sorted(n for n in names if n not in exported)
    assert not missing, missing


def test_library_loads_and_reports_geometry():
    lib = L.gpu_lib()
    assert lib.cubit_abi_version() == 1
    assert lib.cubit_vector_size() == 2048 and lib.cubit_vector_size() % 64 == 0
    assert lib.cubit_row_group_size() == 122880 and lib.cubit_row_group_size() % 64 == 0
    assert lib.cubit_padded_words(1) == 16384
    assert lib.cubit_padded_words(1 << 20) == 16384
    assert lib.cubit_padded_words((1 << 20) + 1) == 32768


def test_errors_are_status_codes_not_exceptions():
    lib = L.gpu_lib()
    rc = lib.cubit_table_scan(None, None, 0, None, None, 0, None, 0)
    assert rc == L.ERR_INVALID
    assert b"null" in lib.cubit_last_error()


def test_copy_stream_calls_reject_null_arguments():
    """The table function's per-task copy streams (cubit_copy_stream_*): status codes, no GPU."""
    lib = L.gpu_lib()
    assert lib.cubit_copy_stream_create(None, None) == L.ERR_INVALID
    assert lib.cubit_copy_stream_destroy(None, None) == L.ERR_INVALID
    assert lib.cubit_memcpy_d2h_stream(None, None, None, None, 0) == L.ERR_INVALID
    assert b"null" in lib.cubit_last_error()


def test_validity_words_layout():
    from cubit_amd.datagen import mask_from_words, validity_from_mask

    rng = np.random.default_rng(3)
    m = rng.random(1000) > 0.5
    w = validity_from_mask(m)
    assert w.dtype == np.uint64 and len(w) == 16
    # LSB-first: bit i of word j is row 64*j + i
    assert bool((int(w[0]) >> 5) & 1) == bool(m[5])
    assert bool((int(w[3]) >> 7) & 1) == bool(m[3 * 64 + 7])
    assert np.array_equal(mask_from_words(w, 1000), m)
