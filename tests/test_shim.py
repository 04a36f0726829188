"""The DuckDB extension shim (duckdb-cubit_amd/shim/cubit_extension.cpp) type-checks against
the reference's own DuckDB v1.1.2 headers: every DuckDB API it uses exists with the
signature it assumes. Needs the reference source tree (this container only); skipped
elsewhere. Nothing is built or linked from the reference."""
import shutil
import subprocess
from pathlib import Path

import pytest

from conftest import ROOT

DUCKDB_INCLUDE = Path("/root/reference/src/include")


@pytest.mark.skipif(not (DUCKDB_INCLUDE / "duckdb.hpp").exists() or shutil.which("g++") is None,
                    reason="DuckDB headers not present")
def test_shim_compiles_against_duckdb_headers():
    r = subprocess.run(["make", "-s", "-C", str(ROOT / "duckdb-cubit_amd"), "shim-check",
                        f"DUCKDB_INCLUDE={DUCKDB_INCLUDE}"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "warning" not in r.stderr, r.stderr[-4000:]
