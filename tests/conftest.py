import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
PKG = ROOT / "duckdb-cubit_amd"
for p in (str(PKG), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)


def _ensure_built():
    need = [PKG / "lib" / "libcubit_datagen.so", PKG / "lib" / "libcubitgpu.so", ROOT / "oracle" / "lib" / "libcubit_oracle.so"]
    if not all(p.exists() for p in need):
        subprocess.run(["make", "-s", "-C", str(PKG), "-j8"], check=True)
    # the oracle (one gcc line, test infrastructure) is kept current with its sources every session
    subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)


_ensure_built()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def golden():
    g = ROOT / "tests" / "golden"
    return {"tpch": json.loads((g / "tpch.json").read_text()),
            "cases": json.loads((g / "reference_cases.json").read_text())}


_LINEITEM = {}


def lineitem(sf):
    from cubit_amd import datagen

    if sf not in _LINEITEM:
        _LINEITEM[sf] = datagen.tpch_lineitem(sf)
    return _LINEITEM[sf]


@pytest.fixture(scope="session")
def li001():
    return lineitem(0.01)


@pytest.fixture(scope="session")
def li01():
    return lineitem(0.1)


@pytest.fixture(scope="session")
def li1():
    return lineitem(1)


def revenue_from_answer(text):
    """'1193053.2253' → scaled integer (DECIMAL(38,4) storage)."""
    whole, frac = text.split(".")
    return int(whole) * 10 ** 4 + int(frac.ljust(4, "0")[:4])
