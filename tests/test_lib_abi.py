"""libphg.so loads and exports every symbol include/phg.h declares (no GPU calls)."""
import ctypes
import os
import re

import pytest

from mpisppy_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "phg.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(phg_[a-z_0-9]+)\s*\(", txt)))


def test_header_symbols_all_bound():
    syms = header_symbols()
    assert len(syms) >= 15
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)


@pytest.mark.skipif(not os.path.exists(_lib.LIB_PATH), reason="libphg.so not built")
def test_library_exports():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for s in header_symbols():
        assert hasattr(lib, s), s
    _lib.load()


def test_struct_layout():
    # phg_batch field order/size must match include/phg.h (64-bit ABI)
    assert ctypes.sizeof(_lib.PhgOpts) == 24
    names = [f[0] for f in _lib.PhgBatch._fields_]
    assert names[:4] == ["S", "n", "m", "nnz"] and names[-3:] == ["scen_global0", "S_global", "virt_nproc"]
