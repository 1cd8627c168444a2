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


def _c_layout(struct, fields):
    """sizeof / offsetof of a header struct as gcc lays it out (the C ABI the library is built to)."""
    import shutil
    import subprocess
    import tempfile
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    body = "\n".join(f'printf("%zu\\n", offsetof({struct}, {f}));' for f in fields)
    src = (f'#include <stdio.h>\n#include <stddef.h>\n#include "phg.h"\nint main(void) {{\n'
           f'printf("%zu\\n", sizeof({struct}));\n{body}\nreturn 0; }}\n')
    with tempfile.TemporaryDirectory() as d:
        c, exe = os.path.join(d, "t.c"), os.path.join(d, "t")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    return [int(v) for v in out]


@pytest.mark.parametrize("struct,cls", [("phg_batch", "PhgBatch"), ("phg_opts", "PhgOpts")])
def test_struct_layout(struct, cls):
    """ctypes mirrors of the header structs have gcc's size and field offsets."""
    ct = getattr(_lib, cls)
    fields = [f[0] for f in ct._fields_]
    want = _c_layout(struct, fields)
    assert ctypes.sizeof(ct) == want[0]
    for f, off in zip(fields, want[1:]):
        assert getattr(ct, f).offset == off, f
