"""Register the in-tree package directory ``mpi-sppy_amd/`` under its import name ``mpisppy_amd``.

The directory name carries a hyphen (repository layout convention), which Python cannot import
directly; ``setup.py`` maps it with ``package_dir`` for installs, and this helper does the same for
in-tree use (tests, bench.py, __graft_entry__.py).
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "mpi-sppy_amd")


def load():
    mod = sys.modules.get("mpisppy_amd")
    if mod is not None:
        return mod
    spec = importlib.util.spec_from_file_location(
        "mpisppy_amd", os.path.join(PKG_DIR, "__init__.py"), submodule_search_locations=[PKG_DIR])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["mpisppy_amd"] = mod
    spec.loader.exec_module(mod)
    return mod
