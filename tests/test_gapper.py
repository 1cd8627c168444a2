"""Solver-tolerance schedules on the host (no GPU): the Gapper extension (mipgapper.py:15-60 restated:
the option set at pre_iter0 from key 0 and at miditer from the iteration's key, into the CURRENT solver
options dict) and PHBase's conv-keyed pdhg_eps schedule (first matching pair, never loosening), and
which extensions keep the pipelined loop."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _pkg  # noqa: E402

_pkg.load()
from mpisppy_amd.extensions.extension import Extension, MultiExtension  # noqa: E402
from mpisppy_amd.extensions.gapper import Gapper  # noqa: E402
from mpisppy_amd.phbase import PHBase  # noqa: E402


class _PH:
    cylinder_rank = 0

    def __init__(self, gapperoptions, **opts):
        self.options = {"verbose": False, "gapperoptions": gapperoptions, **opts}
        self.iter0_solver_options = {"pdhg_eps": 1e-9}
        self.iterk_solver_options = {"pdhg_eps": 1e-9}
        self.current_solver_options = self.iter0_solver_options
        self._PHIter = 0
        self.conv = None


def test_gapper_follows_the_reference_hooks():
    ph = _PH({"mipgapdict": {0: 1e-4, 3: 1e-6, 7: 1e-8}, "solver_option": "pdhg_eps"})
    g = Gapper(ph)
    g.pre_iter0()
    assert ph.iter0_solver_options["pdhg_eps"] == 1e-4          # key 0 -> the iter0 options
    ph.current_solver_options = ph.iterk_solver_options         # end of Iter0 (phbase.py:944)
    seen = []
    for ph._PHIter in range(1, 10):
        g.miditer()
        seen.append(ph.current_solver_options["pdhg_eps"])
    assert seen == [1e-9, 1e-9, 1e-6, 1e-6, 1e-6, 1e-6, 1e-8, 1e-8, 1e-8]
    assert ph.iterk_solver_options is ph.current_solver_options  # mutated in place, as the reference
    assert g.history == [(0, 1e-4), (3, 1e-6), (7, 1e-8)]


def test_gapper_default_option_is_the_references_mipgap():
    ph = _PH({"mipgapdict": {0: 0.01}})
    Gapper(ph).pre_iter0()
    assert ph.current_solver_options["mipgap"] == 0.01 and ph.current_solver_options["pdhg_eps"] == 1e-9


def test_eps_schedule_by_conv_never_loosens():
    ph = _PH(None, pdhg_eps_schedule=[(1e-2, 1e-5), (1e-3, 1e-6), (0.0, 1e-7)])
    ph.current_solver_options = ph.iterk_solver_options
    got = []
    for c in (None, 5e-2, 5e-3, 2e-2, 5e-4, 1e-2, 1e-5):
        ph.conv = c
        PHBase._apply_eps_schedule(ph)
        got.append(ph.current_solver_options["pdhg_eps"])
    assert got == [1e-5, 1e-5, 1e-6, 1e-6, 1e-7, 1e-7, 1e-7]


def test_pipeline_safety():
    ph = _PH({"mipgapdict": {0: 1e-4}, "solver_option": "pdhg_eps"})
    assert Gapper.pipeline_safe and not getattr(Extension(ph), "pipeline_safe", False)
    assert MultiExtension(ph, [Gapper]).pipeline_safe
    assert not MultiExtension(ph, [Gapper, Extension]).pipeline_safe
    fake = type("F", (), {})()
    fake.options = {"pdhg_pipeline": True}
    fake.ph_converger = None
    for ext, ok in ((None, True), (Gapper(ph), True), (Extension(ph), False)):
        fake.extobject = ext
        assert PHBase._can_pipeline(fake) is ok
