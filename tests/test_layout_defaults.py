"""CPU: the per-layout PDHG defaults PHBase resolves when the options leave them unset
(``pdhg_check_every`` None, ``pdhg_keep_omega`` None, ``pdhg_beta_artificial`` 0) -- the values
DESIGN.md (d) measured per kernel layout (round 5; the block kernel's revised by round 6's held-out A/B) -- and that explicit options win over them."""
import pytest

from mpisppy_amd import phbase
from mpisppy_amd.phbase import beta_artificial_default, check_every_default, keep_omega_default


@pytest.mark.parametrize("layout, threads, want", [
    ("local", 32, 32), ("gather", 64, 64), ("mfma", 4, 64), ("block", 256, 64), ("block", 1024, 64),
    ("block", 512, 64), ("border", 512, 32), ("stream", 1024, 32), ("wave", 64, 32)])
def test_check_every_by_layout(layout, threads, want):
    assert check_every_default(layout, threads) == want


@pytest.mark.parametrize("layout, threads, want", [
    ("local", 32, 0.0), ("gather", 64, 0.0), ("block", 256, 0.0), ("block", 1024, 0.0), ("wave", 64, 0.15),
    ("border", 512, 0.36), ("stream", 1024, 0.36), ("mfma", 4, 0.0)])
def test_beta_artificial_by_layout(layout, threads, want):
    assert beta_artificial_default(layout, threads) == want


@pytest.mark.parametrize("layout, want", [("mfma", False), ("local", "blend"), ("block", "blend"), ("border", "blend")])
def test_keep_omega_by_layout(layout, want):
    assert keep_omega_default(layout) == want


class _Eng:
    def __init__(self, layout, lanes):
        self.layout, self.lanes_per_scenario = layout, lanes


def _resolved(options, layout, lanes, current=None):
    ph = phbase.PHBase.__new__(phbase.PHBase)
    ph.options = dict(options)
    ph.current_solver_options = current or {}
    ph.engine = _Eng(layout, lanes)
    return ph._solver_opts()


def test_solver_opts_resolve_by_layout_and_options_win():
    o = _resolved({}, "block", 256)   # (round 5's 96 / 0.15 lost the held-out A/B: phbase.check_every_default)
    assert o["pdhg_check_every"] == 64 and o["pdhg_beta_artificial"] == 0.0 and o["pdhg_keep_omega"] == "blend"
    o = _resolved({}, "wave", 64)
    assert o["pdhg_check_every"] == 32 and o["pdhg_beta_artificial"] == 0.15
    o = _resolved({}, "mfma", 4)
    assert o["pdhg_check_every"] == 64 and o["pdhg_keep_omega"] is False and o["pdhg_beta_artificial"] == 0.0
    o = _resolved({"pdhg_check_every": 32, "pdhg_beta_artificial": 0.25, "pdhg_keep_omega": True}, "block", 256)
    assert o["pdhg_check_every"] == 32 and o["pdhg_beta_artificial"] == 0.25 and o["pdhg_keep_omega"] is True
    # per-iteration solver options override the PH options
    o = _resolved({"pdhg_check_every": 32}, "local", 32, current={"pdhg_check_every": 64, "pdhg_eps": 1e-7})
    assert o["pdhg_check_every"] == 64 and o["pdhg_eps"] == 1e-7
