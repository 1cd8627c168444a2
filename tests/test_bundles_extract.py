"""Extensive forms, proper / loose bundles and the standard-form extractor (CPU).

* ``utils/ef.py`` restates ``create_EF`` (``mpisppy/utils/sputils.py:143-354``): the farmer EF of
  the three textbook scenarios solved by the oracle's HiGHS gives -108390, the value the
  reference's own tests check (``mpisppy/tests/test_ef_ph.py``, farmer EF ``-108390``);
* ``utils/proper_bundler.py`` (``mpisppy/utils/proper_bundler.py:29-122``) and
  ``bundles_per_rank`` (``spbase.py:223-257``): bundle names, members, probabilities;
* ``opt/extract.py``: duck-typed model -> CSR, and back to the engine's LinearModel.  The Pyomo
  path of the extractor cannot run here (Pyomo absent): parity unpinned.
"""
import numpy as np
import pytest

from mpisppy_amd.examples import farmer
from mpisppy_amd.model import LinearModel
from mpisppy_amd.opt import extract, to_linear_model, as_scenario_model
from mpisppy_amd.spbase import SPBase
from mpisppy_amd.utils.ef import create_EF
from mpisppy_amd.utils.proper_bundler import ProperBundler, bundle_scenarios
from oracle import highs


def _solve_lm(m):
    a = m.arrays()
    r = highs.solve(m.sense * a["c"], a["rowptr"], a["colidx"], a["vals"], a["row_lo"], a["row_hi"],
                    a["col_lo"], a["col_hi"])
    assert r.status == "Optimal"
    return m.sense * (r.obj) + m.obj_offset, r.x


def test_farmer_ef_matches_reference_value():
    ef = create_EF(farmer.scenario_names_creator(3), farmer.scenario_creator, {"num_scens": 3})
    assert ef.n == 36 and ef.m == 3 * 10 + 2 * 3
    assert sorted(ef.ref_vars) == [("ROOT", 0), ("ROOT", 1), ("ROOT", 2)]
    assert ef._mpisppy_probability == pytest.approx(1.0)
    obj, x = _solve_lm(ef)
    assert obj == pytest.approx(-108390.0, rel=1e-9)
    # the reference columns are the first scenario's nonants; every copy equals them
    ref = [x[v.col] for _, v in sorted(ef.ref_vars.items())]
    np.testing.assert_allclose(ref, [80.0, 250.0, 170.0], atol=1e-6)   # CORN, SUGAR_BEETS, WHEAT (sorted keys)


def test_proper_bundler_names_and_models():
    pb = ProperBundler(farmer)
    pb.set_kwargs({"num_scens": 6})
    names = pb.bundle_names_creator(3, cfg={"num_scens": 6, "scenarios_per_bundle": 2})
    first = farmer.scenario_names_creator(1)[0]
    inum = int("".join(ch for ch in first if ch.isdigit()))
    assert names == [f"Bundle_{inum}_{inum + 1}", f"Bundle_{inum + 2}_{inum + 3}", f"Bundle_{inum + 4}_{inum + 5}"]
    b = pb.scenario_creator(names[1])
    assert [nd.name for nd in b._mpisppy_node_list] == ["ROOT"]
    assert len(b._mpisppy_node_list[0].nonant_vardata_list) == 3
    assert b._mpisppy_probability == pytest.approx(2.0 / 6.0)
    # a scenario name passes through
    s = pb.scenario_creator(farmer.scenario_names_creator(1, start=inum + 2)[0])
    assert s.n == 12
    with pytest.raises(ValueError):
        pb.bundle_names_creator(2, cfg={"num_scens": 5, "scenarios_per_bundle": 2})


def test_bundle_scenarios_split_like_reference():
    assert bundle_scenarios(list("abcdefg"), 3) == [["a", "b"], ["c", "d"], ["e", "f", "g"]]
    with pytest.raises(RuntimeError):
        bundle_scenarios(list("ab"), 3)


def test_loose_bundles_per_rank():
    opts = {"solver_name": "phg", "PHIterLimit": 1, "defaultPHrho": 1.0, "convthresh": 1e-4,
            "verbose": False, "display_progress": False, "bundles_per_rank": 3}
    sp = SPBase(opts, farmer.scenario_names_creator(6), farmer.scenario_creator,
                scenario_creator_kwargs={"num_scens": 6})
    assert sp.bundling
    assert sp.local_scenario_names == ["rank0bundle0", "rank0bundle1", "rank0bundle2"]
    assert [len(g) for g in sp.names_in_bundles[0].values()] == [2, 2, 2]
    p = [s._mpisppy_probability for s in sp.local_scenarios.values()]
    assert sum(p) == pytest.approx(1.0)
    # EF of all three bundles == EF of the six scenarios (objective of the bundle EFs' EF)
    lm = list(sp.local_scenarios.values())
    tot = sum(pi * _solve_lm(b)[0] for pi, b in zip(p, lm))
    ef_obj = _solve_lm(create_EF(farmer.scenario_names_creator(6), farmer.scenario_creator, {"num_scens": 6}))[0]
    assert tot <= ef_obj + 1e-6 * abs(ef_obj)     # wait-and-see over bundles bounds the EF (min)


class _V:
    def __init__(self, name, lb=None, ub=None, fixed=False, value=None):
        self.name, self.lb, self.ub, self.fixed, self.value = name, lb, ub, fixed, value


class _R:
    def __init__(self, name, terms, lower=None, upper=None, constant=0.0):
        self.name, self.terms, self.lower, self.upper, self.constant = name, terms, lower, upper, constant


class _O:
    def __init__(self, terms, constant=0.0, sense=1):
        self.terms, self.constant, self.sense = terms, constant, sense


class _Duck:
    """min  x + 2 y - z + 3   s.t.  1 <= x + y <= 4,  y - z + 1 >= 0 (constant moved),  z fixed at 0.5"""

    def __init__(self):
        self.name = "duck"
        self.x, self.y, self.z = _V("x", 0, 3), _V("y", None, 2), _V("z", fixed=True, value=0.5)

    def variables(self):
        return [self.x, self.y, self.z]

    def constraints(self):
        return [_R("c1", [(self.x, 1.0), (self.y, 1.0)], 1.0, 4.0),
                _R("c2", [(self.z, -1.0), (self.y, 1.0)], 0.0, None, constant=1.0)]

    def objective(self):
        return _O([(self.x, 1.0), (self.y, 2.0), (self.z, -1.0)], constant=3.0)


def test_duck_model_extraction():
    sf = extract(_Duck())
    np.testing.assert_array_equal(sf.rowptr, [0, 2, 4])
    np.testing.assert_array_equal(sf.colidx, [0, 1, 1, 2])
    np.testing.assert_allclose(sf.vals, [1.0, 1.0, 1.0, -1.0])
    np.testing.assert_allclose(sf.row_lo, [1.0, -1.0])
    np.testing.assert_allclose(sf.row_hi, [4.0, np.inf])
    np.testing.assert_allclose(sf.col_lo, [0.0, -np.inf, 0.5])
    np.testing.assert_allclose(sf.col_hi, [3.0, 2.0, 0.5])
    np.testing.assert_allclose(sf.c, [1.0, 2.0, -1.0])
    assert sf.c0 == 3.0 and sf.sense == 1
    lm = to_linear_model(sf)
    obj, x = _solve_lm(lm)
    # optimum: z = 0.5, y >= z - 1 = -0.5, x + y >= 1: y = -0.5, x = 1.5 -> 1.5 - 1 - 0.5 + 3 = 3.0
    assert obj == pytest.approx(3.0, abs=1e-9)
    np.testing.assert_allclose(x, [1.5, -0.5, 0.5], atol=1e-9)


def test_linear_model_extraction_round_trip():
    m = farmer.scenario_creator(farmer.scenario_names_creator(1)[0], num_scens=3)
    sf = extract(m)
    lm = to_linear_model(sf)
    for k in ("c", "rowptr", "colidx", "vals", "row_lo", "row_hi", "col_lo", "col_hi"):
        np.testing.assert_array_equal(lm.arrays()[k], m.arrays()[k])
    assert as_scenario_model(m) is m
    assert isinstance(lm, LinearModel)
