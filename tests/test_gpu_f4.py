"""GPU: the ``phg`` solver plugin (``opt/phg.py``: ``SolverFactory("phg")``, ``spopt.py:876-913``)
and PH over bundles (``bundles_per_rank``, ``spbase.py:223-257``; proper bundles,
``utils/proper_bundler.py:29-122``), against the CPU oracle (HiGHS).  The Pyomo side of the
plugin cannot run here (Pyomo absent): parity unpinned for it; these tests drive the same plugin
with the engine's LinearModel and a duck-typed model."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from mpisppy_amd.examples import farmer  # noqa: E402
from mpisppy_amd.opt import SolverFactory  # noqa: E402
from mpisppy_amd.ph import PH  # noqa: E402
from mpisppy_amd.utils.ef import create_EF  # noqa: E402
from mpisppy_amd.utils.proper_bundler import ProperBundler  # noqa: E402
from oracle import highs  # noqa: E402
from test_bundles_extract import _Duck  # noqa: E402


def _oracle_obj(m):
    a = m.arrays()
    r = highs.solve(m.sense * a["c"], a["rowptr"], a["colidx"], a["vals"], a["row_lo"], a["row_hi"],
                    a["col_lo"], a["col_hi"])
    return m.sense * r.obj + m.obj_offset


def test_plugin_solves_duck_model_and_loads_values():
    opt = SolverFactory("phg")
    assert opt.available()
    d = _Duck()
    res = opt.solve(d, load_solutions=True)
    assert res.solver.termination_condition == "optimal" and len(res.solution) == 1
    assert res.Problem[0].Upper_bound == pytest.approx(3.0, abs=1e-7)
    assert res.Problem[0].Lower_bound == pytest.approx(3.0, abs=1e-7)
    np.testing.assert_allclose([d.x.value, d.y.value], [1.5, -0.5], atol=1e-6)
    opt.close()


def test_plugin_solve_batch_matches_oracle():
    names = farmer.scenario_names_creator(3)
    models = [farmer.scenario_creator(nm, num_scens=3) for nm in names]
    opt = SolverFactory("phg")
    opt.options["pdhg_eps"] = 1e-9
    res = opt.solve_batch(models)
    for m, r in zip(models, res):
        o = _oracle_obj(m)
        assert r.solver.status == "ok"
        # farmer is a max-profit model written as min cost: Upper = primal objective in min sense
        assert r.Problem[0].Upper_bound == pytest.approx(o, rel=1e-7)
        assert m.objective_value() == pytest.approx(o, rel=1e-7)
    opt.close()


def _ph(names, creator, kw, **extra):
    o = {"solver_name": "phg", "PHIterLimit": 400, "defaultPHrho": 1.0, "convthresh": 1e-7,
         "verbose": False, "display_progress": False}
    o.update(extra)
    ph = PH(o, names, creator, scenario_creator_kwargs=kw)
    conv, eobj, tbound = ph.ph_main()
    return ph, conv, eobj


def test_ph_loose_bundles_reaches_ef():
    ef = _oracle_obj(create_EF(farmer.scenario_names_creator(6), farmer.scenario_creator, {"num_scens": 6}))
    ph, conv, eobj = _ph(farmer.scenario_names_creator(6), farmer.scenario_creator, {"num_scens": 6},
                         bundles_per_rank=3)
    assert ph.local_scenario_names == ["rank0bundle0", "rank0bundle1", "rank0bundle2"]
    assert conv < 1e-6
    assert abs(eobj - ef) <= 1e-5 * abs(ef), (eobj, ef)


def test_ph_proper_bundles_reaches_ef():
    ef = _oracle_obj(create_EF(farmer.scenario_names_creator(6), farmer.scenario_creator, {"num_scens": 6}))
    pb = ProperBundler(farmer)
    pb.set_kwargs({"num_scens": 6})
    names = pb.bundle_names_creator(3, cfg={"num_scens": 6, "scenarios_per_bundle": 2})
    ph, conv, eobj = _ph(names, pb.scenario_creator, {})
    assert conv < 1e-6
    assert abs(eobj - ef) <= 1e-5 * abs(ef), (eobj, ef)
