"""W / xbar files and solution writers through the real engine.

Mirrors ``mpisppy/tests/test_w_writer.py:83-112`` on farmer 3 scenarios (default rho 1):
* WXBarWriter after 5 PH iterations writes W rows[1] = 70.84705093609978 and rows[3] =
  -41.104251445950844, xbar rows[1] = 274.2239371483933 (places=5, the reference's tolerance);
* WXBarReader with the reference's w_file / xbar_file and 1 PH iteration leaves exactly those values
  in the device W / xbar;
* the wheel writes the xhat incumbent's first-stage / tree solution, whose expected cost is the
  inner bound (checked with the oracle's xhat evaluation).
"""
import csv
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from mpisppy_amd.cylinders import LagrangianOuterBound, XhatShuffleInnerBound  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402
from mpisppy_amd.hub import PHHub, WheelSpinner  # noqa: E402
from mpisppy_amd.ph import PH  # noqa: E402
from mpisppy_amd.utils.wxbarreader import WXBarReader  # noqa: E402
from mpisppy_amd.utils.wxbarwriter import WXBarWriter  # noqa: E402
from oracle import models as om  # noqa: E402
from oracle import ph as oph  # noqa: E402

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _opts(**kw):
    o = {"solver_name": "phg", "PHIterLimit": 5, "defaultPHrho": 1.0, "convthresh": 1e-10,
         "verbose": False, "display_progress": False}
    o.update(kw)
    return o


def _wheel(ext, opts, spokes=(), hub_opts=None):
    S = 3
    hub_dict = {"hub_class": PHHub, "hub_kwargs": {"options": hub_opts or {}}, "opt_class": PH,
                "opt_kwargs": {"options": opts, "all_scenario_names": farmer.scenario_names_creator(S),
                               "scenario_creator": farmer.scenario_creator, "extensions": ext,
                               "scenario_creator_kwargs": {"crops_multiplier": 1, "num_scens": S}}}
    return WheelSpinner(hub_dict, list(spokes)).spin()


def test_wxbar_writer(tmp_path):
    wf, xf = str(tmp_path / "w.csv"), str(tmp_path / "x.csv")
    _wheel(WXBarWriter, _opts(W_fname=wf, Xbar_fname=xf))
    rows = list(csv.reader(open(wf)))
    assert len(rows) == 9
    assert abs(float(rows[1][2]) - 70.84705093609978) < 5e-6
    assert abs(float(rows[3][2]) - -41.104251445950844) < 5e-6
    xr = list(csv.reader(open(xf)))
    assert [r[0] for r in xr] == ["DevotedAcreage[CORN0]", "DevotedAcreage[SUGAR_BEETS0]", "DevotedAcreage[WHEAT0]"]
    assert abs(float(xr[1][1]) - 274.2239371483933) < 5e-6
    assert abs(float(xr[0][1]) - 96.88717449844287) < 5e-6


def test_wxbar_reader():
    wheel = _wheel(WXBarReader, _opts(PHIterLimit=1, init_W_fname=os.path.join(GOLD, "ref_w_file.csv"),
                                      init_Xbar_fname=os.path.join(GOLD, "ref_xbar_file.csv")))
    ph = wheel.spcomm.opt
    W, xb = ph.Ws(), ph.xbars()
    assert W[0, 1] == 70.84705093609978
    assert W[1, 0] == -41.104251445950844
    assert xb[1] == 274.2239371483933 and xb[0] == 96.88717449844287


def test_wheel_writes_incumbent(tmp_path):
    spokes = [{"spoke_class": LagrangianOuterBound}, {"spoke_class": XhatShuffleInnerBound}]
    wheel = _wheel(None, _opts(PHIterLimit=200), spokes, {"rel_gap": 0.01})
    fs = str(tmp_path / "sol" / "first_stage.csv")
    assert wheel.write_first_stage_solution(fs)
    xhat = np.array([float(r[1]) for r in csv.reader(open(fs))])
    o = oph.OraclePH(_opts(), om.farmer_names(3), om.farmer, dict(crops_multiplier=1, num_scens=3))
    ib = o.xhat_eval(xhat)
    assert abs(ib - wheel.BestInnerBound) <= 1e-6 * abs(ib), (ib, wheel.BestInnerBound)
    assert wheel.write_tree_solution(str(tmp_path / "tree"))
    assert sorted(os.listdir(tmp_path / "tree")) == ["scen0.csv", "scen1.csv", "scen2.csv"]
    cache = wheel.local_nonant_cache()
    assert list(cache) == ["ROOT"] and len(cache["ROOT"]) == 3
