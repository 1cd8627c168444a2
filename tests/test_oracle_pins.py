"""Pin the CPU oracle (oracle/) against the reference's own known-answer fixtures.

Every value below is copied from the reference test suite / committed baselines:

* ``mpisppy/tests/examples/w_test_data/{w_file,xbar_file}.csv`` (copied to tests/golden/ref_*.csv),
  asserted at places=5 by ``mpisppy/tests/test_w_writer.py:83-112`` -- farmer 3 scen, rho=1, 5 iters
* Lagrangian bound -109499.5160897 (places=1) -- ``mpisppy/tests/test_with_cylinders.py:153``
* farmer EF objective -108390 -- ``doc/src/examples.rst:382``; nonants [80,250,170] --
  ``examples/test_data/farmeref_baseline/farmer.npy``
* farmer-30 trivial bound -137846 (3 s.f.) -- ``mpisppy/tests/test_aph.py:249-253``
* hydro trivial bound 180, E[obj] 190 (2 s.f.) -- ``mpisppy/tests/test_ef_ph.py:643-650``;
  hydro EF Scen7.Pgt[2] = 60 -- ``test_ef_ph.py:608-611``; EF root nonants [30,60,0,54.432] --
  ``examples/test_data/hydroef_baseline/hydro.npy``
"""
import csv
import math
import os

import numpy as np
import pytest

from oracle import models, ph

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def round_pos_sig(x, sig=1):
    return round(x, sig - int(math.floor(math.log10(abs(x)))) - 1)


@pytest.fixture(scope="module")
def farmer3_run():
    opts = dict(defaultPHrho=1.0, PHIterLimit=5, convthresh=1e-10)
    o = ph.OraclePH(opts, models.farmer_names(3), models.farmer,
                    dict(crops_multiplier=1, num_scens=3))
    lag = {}

    def cb(o):
        if o._PHIter == 5:
            lag[5] = o.lagrangian_bound(o.W)

    o.Iter0()
    o.iterk_loop(cb)
    return o, lag


def test_w_file(farmer3_run):
    o, _ = farmer3_run
    rows = list(csv.reader(open(os.path.join(GOLD, "ref_w_file.csv"))))[:9]
    names = models.farmer_names(3)
    sc = models.farmer("scen0", num_scens=3)
    nonant_names = [sc.colnames[c] for c in sc.nonant_cols()]
    for sname, vname, wval in rows:
        k = names.index(sname)
        i = nonant_names.index(vname)
        assert abs(o.W[k, i] - float(wval)) < 5e-6, (sname, vname, o.W[k, i], wval)


def test_xbar_file(farmer3_run):
    o, _ = farmer3_run
    rows = list(csv.reader(open(os.path.join(GOLD, "ref_xbar_file.csv"))))[:3]
    sc = models.farmer("scen0", num_scens=3)
    nonant_names = [sc.colnames[c] for c in sc.nonant_cols()]
    for vname, xval in rows:
        i = nonant_names.index(vname)
        assert abs(o.xbar[0, i] - float(xval)) < 5e-6


def test_lagrangian_bound(farmer3_run):
    _, lag = farmer3_run
    assert abs(lag[5] - (-109499.5160897)) < 0.05


def test_farmer_ef():
    sc = [models.farmer(n, num_scens=3) for n in models.farmer_names(3)]
    obj, xs = ph.ef_solve(sc)
    assert abs(obj - (-108390.0)) < 1e-6
    np.testing.assert_allclose(xs[0], [80.0, 250.0, 170.0], atol=1e-8)


def test_farmer30_trivial_bound():
    names = [f"Scenario{i + 1}" for i in range(30)]
    o = ph.OraclePH(dict(defaultPHrho=1.0, PHIterLimit=0, convthresh=1e-10), names, models.farmer,
                    dict(crops_multiplier=1))
    tb = o.Iter0()
    assert round_pos_sig(-tb, 3) == round_pos_sig(137846, 3)


def test_hydro_ph():
    o = ph.OraclePH(dict(defaultPHrho=1.0, PHIterLimit=10, convthresh=0.001), models.hydro_names(9),
                    models.hydro, dict(branching_factors=(3, 3)))
    conv, eobj, tb = o.ph_main()
    assert round_pos_sig(tb, 2) == 180
    assert round_pos_sig(o.Eobjective(W_on=0, prox_on=0), 2) == 190


def test_hydro_ef():
    sc = [models.hydro(n) for n in models.hydro_names(9)]
    obj, xs = ph.ef_solve(sc)
    np.testing.assert_allclose(xs[0][:4], [30.0, 60.0, 0.0, 54.432], atol=1e-6)
    assert round_pos_sig(xs[6][4], 1) == 60      # Scen7.Pgt[2]


def test_farmer_ef_fixture_generators_agree():
    """The EF fixtures of the north-star test (tests/golden/make_ef_fixtures.py): the exact
    separable solution (used at S = 10 000, where the 1.2M-column LP is out of reach of HiGHS here)
    equals the HiGHS LP extensive form on the same restated scenario LPs (S = 30), objective and
    first-stage solution; and the committed fixtures hold those values."""
    import json
    import os
    import sys
    gold = os.path.join(os.path.dirname(__file__), "golden")
    sys.path.insert(0, gold)
    import make_ef_fixtures as mk
    obj, root = mk.farmer_ef_separable(30)
    c, A, rlo, rhi, clo, chi, cols, n, _ = mk.farmer_ef(30)
    st, x, lp_obj, _, _ = mk.solve_lp(c, A, rlo, rhi, clo, chi, threads=1)
    assert st == "Optimal"
    assert abs(obj - lp_obj) <= 1e-12 * abs(lp_obj)
    np.testing.assert_allclose(root, x[cols], atol=1e-8)
    for S in (30, 1000, 10000):
        d = json.load(open(os.path.join(gold, f"farmer_cm10_ef_S{S}.json")))
        assert d["status"] == "Optimal" and d["S"] == S
        if S == 30:
            assert abs(d["objective"] - obj) <= 1e-12 * abs(obj)
        if "lp_ef_objective" in d:
            assert d["rel_diff_vs_lp_ef"] <= 1e-10
