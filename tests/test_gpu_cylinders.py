"""GPU bound spokes (cylinders.py) against the CPU oracle and the reference's pinned answers.

* Lagrangian outer bound with the hub's W (lagrangian_bounder.py): the reference pins
  -109499.5160897 (test_with_cylinders.py:153, places=1) for farmer 3 scenarios after 5 PH
  iterations; the oracle's lagrangian_bound(W) with the same W agrees to 1e-6 relative.
* Xhat inner bound (xhatshufflelooper_bounder.py, xhat_eval.py): a candidate scenario's nonants
  fixed in every scenario; compared with the oracle's xhat_eval of the same candidate.
* Wheel: hub + both spokes on one GPU terminate on rel_gap with outer <= EF optimum <= inner.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from mpisppy_amd import _lib  # noqa: E402
from mpisppy_amd.cylinders import LagrangianOuterBound, XhatShuffleInnerBound  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402
from mpisppy_amd.hub import PHHub, WheelSpinner  # noqa: E402
from mpisppy_amd.ph import PH  # noqa: E402
from oracle import models as om  # noqa: E402
from oracle import ph as oph  # noqa: E402


def _opts(**kw):
    o = {"solver_name": "phg", "PHIterLimit": 5, "defaultPHrho": 1.0, "convthresh": 1e-10,
         "verbose": False, "display_progress": False}
    o.update(kw)
    return o


def _ph(S=3, cm=1, **kw):
    return PH(_opts(**kw), farmer.scenario_names_creator(S), farmer.scenario_creator,
              scenario_creator_kwargs={"crops_multiplier": cm, "num_scens": S})


def test_lagrangian_spoke_reference_value():
    ph = _ph()
    ph.ph_main(finalize=False)
    sp = LagrangianOuterBound(ph)
    sp.update()
    b = sp.finalize()
    assert abs(b - (-109499.5160897)) < 0.05, b
    o = oph.OraclePH(_opts(), om.farmer_names(3), om.farmer, dict(crops_multiplier=1, num_scens=3))
    ob = o.lagrangian_bound(ph.Ws())
    assert abs(b - ob) <= 1e-6 * abs(ob), (b, ob)
    sp.close()


@pytest.mark.parametrize("S,cm", [(3, 1), (12, 2)])
def test_xhat_spoke_vs_oracle(S, cm):
    ph = _ph(S, cm)
    ph.ph_main(finalize=False)
    sp = XhatShuffleInnerBound(ph)
    sp.update()
    b = sp.finalize()
    cand = sp.current
    xhat = ph.nonants()[cand]
    o = oph.OraclePH(_opts(), om.farmer_names(S), om.farmer, dict(crops_multiplier=cm, num_scens=S))
    ob = o.xhat_eval(xhat)
    assert ob is not None and b is not None
    assert abs(b - ob) <= 1e-6 * abs(ob), (b, ob)
    sp.close()


def test_wheel_hub_and_spokes_gap():
    S = 3
    hub_dict = {"hub_class": PHHub, "hub_kwargs": {"options": {"rel_gap": 0.01}}, "opt_class": PH,
                "opt_kwargs": {"options": _opts(PHIterLimit=200), "all_scenario_names": farmer.scenario_names_creator(S),
                               "scenario_creator": farmer.scenario_creator,
                               "scenario_creator_kwargs": {"crops_multiplier": 1, "num_scens": S}}}
    spokes = [{"spoke_class": LagrangianOuterBound}, {"spoke_class": XhatShuffleInnerBound}]
    wheel = WheelSpinner(hub_dict, spokes).spin()
    ob, ib = wheel.BestOuterBound, wheel.BestInnerBound
    ef = -108390.0                      # farmer EF optimum (doc/src/examples.rst:382)
    assert ob <= ef + 1e-3 and ib >= ef - 1e-3, (ob, ib)
    assert (ib - ob) / abs(ob) <= 0.01 + 1e-9, (ob, ib)
    assert wheel.spcomm.opt._PHIter < 200


def _np_safe_bound(batch, y, c_min, lo, hi, sense, off):
    """numpy restatement of bound.hip for an LP (no prox), unscaled: the duals sign-projected onto
    the finite row bounds, r = c - A^T y, the free columns' reduced costs repaired by moving their
    rows' duals toward 0 (free columns ascending, each column's rows ascending), then the
    certificate sum_i y_i (lo_i | hi_i) + sum_j min over [lo_j, hi_j] of r_j x_j."""
    m, n = batch.m, batch.n
    rp, ci = batch.rowptr, batch.colidx
    rows = np.repeat(np.arange(m), np.diff(rp))
    out = []
    for s in range(batch.S):
        v = batch.vals[s]
        Y = y[s].copy()
        Y[(Y > 0) & ~np.isfinite(batch.rl[s])] = 0.0
        Y[(Y < 0) & ~np.isfinite(batch.ru[s])] = 0.0
        R = c_min[s] - np.bincount(ci, weights=v * Y[rows], minlength=n)
        free = [j for j in range(n) if not (np.isfinite(lo[:, j]).all() and np.isfinite(hi[:, j]).all())]
        for _ in range(4):
            anyv = False
            for j in free:
                r = R[j]
                if r < 0 and not np.isfinite(hi[s, j]):
                    need, d = -r, 1
                elif r > 0 and not np.isfinite(lo[s, j]):
                    need, d = r, -1
                else:
                    continue
                anyv = True
                for p in np.nonzero(ci == j)[0]:
                    if need <= 0:
                        break
                    i, av = rows[p], v[p]
                    cap = d * av * Y[i]
                    if not cap > 0:
                        continue
                    dl = min(need, cap)
                    y1 = 0.0 if dl == cap else Y[i] - d * dl / av
                    dy = y1 - Y[i]
                    Y[i] = y1
                    R[ci[rp[i]:rp[i + 1]]] -= v[rp[i]:rp[i + 1]] * dy
                    need -= dl
            if not anyv:
                break
        t = np.sum(np.where(Y > 0, Y * np.where(Y > 0, batch.rl[s], 0), np.where(Y < 0, Y * batch.ru[s], 0)))
        with np.errstate(invalid="ignore"):
            t += np.sum(np.where(R > 0, R * lo[s], np.where(R < 0, R * hi[s], 0.0)))
        out.append(sense * (t + off[s]))
    return np.array(out)


@pytest.mark.parametrize("cap", [16, 64, 256])
def test_safe_bounds_at_iteration_cap(cap):
    """Solves stopped at the PDHG iteration cap still give VALID bounds (phg_opts.safe_bound,
    bound.hip): Iter0's trivial bound and the Lagrangian spoke's bound are finite and at or below
    the exact LP values (the oracle's HiGHS), and equal to the numpy restatement of the certificate
    built from the device's dual iterate (presolve off, so the rows are the caller's).  With the
    safe bounds switched off the old behaviour holds: no bound at the cap."""
    from mpisppy_amd.engine import implied_bounds
    cp = {"pdhg_max_iter": cap}
    ph = _ph(3, 1, iter0_solver_options=cp, iterk_solver_options=cp, PHIterLimit=3, pdhg_presolve=False)
    ph.PH_Prep()
    tb = ph.Iter0()
    assert (ph.engine.get_i32(_lib.I_STATUS) == 1).all()
    o = oph.OraclePH(_opts(), om.farmer_names(3), om.farmer, dict(crops_multiplier=1, num_scens=3))
    otb = o.Iter0()
    assert np.isfinite(tb) and tb <= otb + 1e-9 * abs(otb), (tb, otb)
    b = ph.engine.batch
    lo, hi, _ = implied_bounds(b)
    y = ph.engine.get(_lib.F_Y).reshape(b.S, b.m)
    want = _np_safe_bound(b, y, b.sense * b.c, lo, hi, b.sense, b.sense * b.off)
    got = ph.engine.get(_lib.F_BOUND)
    np.testing.assert_allclose(got, want, rtol=1e-9, atol=1e-9)
    ph.iterk_loop()
    sp = LagrangianOuterBound(ph, options={"pdhg_max_iter": cap})
    sp.update()
    lb = sp.finalize()
    olb = o.lagrangian_bound(ph.Ws())
    assert lb is not None and lb <= olb + 1e-9 * abs(olb), (lb, olb)
    sp.close()
    # safe bounds off: an iteration-limited solve certifies nothing
    ph2 = _ph(3, 1, iter0_solver_options=cp, PHIterLimit=1, pdhg_safe_bound=False)
    ph2.PH_Prep()
    assert ph2.Iter0() == -np.inf


def test_safe_bounds_converged_match_exact():
    """At convergence the safe certificate is the LP optimum: Iter0 trivial bound of farmer 30
    scenarios (cm=1) within 1e-7 of the oracle's, and the reference's pinned -137846 (3 s.f.,
    test_aph.py:249-253)."""
    names = [f"Scenario{k}" for k in range(1, 31)]
    ph = PH(_opts(PHIterLimit=1), names, farmer.scenario_creator,
            scenario_creator_kwargs={"crops_multiplier": 1, "num_scens": 30})
    ph.PH_Prep()
    tb = ph.Iter0()
    o = oph.OraclePH(_opts(), names, om.farmer, dict(crops_multiplier=1, num_scens=30))
    otb = o.Iter0()
    assert tb <= otb + 1e-9 * abs(otb)
    assert abs(tb - otb) <= 1e-7 * abs(otb), (tb, otb)
    assert round(tb, -3) == -138000.0


def test_spoke_copy_ordered_against_queued_hub_updates():
    """The spoke's copy of the hub's W (phg_copy_from, on the spoke's stream) is ordered both ways
    against the hub's stream: hub W updates queued right after the copy never tear it, so every
    copy satisfies sum_s p_s W_s = 0 and equals one of the hub's W states (ADVICE: cross-stream
    ordering).  10 000 scenarios x 30 nonants, so a torn copy would be likely if unordered."""
    ph = _ph(10000, 10, PHIterLimit=2)
    ph.ph_main(finalize=False)
    sp = LagrangianOuterBound(ph)
    p = ph.engine.batch.prob
    for _ in range(4):
        before = ph.engine.get(_lib.F_W)
        sp.engine.copy_from(ph.engine, _lib.F_W)      # queued on the spoke's stream
        ph.Compute_Xbar()                             # hub updates queued right behind it
        ph.Update_W()
        ph.engine.sync()
        sp.engine.sync()
        Wc = sp.engine.get(_lib.F_W)
        assert np.array_equal(Wc, before)
        Wc = Wc.reshape(len(p), -1)
        assert np.abs(p @ Wc).max() <= 1e-9 * max(1.0, np.abs(Wc).max())
    sp.close()
