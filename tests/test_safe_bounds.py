"""Implied column bounds behind the safe outer bounds (``phg_implied_bounds``, host-only: no GPU).

``phg_opts.safe_bound`` (bound.hip) turns any dual iterate into a weak-duality certificate by
charging reduced costs against a box that holds every feasible point; an infinite column bound is
replaced by one the rows imply.  Checked here: the box holds every vertex HiGHS finds for random
objectives on the same feasible set (so it holds the feasible set's optimal faces the bound is about),
finite bounds are kept as given, and on farmer the only columns left unbounded are QuantityPurchased
(no row caps a purchase; ``examples/farmer/farmer.py:195-203``) -- the ones the kernel's dual repair
handles.
"""
import numpy as np
import pytest

from mpisppy_amd import spbase
from mpisppy_amd.engine import BatchArrays, implied_bounds
from mpisppy_amd.examples import farmer, hydro, netdes, sslp
from oracle import highs


def _batch(names, creator, kw, all_nodenames=None):
    opts = {"solver_name": "phg", "PHIterLimit": 1, "defaultPHrho": 1, "convthresh": 0,
            "verbose": False, "display_progress": False}
    sp = spbase.SPBase(opts, names, creator, all_nodenames=all_nodenames, scenario_creator_kwargs=kw)
    models = [sp.local_scenarios[n] for n in sp.local_scenario_names]
    return BatchArrays(models, sp.all_nodenames, [m._mpisppy_probability for m in models], 0, len(names), 1)


CASES = {
    "farmer": lambda: _batch(farmer.scenario_names_creator(6), farmer.scenario_creator,
                             {"crops_multiplier": 10, "num_scens": 6}),
    "hydro": lambda: _batch(hydro.scenario_names_creator(9), hydro.scenario_creator, {"branching_factors": [3, 3]},
                            spbase.create_nodenames_from_branching_factors([3, 3])),
    "sslp": lambda: _batch(sslp.scenario_names_creator(3), sslp.scenario_creator, {}),
    "netdes": lambda: _batch(netdes.scenario_names_creator(2), netdes.scenario_creator, {"num_scens": 2}),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_implied_box_holds_optimal_vertices(case):
    b = CASES[case]()
    lo, hi, nfree = implied_bounds(b)
    assert lo.shape == (b.S, b.n)
    # finite bounds kept exactly; every new one is finite and on the right side
    fl, fh = np.isfinite(b.cl), np.isfinite(b.cu)
    assert np.array_equal(lo[fl], b.cl[fl]) and np.array_equal(hi[fh], b.cu[fh])
    assert np.all(lo <= hi)
    rng = np.random.default_rng(7)
    for s in range(min(b.S, 2)):
        for trial in range(3 if b.n <= 1000 else 1):
            c = b.c[s] if trial == 0 else rng.normal(size=b.n) * (1.0 + np.abs(b.c[s]))
            # random objectives may be unbounded on the columns the rows leave free: keep those at 0
            if trial:
                c = np.where(np.isfinite(lo[s]) & np.isfinite(hi[s]), c, np.abs(c))
            r = highs.solve(c, b.rowptr, b.colidx, b.vals[s], b.rl[s], b.ru[s], b.cl[s], b.cu[s],
                            presolve="off")
            if r.status != "Optimal":
                continue
            tol = 1e-7 * (1.0 + np.abs(r.x))
            assert np.all(r.x >= lo[s] - tol) and np.all(r.x <= hi[s] + tol), (case, s, trial)


def test_farmer_free_columns_are_purchases():
    b = CASES["farmer"]()
    lo, hi, nfree = implied_bounds(b)
    m = farmer.scenario_creator("scen0", crops_multiplier=10, num_scens=6)
    names = m.column_names()
    free = [names[j] for j in range(b.n) if not (np.isfinite(lo[:, j]).all() and np.isfinite(hi[:, j]).all())]
    assert nfree == len(free) == 30
    assert all(nm.startswith("QuantityPurchased") for nm in free), free
    # quantities sold: capped by yield x acreage (LimitAmountSold) <= yield x total acreage
    sold = [j for j, nm in enumerate(names) if nm.startswith("QuantitySuperQuotaSold")]
    assert np.isfinite(hi[:, sold]).all()
    assert (hi[:, sold] <= 30.0 * 500 * 10).all()   # yields < 30 t/acre, 5 000 acres


@pytest.mark.parametrize("case", ["netdes", "sslp"])
def test_value_forms_expand_identically(case):
    """phg_batch.vals_form: the shared [nnz] form (sslp: only the right-hand sides
    vary) and the sparse delta list (netdes: only the vubs' u_e vary) reach the host-side entry
    points as the same per-scenario matrices -- phg_implied_bounds returns the same bits as for the
    [S*nnz] form; a malformed delta list is rejected."""
    from mpisppy_amd import _lib
    b = CASES[case]()
    ref = implied_bounds(b)
    forms = [_lib.VALS_DELTA] + ([_lib.VALS_SHARED] if (b.vals == b.vals[0]).all() else [])
    if case == "netdes":
        assert 0 < int((b.vals != b.vals[0]).any(axis=0).sum()) <= 1470   # the vubs' u_e only
    for form in forms:
        b.vals_form = form
        got = implied_bounds(b)
        assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]) and got[2] == ref[2]
    b.vals_form = _lib.VALS_DELTA
    cs, keep = b.c_struct()
    if cs.n_delta >= 2:
        pos = np.array([cs.delta_pos[1], cs.delta_pos[0]], np.int32)   # not increasing
        keep.append(pos)
        cs.n_delta, cs.delta_pos = 2, _lib.ptr(pos)
        lo = np.empty(b.S * b.n)
        hi = np.empty(b.S * b.n)
        assert _lib.load().phg_implied_bounds(__import__("ctypes").byref(cs), _lib.ptr(lo), _lib.ptr(hi), None) != 0
        assert b"strictly increasing" in _lib.load().phg_last_error()
    b.vals_form = _lib.VALS_PER_SCENARIO
