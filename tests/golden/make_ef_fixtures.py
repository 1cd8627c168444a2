"""Generate the extensive-form (EF) golden fixtures of the north-star target (run in the container,
not on the GPU box; the outputs are committed next to this script).

The north-star target is "farmer with 10k scenarios reaches PH convergence < 1e-4 with objective
within 1e-6 of the reference".  The reference's answer for that instance is its EF optimum
(``mpisppy/utils/sputils.py:143-357`` create_EF: block-diagonal scenario LPs, objective
sum_s p_s f_s, nonanticipativity rows x_{s,ROOT,i} = x_{first scenario,ROOT,i}), solved by a CPU LP
solver.  Here the EF is solved by the oracle's HiGHS 1.8 (scipy's bundled copy) -- the same
restated scenario LPs (``oracle.models.farmer``, pinned to the reference's fixtures by
``tests/test_oracle_pins.py``) stacked with scipy.sparse instead of ``oracle.ph.ef_solve``'s
Python loops, so 10 000 scenarios x 120 columns build in seconds.

Output: ``farmer_cm{cm}_ef_S{S}.json`` = {objective, root nonants (ROOT node order: sorted
DevotedAcreage keys), HiGHS status / iterations / time, instance}.

    python tests/golden/make_ef_fixtures.py 1000 10000
    python tests/golden/make_ef_fixtures.py ph 30       # the oracle's PH to conv < 1e-4
"""
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import models as om  # noqa: E402
from scipy.optimize._highspy import _core as _hc  # noqa: E402


def farmer_ef(S, cm=10):
    scens = [om.farmer(nm, crops_multiplier=cm, num_scens=S) for nm in om.farmer_names(S)]
    arrs = [s.arrays() for s in scens]
    n = scens[0].n
    m = scens[0].m
    cols = np.array(scens[0].nonant_cols(), dtype=np.int64)
    N = len(cols)
    blocks = [sp.csr_matrix((a["vals"], a["colidx"], a["rowptr"]), shape=(m, n)) for a in arrs]
    A = sp.block_diag(blocks, format="csr")
    # nonanticipativity: x_{s, col_i} - x_{0, col_i} = 0 for s >= 1 (create_EF ties every scenario
    # to the node's first scenario)
    r = np.arange((S - 1) * N)
    s_of = 1 + r // N
    i_of = r % N
    na = sp.csr_matrix((np.concatenate([np.ones(len(r)), -np.ones(len(r))]),
                        (np.concatenate([r, r]), np.concatenate([s_of * n + cols[i_of], cols[i_of]]))),
                       shape=((S - 1) * N, S * n))
    A = sp.vstack([A, na], format="csr")
    p = 1.0 / S
    c = np.concatenate([p * a["c"] for a in arrs])
    rlo = np.concatenate([a["row_lo"] for a in arrs] + [np.zeros((S - 1) * N)])
    rhi = np.concatenate([a["row_hi"] for a in arrs] + [np.zeros((S - 1) * N)])
    clo = np.concatenate([a["col_lo"] for a in arrs])
    chi = np.concatenate([a["col_hi"] for a in arrs])
    return c, A, rlo, rhi, clo, chi, cols, n, scens


def _fin(v):
    v = np.asarray(v, dtype=np.float64)
    return np.where(np.isfinite(v), v, np.where(v > 0, _hc.kHighsInf, -_hc.kHighsInf))


def solve_lp(c, A, rlo, rhi, clo, chi, solver="ipm", threads=8):
    h = _hc._Highs()
    h.setOptionValue("output_flag", False)
    h.setOptionValue("threads", threads)
    h.setOptionValue("solver", solver)
    h.setOptionValue("primal_feasibility_tolerance", 1e-9)
    h.setOptionValue("dual_feasibility_tolerance", 1e-9)
    if solver == "ipm":
        h.setOptionValue("ipm_optimality_tolerance", 1e-12)
        h.setOptionValue("run_crossover", "on")
    lp = _hc.HighsLp()
    lp.num_col_ = len(c)
    lp.num_row_ = A.shape[0]
    lp.col_cost_ = np.asarray(c, np.float64)
    lp.col_lower_ = _fin(clo)
    lp.col_upper_ = _fin(chi)
    lp.row_lower_ = _fin(rlo)
    lp.row_upper_ = _fin(rhi)
    Ac = A.tocsc()
    lp.a_matrix_.format_ = _hc.MatrixFormat.kColwise
    lp.a_matrix_.start_ = Ac.indptr.astype(np.int32)
    lp.a_matrix_.index_ = Ac.indices.astype(np.int32)
    lp.a_matrix_.value_ = Ac.data.astype(np.float64)
    h.passModel(lp)
    t0 = time.perf_counter()
    h.run()
    dt = time.perf_counter() - t0
    st = h.modelStatusToString(h.getModelStatus())
    sol = h.getSolution()
    info = h.getInfo()
    return st, np.array(sol.col_value), float(info.objective_function_value), dt, {
        "simplex_iterations": int(info.simplex_iteration_count), "ipm_iterations": int(info.ipm_iteration_count)}


def main(sizes, cm=10):
    for S in sizes:
        t0 = time.perf_counter()
        c, A, rlo, rhi, clo, chi, cols, n, scens = farmer_ef(S, cm)
        tb = time.perf_counter() - t0
        st, x, obj, dt, it = solve_lp(c, A, rlo, rhi, clo, chi)
        root = x[cols]
        # every scenario's nonants equal the root's (nonanticipativity holds to the solver tolerance)
        X = x.reshape(S, n)[:, cols]
        na_err = float(np.max(np.abs(X - root)))
        ax = A @ x
        feas = float(max(np.max(np.maximum(rlo - ax, 0)), np.max(np.maximum(ax - rhi, 0))))
        out = {"instance": f"farmer crops_multiplier={cm}, scen0..scen{S - 1}, p=1/S (examples/farmer/farmer.py)",
               "S": S, "cm": cm, "objective": obj, "root_nonants": root.tolist(),
               "nonant_names": [v.name for v in [None] * 0] or None,
               "solver": "HiGHS 1.8.0 (scipy) ipm + crossover, tol 1e-9", "status": st,
               "solve_seconds": round(dt, 2), "build_seconds": round(tb, 2), **it,
               "max_nonanticipativity_violation": na_err, "max_row_violation": feas}
        out.pop("nonant_names")
        fn = os.path.join(HERE, f"farmer_cm{cm}_ef_S{S}.json")
        with open(fn, "w") as f:
            json.dump(out, f, indent=1)
        print(fn, st, obj, f"{dt:.1f}s", flush=True)


def oracle_ph(S=30, cm=10, thr=1e-4, max_iter=5000):
    """The oracle's own PH to convergence on the same instance (``oracle/ph.py``, HiGHS subproblem
    solves certified by KKT checks): ``oracle_ph_farmer_cm{cm}_S{S}.json``."""
    from oracle import ph as oph
    opts = {"defaultPHrho": 1.0, "PHIterLimit": max_iter, "convthresh": thr}
    t0 = time.perf_counter()
    o = oph.OraclePH(opts, om.farmer_names(S), om.farmer, dict(crops_multiplier=cm, num_scens=S))
    conv, eobj, tb = o.ph_main()
    out = {"instance": f"farmer crops_multiplier={cm}, scen0..scen{S - 1}, rho=1, convthresh={thr}",
           "S": S, "cm": cm, "conv": conv, "ph_iters": o._PHIter, "Eobj": eobj, "trivial_bound": tb,
           "xbar": list(map(float, o.xbar[0])), "seconds": round(time.perf_counter() - t0, 1)}
    fn = os.path.join(HERE, f"oracle_ph_farmer_cm{cm}_S{S}.json")
    with open(fn, "w") as f:
        json.dump(out, f, indent=1)
    print(fn, o._PHIter, conv, eobj, flush=True)


if __name__ == "__main__":
    if sys.argv[1:2] == ["ph"]:
        oracle_ph(*[int(a) for a in sys.argv[2:3]])
    else:
        main([int(a) for a in sys.argv[1:]] or [1000])
