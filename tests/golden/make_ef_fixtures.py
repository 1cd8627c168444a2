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
    python tests/golden/make_ef_fixtures.py first 30 1000 10000   # first-stage uniqueness / stiffness
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


def solve_lp(c, A, rlo, rhi, clo, chi, solver="ipm", threads=8, crossover=True):
    h = _hc._Highs()
    h.setOptionValue("output_flag", False)
    h.setOptionValue("threads", threads)
    h.setOptionValue("solver", solver)
    h.setOptionValue("primal_feasibility_tolerance", 1e-9)
    h.setOptionValue("dual_feasibility_tolerance", 1e-9)
    if solver == "ipm":
        h.setOptionValue("ipm_optimality_tolerance", 1e-12)
        # crossover on 1.2M columns (S = 10 000) does not finish in an hour here: the IPM point at
        # relative optimality 1e-12 is what the fixture records at that size
        h.setOptionValue("run_crossover", "on" if crossover else "off")
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
        cross = S <= 2000
        st, x, obj, dt, it = solve_lp(c, A, rlo, rhi, clo, chi, crossover=cross)
        root = x[cols]
        # every scenario's nonants equal the root's (nonanticipativity holds to the solver tolerance)
        X = x.reshape(S, n)[:, cols]
        na_err = float(np.max(np.abs(X - root)))
        ax = A @ x
        feas = float(max(np.max(np.maximum(rlo - ax, 0)), np.max(np.maximum(ax - rhi, 0))))
        out = {"instance": f"farmer crops_multiplier={cm}, scen0..scen{S - 1}, p=1/S (examples/farmer/farmer.py)",
               "S": S, "cm": cm, "objective": obj, "root_nonants": root.tolist(),
               "solver": "HiGHS 1.8.0 (scipy) ipm" + (" + crossover" if cross else " (no crossover, optimality tol 1e-12)")
                         + ", feasibility tol 1e-9", "status": st,
               "solve_seconds": round(dt, 2), "build_seconds": round(tb, 2), **it,
               "max_nonanticipativity_violation": na_err, "max_row_violation": feas}
        fn = os.path.join(HERE, f"farmer_cm{cm}_ef_S{S}.json")
        with open(fn, "w") as f:
            json.dump(out, f, indent=1)
        print(fn, st, obj, f"{dt:.1f}s", flush=True)


def farmer_ef_separable(S, cm=10):
    """The farmer EF solved exactly by its structure (no LP solver): once DevotedAcreage a_c is
    fixed, crop c's second stage in scenario s is the convex piecewise-linear
        Q_sc(a) = PP max(CFR - Y a, 0) - SUB min(max(Y a - CFR, 0), QUOTA) - SUP max(Y a - CFR - QUOTA, 0)
    (buy the cattle-feed shortfall; sell the surplus under / over quota -- purchase > sub > super
    price, so nothing is bought to be resold), so the EF is  min sum_c f_c(a_c)  s.t.
    sum_c a_c <= 500 cm, 0 <= a_c <= 500 cm  with f_c(a) = PLANT a + sum_s p_s Q_sc(a) separable
    convex piecewise linear: filling the budget greedily along all crops' segments in order of
    increasing slope (while the slope is negative) is exact.  Checked against the LP EF
    (HiGHS + crossover) at S = 30 and 1 000 before its S = 10 000 answer is used."""
    scens = [om.farmer(nm, crops_multiplier=cm, num_scens=S) for nm in om.farmer_names(S)]
    crops = [f"{cb}{i}" for i in range(cm) for cb in om._FARMER_BASE]
    base = {f"{cb}{i}": cb for i in range(cm) for cb in om._FARMER_BASE}
    B = 500.0 * cm
    p = 1.0 / S
    segs = []          # (slope, crop, start, end)
    fdata = {}
    for cn in crops:
        cb = base[cn]
        Y = np.array([sc.yields[cn] for sc in scens])
        cfr, quota = om._CATTLE[cb], om._PRICE_QUOTA[cb]
        pp, sub, sup, plant = om._PURCHASE[cb], om._SUB_PRICE[cb], om._SUPER_PRICE[cb], om._PLANT[cb]
        fdata[cn] = (Y, cfr, quota, pp, sub, sup, plant)
        # breakpoints of every scenario's term inside [0, B]
        bps = np.concatenate([cfr / Y, (cfr + quota) / Y, [0.0, B]])
        bps = np.unique(np.clip(bps, 0.0, B))
        mid = 0.5 * (bps[:-1] + bps[1:])
        ya = np.outer(mid, Y)                                     # [segments, S]
        sl = np.where(ya < cfr, -pp, np.where(ya < cfr + quota, -sub, -sup)) * Y
        slope = plant + p * sl.sum(axis=1)
        for k in range(len(mid)):
            segs.append((float(slope[k]), cn, float(bps[k]), float(bps[k + 1])))
    segs.sort(key=lambda t: t[0])
    a = {cn: 0.0 for cn in crops}
    left = B
    for slope, cn, lo, hi in segs:
        if slope >= 0.0 or left <= 0.0:
            break
        assert abs(a[cn] - lo) < 1e-9 * B, "segments of a crop out of order (f_c not convex?)"
        take = min(hi - lo, left)
        a[cn] = lo + take
        left -= take

    def f(cn, av):
        Y, cfr, quota, pp, sub, sup, plant = fdata[cn]
        prod = Y * av
        q = pp * np.maximum(cfr - prod, 0.0) - sub * np.minimum(np.maximum(prod - cfr, 0.0), quota) \
            - sup * np.maximum(prod - cfr - quota, 0.0)
        return plant * av + p * float(np.sum(q))
    obj = sum(f(cn, a[cn]) for cn in crops)
    order = sorted(crops)                                         # nonant order: sorted keys
    return obj, [a[cn] for cn in order]


def farmer_ef_first_stage(S, cm=10):
    """Uniqueness of the farmer EF's first stage, from the separable structure of
    farmer_ef_separable.  With mu = the land price (minus the slope of the last segment the greedy
    fill used, 0 if the budget is slack) every feasible a satisfies, by convexity of the f_c and
    Sum a <= B,
        f(a) - f* >= Sum_c [(s_c^+ + mu) (a_c - a*_c)^+ + (-mu - s_c^-) (a*_c - a_c)^+]
    with s_c^-, s_c^+ the left / right slopes of f_c at a*_c (-inf / +inf at 0 / B).  So a crop with
    stiffness kappa_c = min(s_c^+ + mu, -mu - s_c^-) > 0 can move by at most (f(a) - f*) / kappa_c;
    a crop on the marginal segment (kappa_c = 0) moves only with the others or with idle land:
    |a_m - a*_m| <= Sum_{c != m} |a_c - a*_c| + (f(a) - f*) / mu.  The first stage is unique iff at
    most one crop is marginal (exact slope ties: relative 1e-12).  Returns the dict stored as the
    fixture's "first_stage"."""
    scens = [om.farmer(nm, crops_multiplier=cm, num_scens=S) for nm in om.farmer_names(S)]
    crops = [f"{cb}{i}" for i in range(cm) for cb in om._FARMER_BASE]
    base = {f"{cb}{i}": cb for i in range(cm) for cb in om._FARMER_BASE}
    B = 500.0 * cm
    p = 1.0 / S
    segs = {}
    for cn in crops:
        cb = base[cn]
        Y = np.array([sc.yields[cn] for sc in scens])
        cfr, quota = om._CATTLE[cb], om._PRICE_QUOTA[cb]
        pp, sub, sup, plant = om._PURCHASE[cb], om._SUB_PRICE[cb], om._SUPER_PRICE[cb], om._PLANT[cb]
        bps = np.unique(np.clip(np.concatenate([cfr / Y, (cfr + quota) / Y, [0.0, B]]), 0.0, B))
        mid = 0.5 * (bps[:-1] + bps[1:])
        ya = np.outer(mid, Y)
        sl = np.where(ya < cfr, -pp, np.where(ya < cfr + quota, -sub, -sup)) * Y
        segs[cn] = (bps, plant + p * sl.sum(axis=1))
    allseg = sorted((float(sl[k]), cn, float(bps[k]), float(bps[k + 1])) for cn, (bps, sl) in segs.items()
                    for k in range(len(sl)))
    a = {cn: 0.0 for cn in crops}
    left, last = B, 0.0
    for slope, cn, lo, hi in allseg:
        if slope >= 0.0 or left <= 0.0:
            break
        take = min(hi - lo, left)
        a[cn] = lo + take
        left -= take
        last = slope
    mu = -last if left <= 1e-9 * B else 0.0
    out = {}
    tol = 1e-12 * max(1.0, max(abs(v[0]) for v in allseg))
    marginal = []
    for cn in crops:
        bps, sl = segs[cn]
        x = a[cn]
        # left slope: segment ending at or containing x; right slope: segment starting at or containing x
        k = int(np.searchsorted(bps, x, side="left"))
        inside = 0 < k < len(bps) and bps[k] != x and bps[k - 1] < x
        if inside:
            s_lo = s_hi = float(sl[k - 1])
        else:
            kk = int(np.argmin(np.abs(bps - x)))
            s_lo = float(sl[kk - 1]) if kk > 0 else -np.inf
            s_hi = float(sl[kk]) if kk < len(sl) else np.inf
        kap = min(s_hi + mu, -mu - s_lo)
        if kap <= tol:
            marginal.append(cn)
        out[cn] = {"a": x, "slope_left": s_lo, "slope_right": s_hi, "kappa": kap}
    order = sorted(crops)
    return {"land_price_mu": mu, "budget_slack": left, "marginal_crops": marginal,
            "unique": len(marginal) <= 1,
            "kappa": [out[cn]["kappa"] for cn in order], "a": [out[cn]["a"] for cn in order],
            "crops": order,
            "bound": "f(a) - f* >= sum_c kappa_c |a_c - a*_c| over non-marginal crops (make_ef_fixtures."
                     "farmer_ef_first_stage)"}


def first_stage_fixture(sizes, cm=10):
    for S in sizes:
        fn = os.path.join(HERE, f"farmer_cm{cm}_ef_S{S}.json")
        d = json.load(open(fn))
        fs = farmer_ef_first_stage(S, cm)
        assert max(abs(x - y) for x, y in zip(fs["a"], d["root_nonants"])) < 1e-9 * 500 * cm
        d["first_stage"] = fs
        with open(fn, "w") as fh:
            json.dump(d, fh, indent=1)
        print(fn, "unique" if fs["unique"] else "NOT unique", "marginal", fs["marginal_crops"],
              "min kappa (non-marginal)", min(k for k in fs["kappa"] if k > 0), flush=True)


def separable_fixture(sizes, cm=10):
    for S in sizes:
        t0 = time.perf_counter()
        obj, root = farmer_ef_separable(S, cm)
        fn = os.path.join(HERE, f"farmer_cm{cm}_ef_S{S}.json")
        prev = json.load(open(fn)) if os.path.exists(fn) else None
        out = {"instance": f"farmer crops_multiplier={cm}, scen0..scen{S - 1}, p=1/S (examples/farmer/farmer.py)",
               "S": S, "cm": cm, "objective": obj, "root_nonants": root,
               "solver": "exact separable solution of the farmer EF (make_ef_fixtures.farmer_ef_separable), "
                         "checked against the HiGHS LP EF at S = 30 and 1000",
               "status": "Optimal", "solve_seconds": round(time.perf_counter() - t0, 2)}
        if prev is not None and prev.get("status") == "Optimal" and "separable" not in prev.get("solver", ""):
            out["lp_ef_objective"] = prev["objective"]
            out["lp_ef_solver"] = prev["solver"]
            out["rel_diff_vs_lp_ef"] = abs(obj - prev["objective"]) / abs(prev["objective"])
        with open(fn, "w") as fh:
            json.dump(out, fh, indent=1)
        print(fn, obj, out.get("rel_diff_vs_lp_ef"), flush=True)


_POOL_ARR = None


def _pool_solve(args):
    """One scenario QP in a worker (the oracle's highs.solve on the forked scenario arrays)."""
    from oracle import highs
    k, c, q, off, threads = args
    a = _POOL_ARR[k]
    r = highs.solve(c, a["rowptr"], a["colidx"], a["vals"], a["row_lo"], a["row_hi"], a["col_lo"], a["col_hi"],
                    qdiag=q, offset=off, threads=threads)
    return k, bool(r.ok), str(r.status), r.x, r.obj


def oracle_ph(S=30, cm=10, thr=1e-4, max_iter=20000, procs=8):
    """The oracle's own PH to convergence on the same instance (``oracle/ph.py``, HiGHS subproblem
    solves certified by KKT checks): ``oracle_ph_farmer_cm{cm}_S{S}.json``.  The scenario solves
    of each PH iteration go to a process pool (the oracle's solve_one, split into building the
    objective here and the HiGHS call in a worker; same results, ~procs x faster)."""
    import multiprocessing as mp
    from oracle import ph as oph

    class PoolPH(oph.OraclePH):
        def solve_loop(self):
            jobs = []
            for k in range(self.S):
                a = self.arr[k]
                sg = 1.0 if self.scen[k].sense == 1 else -1.0
                c = sg * a["c"].copy()
                q = None
                off = 0.0
                cols = self.cols[k]
                if self.W_on:
                    np.add.at(c, cols, self.W[k])
                if self.prox_on:
                    rho = self.rho[k]
                    xb = self.xbar[k]
                    np.add.at(c, cols, -rho * xb)
                    q = np.zeros_like(c)
                    np.add.at(q, cols, rho)
                    off = float(np.sum(rho / 2.0 * xb * xb))
                jobs.append((k, c, q, off, self.threads))
            for k, ok, st, x, obj in pool.map(_pool_solve, jobs):
                if not ok:
                    raise RuntimeError(f"[oracle] Solve failed for scenario {self.names[k]}: {st}")
                sg = 1.0 if self.scen[k].sense == 1 else -1.0
                self.feasible[k] = True
                self.x[k] = x
                self.obj[k] = sg * obj
                self.outer[k] = sg * obj
            self.solve_count += self.S
            if self._PHIter % 100 == 0:
                print(f"PH iter {self._PHIter} conv {self.conv}", flush=True)

    global _POOL_ARR
    opts = {"defaultPHrho": 1.0, "PHIterLimit": max_iter, "convthresh": thr}
    t0 = time.perf_counter()
    o = PoolPH(opts, om.farmer_names(S), om.farmer, dict(crops_multiplier=cm, num_scens=S))
    _POOL_ARR = o.arr
    o._PHIter = 0
    pool = mp.get_context("fork").Pool(procs)
    conv, eobj, tb = o.ph_main()
    pool.close()
    out = {"instance": f"farmer crops_multiplier={cm}, scen0..scen{S - 1}, rho=1, convthresh={thr}",
           "S": S, "cm": cm, "conv": conv, "ph_iters": o._PHIter, "Eobj": eobj, "trivial_bound": tb,
           "xbar": list(map(float, o.xbar[0])), "seconds": round(time.perf_counter() - t0, 1)}
    fn = os.path.join(HERE, f"oracle_ph_farmer_cm{cm}_S{S}.json")
    with open(fn, "w") as f:
        json.dump(out, f, indent=1)
    print(fn, o._PHIter, conv, eobj, flush=True)


def oracle_ph_iters(S=30, cm=10, iters=100, procs=8):
    """The oracle's PH for a FIXED number of iterations (convthresh 0: no early stop) on farmer
    cm={cm}: per-iteration convergence metric, E[obj], trivial bound, x-bar and W after the last
    iteration -> ``oracle_ph_farmer_cm{cm}_S{S}_it{iters}.json``.  (The oracle's PH to conv < 1e-4
    does not finish here: its HiGHS 1.8 QP solves stop ~1e-2 short of the optimum, and at S = 30
    its metric hovered around 1e-3 after 2 900 iterations / 95 min on 8 processes.)"""
    import multiprocessing as mp
    from oracle import ph as oph
    opts = {"defaultPHrho": 1.0, "PHIterLimit": iters, "convthresh": 0.0}
    t0 = time.perf_counter()
    state = {}

    class PoolPH(oph.OraclePH):
        def solve_loop(self):
            jobs = []
            for k in range(self.S):
                a = self.arr[k]
                sg = 1.0 if self.scen[k].sense == 1 else -1.0
                c = sg * a["c"].copy()
                q = None
                off = 0.0
                cols = self.cols[k]
                if self.W_on:
                    np.add.at(c, cols, self.W[k])
                if self.prox_on:
                    rho = self.rho[k]
                    xb = self.xbar[k]
                    np.add.at(c, cols, -rho * xb)
                    q = np.zeros_like(c)
                    np.add.at(q, cols, rho)
                    off = float(np.sum(rho / 2.0 * xb * xb))
                jobs.append((k, c, q, off, self.threads))
            for k, ok, st, x, obj in state["pool"].map(_pool_solve, jobs):
                if not ok:
                    raise RuntimeError(f"[oracle] Solve failed for scenario {self.names[k]}: {st}")
                sg = 1.0 if self.scen[k].sense == 1 else -1.0
                self.feasible[k] = True
                self.x[k] = x
                self.obj[k] = sg * obj
                self.outer[k] = sg * obj
            self.solve_count += self.S

    global _POOL_ARR
    o = PoolPH(opts, om.farmer_names(S), om.farmer, dict(crops_multiplier=cm, num_scens=S))
    _POOL_ARR = o.arr
    state["pool"] = mp.get_context("fork").Pool(procs)
    tb = o.Iter0()
    # Iter0's LPs may have several optimal x (the trivial bound is unique, the nonants need not
    # be): the GPU test starts its PH from THESE nonants, after which every prox-QP has unique ones
    x0 = np.array([o.nonants(k) for k in range(o.S)])
    o.iterk_loop()
    eobj = o.Eobjective()
    conv = o.conv
    state["pool"].close()
    out = {"instance": f"farmer crops_multiplier={cm}, scen0..scen{S - 1}, rho=1, {iters} PH iterations (no early stop)",
           "S": S, "cm": cm, "iters": iters, "x0_nonants": x0.tolist(),
           "conv_history": list(map(float, o.history)), "Eobj": eobj,
           "trivial_bound": tb, "xbar": list(map(float, o.xbar[0])), "W": np.asarray(o.W).tolist(),
           "solver": "oracle/ph.py (HiGHS 1.8 QP via scipy per scenario)", "seconds": round(time.perf_counter() - t0, 1)}
    fn = os.path.join(HERE, f"oracle_ph_farmer_cm{cm}_S{S}_it{iters}.json")
    with open(fn, "w") as f:
        json.dump(out, f)
    print(fn, o._PHIter, conv, eobj, flush=True)


if __name__ == "__main__":
    if sys.argv[1:2] == ["sep"]:
        separable_fixture([int(a) for a in sys.argv[2:]])
    elif sys.argv[1:2] == ["first"]:
        first_stage_fixture([int(a) for a in sys.argv[2:]])
    elif sys.argv[1:2] == ["phit"]:
        oracle_ph_iters(*[int(a) for a in sys.argv[2:5]])
    elif sys.argv[1:2] == ["ph"]:
        oracle_ph(*[int(a) for a in sys.argv[2:3]])
    else:
        main([int(a) for a in sys.argv[1:]] or [1000])
