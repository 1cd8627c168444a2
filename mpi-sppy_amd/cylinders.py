"""Bound spokes on the MI355X engine (restates ``mpisppy/cylinders/lagrangian_bounder.py:13-98``,
``mpisppy/cylinders/xhatshufflelooper_bounder.py:14-240`` and the spoke side of
``mpisppy/cylinders/spoke.py``).

The reference runs every cylinder in its own MPI ranks and exchanges W / nonants / bounds through
one-sided MPI windows.  Here a spoke is a second (third) ``libphg`` handle on the SAME GPU as the
hub, holding the same scenario batch, with its own HIP stream:

* the hub's ``sync`` (once per PH iteration, ``phbase.py:1037-1040``) hands W / nonants over
  device-to-device (``phg_copy_from`` / ``phg_fix_from``: an event on the hub's stream orders the
  copy behind the hub's queued work, nothing goes through the host);
* the spoke's batched solve then runs on its own stream, overlapping the hub's next PDHG launch;
* at the next ``sync`` the hub collects the bound only if the spoke's stream is idle
  (``phg_query``), so the hub never waits on a spoke -- the asynchrony of the reference's wheel.

Bounds are expectations ``sum_s p_s (.)`` (``spopt.py:344-422``), ``math.fsum`` per rank and a SUM
across ranks (the collect / skip decision is made collectively so every rank takes part).
"""
import math
import random

import numpy as np

from . import _lib
from .engine import Engine



def safe_bound_mode(eps):
    """``phg_opts.safe_bound`` for an outer-bound solve at tolerance ``eps``: 1 (certificates for the
    scenarios that stopped short; a converged scenario keeps its dual objective, accurate to ~eps on
    either side of its optimum, as a CPU solver's bound at its tolerances) when eps is tight, 2 (a
    weak-duality certificate for every scenario) when it is loose enough (> 1e-8) for that accuracy
    to show -- UC's Lagrangian subproblems run at 1e-6."""
    return 2 if eps > 1e-8 else 1

class _BoundSpoke:
    converger_spoke_char = "?"
    bound_kind = None            # "outer" or "inner"

    def __init__(self, hub_opt, options=None):
        self.hub_opt = hub_opt
        self.options = dict(options or {})
        he = hub_opt.engine
        if he is None:
            raise RuntimeError("the hub's engine must exist before its spokes (call PH_Prep first)")
        dev = int(hub_opt.options.get("device", 0))
        try:
            import torch
            if torch.cuda.is_available():
                dev = torch.cuda.current_device()
        except ImportError:
            pass
        # same batch (host arrays), same layout; the spoke's handle creates its own stream
        self.engine = Engine(he.batch, device=dev, stream=None, exchange=None,
                             layout=hub_opt.options.get("pdhg_layout", "auto"),
                             presolve=hub_opt.options.get("pdhg_presolve", True))
        self.engine.set(_lib.F_RHO, he.get(_lib.F_RHO))
        self.pending = False
        self.bound = None
        self.launches = 0
        self.collected = 0

    # ------------------------------------------------------------------ collective helpers
    def _all_idle(self):
        idle = self.engine.idle()
        if self.hub_opt.n_proc > 1:
            return self.hub_opt.mpicomm.allreduce_scalar(0.0 if idle else 1.0) == 0.0
        return idle

    def _rank_fsum(self, vals):
        return self.hub_opt._rank_fsum(vals)

    def _solve_opts(self):
        o = self.hub_opt._solver_opts()
        o.update({k: v for k, v in self.options.items() if k.startswith("pdhg_")})
        return o

    # ------------------------------------------------------------------ protocol
    def update(self, block=False):
        """Called from the hub's sync: collect the finished bound (or None), launch the next solve."""
        b = None
        if self.pending:
            if not block and not self._all_idle():
                return None          # still solving: the hub goes on without waiting
            self.engine.sync()
            b = self._collect()
            self.pending = False
            self.collected += 1
            if b is not None:
                self.bound = b if self.bound is None else self._better(b, self.bound)
        if self._launch():
            self.pending = True
            self.launches += 1
        return b

    def finalize(self):
        """Wait for the spoke's last solve and return its best bound."""
        if self.pending:
            self.engine.sync()
            b = self._collect()
            self.pending = False
            if b is not None:
                self.bound = b if self.bound is None else self._better(b, self.bound)
        return self.bound

    def _better(self, new, old):
        mini = self.hub_opt.is_minimizing
        if self.bound_kind == "outer":
            return max(new, old) if mini else min(new, old)
        return min(new, old) if mini else max(new, old)

    def close(self):
        self.engine.close()


class LagrangianOuterBound(_BoundSpoke):
    """``lagrangian_bounder.py``: solve every scenario with the hub's W, prox off; the outer bound
    is sum_s p_s (dual bound_s) -- each a weak-duality certificate of the scenario's Lagrangian
    subproblem from its dual iterate (``phg_opts.safe_bound``), valid whatever the solve's status."""
    converger_spoke_char = "L"
    bound_kind = "outer"

    def _launch(self):
        # the hub's W, and the hub's last prox-QP solution as the warm start (x, y and the primal
        # weight, phg_copy_from PHG_F_WARM): as PH converges x -> xbar and the prox-QP's duals
        # become the Lagrangian LP's, so the LP starts next to its optimum.  Measured on farmer
        # cm=10 at conv 1e-4 (tools/lagr_diag.py): S = 1 000, PDHG cap 200 000 -- cold start 17
        # scenarios at the cap, bound 3.3e-4 below the EF; hub warm start none, 4.3e-6 below.
        self.engine.copy_from(self.hub_opt.engine, _lib.F_W)
        self.engine.copy_from(self.hub_opt.engine, _lib.F_WARM)
        o = self._solve_opts()
        self.engine.solve(1, 0, eps=o["pdhg_eps"], max_iter=o["pdhg_max_iter"],
                          check_every=o["pdhg_check_every"], warm_start=3,
                          schedule=o["pdhg_schedule"], safe_bound=safe_bound_mode(o["pdhg_eps"]))
        return True

    def _collect(self):
        # every scenario's bound is a certificate (safe_bound); only a scenario whose dual iterate
        # gives none (-inf, or a NaN solve) voids this round's bound
        st = self.engine.get_i32(_lib.I_STATUS)
        b = self.engine.get(_lib.F_BOUND)
        ok = float(bool(np.isfinite(b).all() and (st != 2).all()))
        if self.hub_opt.n_proc > 1:
            ok = float(self.hub_opt.mpicomm.allreduce_scalar(1.0 - ok) == 0.0)
        if not ok:
            return None
        p = self.engine.batch.prob
        return self._rank_fsum([p[k] * b[k] for k in range(len(b))])


class XhatShuffleInnerBound(_BoundSpoke):
    """``xhatshufflelooper_bounder.py``: cycle through the scenarios in a seeded shuffle
    (``random.Random(42).sample``); each try fixes every scenario's nonants to the candidate
    scenario's current hub nonants (two-stage) and solves all scenarios; if all are solved the
    inner bound is sum_s p_s obj_s (W and prox off, ``xhat_eval.py:102-170``)."""
    converger_spoke_char = "X"
    bound_kind = "inner"

    def __init__(self, hub_opt, options=None):
        super().__init__(hub_opt, options)
        if self.engine.batch.L != 1:
            raise NotImplementedError("XhatShuffleInnerBound on the GPU engine supports two-stage problems")
        rs = random.Random()
        rs.seed(42)
        names = list(enumerate(hub_opt.all_scenario_names))
        self.order = [k for k, _ in rs.sample(names, len(names))]
        self.pos = 0
        self.current = None
        self.best_candidate = None
        self.best_X = None           # local scenarios x n: the incumbent's full solution
        # an infeasible fixing would run PDHG to its cap: tries use a smaller one
        self.max_iter = int(self.options.get("xhat_max_iter", 20000))
        # fixed values may get a box of half-width xhat_fix_tol * max(1, |v|) (phg_opts.fix_tol);
        # first-stage rows are dropped by the kernels while the nonants are fixed (row_bounds)
        self.fix_tol = float(self.options.get("xhat_fix_tol", 0.0))

    def _candidate_row(self, gidx):
        """Nonants of global scenario gidx from the hub (host vector; summed over ranks)."""
        ho = self.hub_opt
        loc = gidx - ho.scen_global0
        N = ho.engine.N
        row = np.zeros(N)
        if 0 <= loc < ho.engine.S:
            row = ho.engine.get(_lib.F_XN).reshape(ho.engine.S, N)[loc].copy()
        if ho.n_proc > 1:
            row = np.asarray(ho.mpicomm.allreduce_array(row))
        return row

    def _launch(self):
        gidx = self.order[self.pos % len(self.order)]
        self.pos += 1
        ho = self.hub_opt
        loc = gidx - ho.scen_global0
        if ho.n_proc == 1:
            self.engine.fix_from(ho.engine, loc)
        else:
            self.engine.set(_lib.F_FIXED, np.tile(self._candidate_row(gidx), self.engine.S))
        self.current = gidx
        o = self._solve_opts()
        self.engine.solve(0, 0, eps=o["pdhg_eps"], max_iter=min(self.max_iter, o["pdhg_max_iter"]),
                          check_every=o["pdhg_check_every"], warm_start=1 if self.launches else 0,
                          fix_nonants=True, schedule=o["pdhg_schedule"], fix_tol=self.fix_tol)
        return True

    def _collect(self):
        st = self.engine.get_i32(_lib.I_STATUS)
        bad = float((st != 0).sum())
        if self.hub_opt.n_proc > 1:
            bad = self.hub_opt.mpicomm.allreduce_scalar(bad)
        if bad:
            return None              # infeasible (or not solved to tolerance): no bound
        obj = self.engine.get(_lib.F_OBJ)
        p = self.engine.batch.prob
        val = self._rank_fsum([p[k] * obj[k] for k in range(len(obj))])
        if self.bound is None or self._better(val, self.bound) == val:
            # spoke.py:335-367 (update_if_improving / _cache_best_solution): keep the incumbent
            self.best_candidate = self.current
            self.best_X = self.engine.get(_lib.F_X).reshape(self.engine.S, -1)
        return val


def fixed_rows_violation(batch, xhat):
    """Largest violation, relative to max(1, |bound|), of the rows whose columns are all nonants
    (first-stage rows) by the candidate ``xhat`` over the batch's scenarios.  With the nonants fixed
    these rows are constants, which the kernels drop (phg_internal.h: row_bounds) -- as a CPU
    solver's presolve does -- so the candidate's feasibility for them is decided here."""
    cols = np.asarray(batch.nonant_col)
    pos = {int(c): k for k, c in enumerate(cols)}
    worst = 0.0
    for i in range(batch.m):
        p0, p1 = int(batch.rowptr[i]), int(batch.rowptr[i + 1])
        cj = batch.colidx[p0:p1]
        if p1 == p0 or any(int(c) not in pos for c in cj):
            continue
        xv = np.array([xhat[pos[int(c)]] for c in cj])
        ax = batch.vals[:, p0:p1] @ xv
        lo, hi = batch.rl[:, i], batch.ru[:, i]
        with np.errstate(invalid="ignore"):
            v = np.maximum(np.where(np.isfinite(lo), (lo - ax) / np.maximum(1.0, np.abs(lo)), 0.0),
                           np.where(np.isfinite(hi), (ax - hi) / np.maximum(1.0, np.abs(hi)), 0.0))
        worst = max(worst, float(np.max(v)))
    return worst


def evaluate_xhat(opt, xhat, eps=None, max_iter=200000, fix_tol=0.0, feas_tol=1e-7):
    """Inner bound of a two-stage candidate (``xhat_eval.py:102-170`` / ``xhatbase.py:42-235``):
    every local scenario's nonants fixed to ``xhat`` (one vector, node order), W and prox off, one
    batched solve on a temporary handle holding ``opt``'s batch; sum_s p_s obj_s (math.fsum per
    rank, SUM across ranks) if every scenario reached the KKT tolerance, else None.

    First-stage rows (every column a nonant) are checked here against ``feas_tol`` relative to
    max(1, |bound|) -- the part the CPU solver's feasibility tolerance plays in the reference -- and
    dropped from the device solves (they are constants once the nonants are fixed).  A candidate
    assembled from first-order solves at relative KKT 1e-9 meets such a row only to
    eps (1 + ||b||): on farmer cm=10 (quota bounds of 1e5 in b) up to ~5e-4 acres on the
    5 000-acre total-acreage row, hence 1e-7.  ``fix_tol`` (phg_opts.fix_tol) additionally lets each
    fixed value move by fix_tol * max(1, |v|) (0: exact)."""
    he = opt.engine
    if he.batch.L != 1:
        raise NotImplementedError("evaluate_xhat: two-stage batches")
    viol = fixed_rows_violation(he.batch, np.asarray(xhat, np.float64))
    if opt.n_proc > 1:
        viol = opt.mpicomm.allreduce_scalar(viol)   # sum over ranks >= the largest (conservative)
    evaluate_xhat.last_violation = viol
    if viol > feas_tol:
        return None
    dev = 0
    try:
        import torch
        if torch.cuda.is_available():
            dev = torch.cuda.current_device()
    except ImportError:
        pass
    eng = Engine(he.batch, device=dev, stream=None, exchange=None,
                 layout=opt.options.get("pdhg_layout", "auto"), presolve=opt.options.get("pdhg_presolve", True))
    try:
        eng.set(_lib.F_FIXED, np.tile(np.asarray(xhat, np.float64), eng.S))
        o = opt._solver_opts()
        eng.solve(0, 0, eps=eps or o["pdhg_eps"], max_iter=max_iter, check_every=o["pdhg_check_every"],
                  warm_start=0, fix_nonants=True, schedule=False, fix_tol=fix_tol)
        eng.sync()
        st = eng.get_i32(_lib.I_STATUS)
        evaluate_xhat.last_status_counts = np.bincount(st, minlength=3).tolist()
        bad = float((st != 0).sum())
        if opt.n_proc > 1:
            bad = opt.mpicomm.allreduce_scalar(bad)
        if bad:
            return None
        obj = eng.get(_lib.F_OBJ)
        p = eng.batch.prob
        return opt._rank_fsum([p[k] * obj[k] for k in range(len(obj))])
    finally:
        eng.close()


def evaluate_lagrangian(opt, eps=None, max_iter=200000, warm=True):
    """Lagrangian outer bound with ``opt``'s current W (``lagrangian_bounder.py:21-44``): every
    local scenario with W on and prox off, one batched solve on a temporary handle; sum_s p_s
    bound_s, each a weak-duality certificate from the scenario's dual iterate (``phg_opts.
    safe_bound``: valid also where a solve stops at ``max_iter``), or None if some scenario's
    iterate certifies nothing (-inf).  ``warm``: start from ``opt``'s last solution (x, y, primal
    weight; see LagrangianOuterBound._launch)."""
    he = opt.engine
    dev = 0
    try:
        import torch
        if torch.cuda.is_available():
            dev = torch.cuda.current_device()
    except ImportError:
        pass
    eng = Engine(he.batch, device=dev, stream=None, exchange=None,
                 layout=opt.options.get("pdhg_layout", "auto"), presolve=opt.options.get("pdhg_presolve", True))
    try:
        eng.copy_from(he, _lib.F_W)
        if warm:
            eng.copy_from(he, _lib.F_WARM)
        o = opt._solver_opts()
        eng.solve(1, 0, eps=eps or o["pdhg_eps"], max_iter=max_iter, check_every=o["pdhg_check_every"],
                  warm_start=3 if warm else 0, schedule=False, safe_bound=safe_bound_mode(eps or o["pdhg_eps"]))
        eng.sync()
        st = eng.get_i32(_lib.I_STATUS)
        evaluate_lagrangian.last_status_counts = np.bincount(st, minlength=3).tolist()
        b = eng.get(_lib.F_BOUND)
        bad = float((~np.isfinite(b)).sum() + (st == 2).sum())
        if opt.n_proc > 1:
            bad = opt.mpicomm.allreduce_scalar(bad)
        if bad:
            return None
        p = eng.batch.prob
        return opt._rank_fsum([p[k] * b[k] for k in range(len(b))])
    finally:
        eng.close()


def spoke_from_dict(hub_opt, spoke_dict):
    """Build a spoke from a reference-shaped spoke dict (``spin_the_wheel.py``):
    {"spoke_class": cls, "opt_kwargs": {"options": {...}}, "spoke_kwargs": {...}}."""
    cls = spoke_dict["spoke_class"]
    opts = dict((spoke_dict.get("opt_kwargs") or {}).get("options", {}) or {})
    opts.update((spoke_dict.get("spoke_kwargs") or {}).get("options", {}) or {})
    return cls(hub_opt, options=opts)


def gaps(hub):
    """``hub.py:82-103``: absolute and relative gap between the best inner and outer bounds."""
    if hub.opt.is_minimizing:
        abs_gap = hub.BestInnerBound - hub.BestOuterBound
    else:
        abs_gap = hub.BestOuterBound - hub.BestInnerBound
    if math.isfinite(abs_gap) and hub.BestOuterBound != 0 and math.isfinite(hub.BestOuterBound):
        rel_gap = abs_gap / abs(hub.BestOuterBound)
    else:
        rel_gap = float("inf")
    return abs_gap, rel_gap
