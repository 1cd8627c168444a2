"""The ``phg`` solver plugin: LP / diagonal-QP solves through the C ABI with the plugin surface
``SPOpt`` uses on its solvers (``mpisppy/spopt.py:876-913`` creation, ``:99-247`` use):

* ``SolverFactory("phg")`` -> :class:`PHGSolver` (``spopt.py:884``, one plugin per subproblem);
  :func:`register_solver` adds names, and on import the plugin registers itself with Pyomo's
  ``SolverFactory`` when Pyomo is importable (parity unpinned: Pyomo is absent here);
* ``options`` dict (``spopt.py:171-172``): ``pdhg_eps`` (relative KKT tolerance, default 1e-9),
  ``pdhg_max_iter``, ``pdhg_check_every``, ``pdhg_layout``, ``pdhg_warm_start`` (default on: a
  solve starts from the plugin's previous primal / dual solution, as a persistent CPU solver does);
* ``solve(model, tee=False, load_solutions=True, save_results=True)`` (``:185-187``) -> a results
  object with ``.solver.status``, ``.solver.termination_condition``, ``len(.solution)``,
  ``.solution(0).status`` (``sputils.py:29-34``), ``.solution(0).variable`` (name -> {"Value": v},
  what Pyomo's ``ModelSolutions.load_from`` reads, ``spopt.py:221``) and
  ``.Problem[0].Lower_bound / Upper_bound`` (``:225-230``: the dual bound and primal objective in
  the model's sense);
* the persistent calls ``set_instance`` (``:933-960``), ``set_objective`` (``:147-160``),
  ``update_var`` (``:590-640``), ``load_vars`` (``:219``).  With Pyomo importable the class derives
  from Pyomo's ``PersistentSolver``, so ``sputils.is_persistent`` (``sputils.py:384-386``) sends the
  reference's ``solve_one`` down its ``set_objective`` / ``load_vars`` branch; :func:`is_persistent`
  is the same test here;
* ``solve_batch(models)``: every model of ONE sparsity pattern in one launch.

**Models mutated in place.** The reference builds each scenario model ONCE and changes its mutable
Params (W, xbars, rho, W_on, prox_on) between iterations (``phbase.py:621-638, 716-760``); it then
calls ``solve(s, load_solutions=False)`` on the SAME object every iteration and, for a
non-persistent plugin, never calls ``set_objective``.  So every ``solve`` re-reads the objective
(linear part, diagonal, constant: ``extract.objective_of``) and the column bounds
(``extract.column_bounds_of``: ``_fix_nonants`` fixes variables in place) -- the matrix is extracted
once per model.  ONE engine per plugin is kept and reused: it holds the matrix, the bounds and the
first extraction's cost ``c0``, with EVERY column a plugin-private nonant, so a later objective
``c + 1/2 sum q_j x_j^2`` enters as the C ABI's PH terms: W = c - c0 (min form), rho = q, xbar = 0,
both terms on -- ``c0 + W + rho (x - 0)`` is ``c``, the diagonal is ``q``, exactly.  The constant's
change is added to the objective and the bound on the host.  Only a change of the column bounds
(or the sense) reloads the engine (``rebuilds`` counts the loads).

A concave (min-form negative) diagonal raises.  The GPU engine is the only solver: there is no CPU
fallback (the library loads or the plugin raises).  Reported bounds are weak-duality certificates
of the solve's dual iterate for every solve (``phg_opts.safe_bound`` = 2): never on the wrong side
of the optimum, also at ``maxIterations`` (a converged solve's own dual objective can sit
eps (1 + |p| + |d|) above it).
"""
import os

import numpy as np

from ..engine import BatchArrays, Engine
from ..model import LinearModel, VarData
from ..scenario_tree import ScenarioNode
from .. import _lib
from .extract import as_scenario_model, column_bounds_of, load_values, objective_of

try:   # pragma: no cover -- Pyomo is not importable on the build container / GPU box
    from pyomo.solvers.plugins.solvers.persistent_solver import PersistentSolver as _PersistentBase
    from pyomo.opt import SolutionStatus as _SolS, SolverStatus as _SolverS, TerminationCondition as _TC
    _PYOMO = True
except Exception:
    _PYOMO = False

    class _PersistentBase:
        """Stand-in for Pyomo's ``PersistentSolver`` (absent here): the type ``is_persistent`` tests."""

    class _SolverS:
        ok, warning, error = "ok", "warning", "error"

    class _TC:
        optimal, maxIterations, error = "optimal", "maxIterations", "error"

    class _SolS:
        optimal, feasible = "optimal", "feasible"


def is_persistent(solver):
    """``sputils.is_persistent`` (``sputils.py:384-386``): an instance of (Pyomo's) PersistentSolver."""
    return isinstance(solver, _PersistentBase)


class _SolverInfo:
    def __init__(self, status, tc, iters, kkt):
        self.status = status
        self.termination_condition = tc
        self.iterations = iters
        self.kkt = kkt


class _Problem:
    def __init__(self, lb, ub, sense):
        self.Lower_bound, self.Upper_bound = (lb, ub) if sense == 1 else (ub, lb)
        self.lower_bound, self.upper_bound = self.Lower_bound, self.Upper_bound


class _Solution:
    def __init__(self, status, x, names):
        self.status = status
        self.x = x
        # Pyomo's results layout: variable label -> {"Value": v} (ModelSolutions.load_from by name)
        self.variable = {nm: {"Value": float(v)} for nm, v in zip(names, x)}


class Results:
    """Pyomo-results-like object of one solve."""

    def __init__(self, st, iters, kkt, obj, bound, sense, x, names):
        tc = {0: _TC.optimal, 1: _TC.maxIterations}.get(int(st), _TC.error)
        status = {0: _SolverS.ok, 1: _SolverS.warning}.get(int(st), _SolverS.error)
        self.solver = _SolverInfo(status, tc, int(iters), float(kkt))
        # bounds in the model's sense: a min problem's dual bound is the lower bound
        self.Problem = [_Problem(float(bound), float(obj), sense)]
        self.problem = self.Problem
        self._solutions = ([_Solution(_SolS.optimal if st == 0 else _SolS.feasible, x, names)]
                           if st in (0, 1) else [])

    @property
    def solution(self):
        res = self

        class _SolList(list):
            def __call__(self, i):
                return self[i]

        return _SolList(res._solutions)


class _PluginScenario:
    """The plugin's view of one model: its standard form (attributes forwarded) with the plugin's own
    tree -- every column a ROOT nonant -- and unit probability coefficients, without touching the
    caller's model."""

    def __init__(self, lm, nodes):
        self._lm = lm
        self._mpisppy_node_list = nodes
        self._mpisppy_data = type("MpisppyData", (), {})()
        self._mpisppy_data.prob_coeff = {nd.name: 1.0 for nd in nodes}
        self._mpisppy_data.has_variable_probability = False

    def __getattr__(self, k):
        return getattr(self._lm, k)


class PHGSolver(_PersistentBase):
    """Persistent-style plugin over libphg: one engine per instance, built at the first solve of a
    model (or batch) and reused by every later solve of the same model objects."""

    name = "phg"

    def __init__(self, **kwds):
        if _PYOMO:   # pragma: no cover -- parity unpinned (Pyomo absent)
            _PersistentBase.__init__(self, type="phg")
        self.options = dict(kwds.get("options", {}))
        self._models = None
        self._lms = None
        self._engine = None
        self._pending_obj = None
        self._X = None
        self.rebuilds = 0     # engine loads (matrix + bounds); a PH run on one model needs one
        self.bound_updates = 0   # column-bound changes applied to the loaded engine (no reload)
        self.solves = 0
        self.pdhg_iterations = 0   # PDHG iterations over all solves (diagnostic)

    # ------------------------------------------------------------------ plugin surface
    def available(self, exception_flag=False):
        try:
            _lib.load()
            return True
        except Exception:
            if exception_flag:
                raise
            return False

    def set_instance(self, model, **kwds):
        self._set([model])

    def set_objective(self, obj=None):
        """``spopt.py:147-160``: the objective is re-read at the next solve anyway; a Pyomo objective
        handed here is the one read."""
        self._pending_obj = obj

    def update_var(self, var=None):
        """``spopt.py:590-640`` (``_fix_nonants`` / ``_restore_nonants``): bounds are re-read at the
        next solve."""

    def solve(self, model=None, tee=False, load_solutions=True, save_results=True, **kwds):
        if model is not None and (self._models is None or len(self._models) != 1 or self._models[0] is not model):
            self._set([model])
        if self._models is None:
            raise RuntimeError("PHGSolver.solve: no model (call set_instance or pass one)")
        return self._solve(tee, load_solutions)[0]

    def solve_batch(self, models, tee=False, load_solutions=True):
        models = list(models)
        if self._models is None or len(self._models) != len(models) or any(
                a is not b for a, b in zip(self._models, models)):
            self._set(models)
        return self._solve(tee, load_solutions)

    def load_vars(self, vars_to_load=None):
        """``spopt.py:219``: the last solve's values into the model's variables (all, or the given
        ones)."""
        if self._engine is None or self._X is None:
            raise RuntimeError("PHGSolver.load_vars: nothing solved yet")
        self._load(self._X, vars_to_load)

    def close(self):
        if self._engine is not None:
            self._engine.close()
            self._engine = None

    # ------------------------------------------------------------------ internals
    def _set(self, models):
        self._models = models
        self._lms = None          # new model objects: extract their standard forms at the next solve
        self._X = None

    def _extract(self):
        lms = []
        for md in self._models:
            lm = as_scenario_model(md)
            if not isinstance(lm, LinearModel) or lm.n == 0:
                raise ValueError("PHGSolver: empty model")
            lms.append(lm)
        self._lms = lms
        self._sfs = [getattr(lm, "_source_sf", None) for lm in lms]
        self.close()

    def _current(self):
        """(c, q, c0, sense, lo, hi) of every model as it stands now (the re-read)."""
        out = []
        for md, lm, sf in zip(self._models, self._lms, self._sfs):
            src = lm if sf is None else md
            c, q, c0, sense = objective_of(src, sf, self._pending_obj if len(self._models) == 1 else None)
            lo, hi = column_bounds_of(src, sf)
            out.append((c, q, c0, sense, lo, hi))
        self._pending_obj = None
        return out

    def _build(self, cur):
        """Load the engine on the models' matrix with the CURRENT bounds; every column is a nonant
        of the plugin's ROOT node, so later objectives enter as W / rho (module docstring)."""
        import torch
        views = []
        for lm, sf, (c, q, c0, sense, lo, hi) in zip(self._lms, self._sfs, cur):
            if sf is not None:             # the plugin's own copy: base cost and bounds = the current ones
                lm._cost = list(c)         # (a LinearModel handed in directly already holds them)
                lm.obj_offset, lm.sense = c0, sense
                lm._lo, lm._hi = list(lo), list(hi)
            names = lm.column_names()
            nodes = [ScenarioNode("ROOT", 1.0, 1, None, [VarData(lm, j, names[j]) for j in range(lm.n)], lm)]
            views.append(_PluginScenario(lm, nodes))
        S = len(views)
        batch = BatchArrays(views, ["ROOT"], [1.0 / S] * S, 0, S, 1)
        self.close()
        dev = torch.cuda.current_device()
        self._engine = Engine(batch, device=dev, layout=self.options.get("pdhg_layout", "auto"))
        self._engine.set(_lib.F_XBAR, np.zeros(self._lms[0].n))
        self._base = [(c.copy(), c0, sense, lo.copy(), hi.copy()) for c, q, c0, sense, lo, hi in cur]
        self._warm = False
        self._sent_w = self._sent_rho = None
        self.rebuilds += 1

    def _solve(self, tee, load_solutions):
        if self._lms is None:
            self._extract()
        cur = self._current()
        for (c, q, c0, sense, lo, hi) in cur:
            if (sense * q < 0).any():
                raise ValueError("PHGSolver: the quadratic objective is not convex (min-form diagonal < 0)")
        if self._engine is None or any(b[2] != k[3] for b, k in zip(self._base, cur)):
            self._build(cur)
        elif any(not np.array_equal(b[3], k[4]) or not np.array_equal(b[4], k[5]) for b, k in zip(self._base, cur)):
            # fixed / freed variables (spopt.py:590-640): the bounds change on the device (phg_set_col_bounds),
            # the engine -- matrix, scaling, layout, warm start -- stays
            self._engine.set_col_bounds(np.stack([k[4] for k in cur]), np.stack([k[5] for k in cur]))
            self._base = [(b[0], b[1], b[2], k[4].copy(), k[5].copy()) for b, k in zip(self._base, cur)]
            self.bound_updates += 1
        eng = self._engine
        # the objective now, as PH terms on the loaded base cost (min form): W = c - c0, rho = q
        # (each upload only when it changed: PH's rho is fixed, W moves every iteration)
        w = np.concatenate([sense * (c - b[0]) for (c, q, c0, sense, lo, hi), b in zip(cur, self._base)])
        r = np.concatenate([sense * q for (c, q, c0, sense, lo, hi) in cur])
        if self._sent_w is None or not np.array_equal(w, self._sent_w):
            eng.set(_lib.F_W, w)
            self._sent_w = w
        if self._sent_rho is None or not np.array_equal(r, self._sent_rho):
            eng.set(_lib.F_RHO, r)
            self._sent_rho = r
        # warm start from the previous solution (bit 0) and its primal weight (bit 1, as the batched PH)
        ws = self.options.get("pdhg_warm_start", True)
        warm = (int(os.environ.get("PHG_PLUGIN_WARM", "3")) if ws is True else int(ws)) if self._warm else 0
        eng.solve(1, 1, eps=float(self.options.get("pdhg_eps", 1e-9)),
                  max_iter=int(self.options.get("pdhg_max_iter", 200000)),
                  check_every=int(self.options.get("pdhg_check_every", 32)), warm_start=warm, safe_bound=2)
        st, it, kkt, obj, bnd, X = eng.results()     # one synchronisation (phg_solve_results)
        self._warm = True
        self.solves += 1
        self.pdhg_iterations += int(it.sum())
        self._X = X
        out = []
        for s, ((c, q, c0, sense, lo, hi), b) in enumerate(zip(cur, self._base)):
            dk = c0 - b[1]            # the objective constant's change since the load (model sense)
            out.append(Results(st[s], it[s], kkt[s], obj[s] + dk, bnd[s] + dk, sense, X[s],
                               self._lms[s].column_names()))
        if tee:
            for s, r in enumerate(out):
                print(f"[phg] {getattr(self._lms[s], 'name', s)}: {r.solver.termination_condition} "
                      f"obj={r.Problem[0].Upper_bound if cur[s][3] == 1 else r.Problem[0].Lower_bound} "
                      f"iters={r.solver.iterations} kkt={r.solver.kkt:.2e}")
        if load_solutions:
            self._load(X)
        return out

    def _load(self, X, vars_to_load=None):
        for lm, x in zip(self._lms, X):
            load_values(lm, x, vars_to_load)


_REGISTRY = {"phg": PHGSolver}


def register_solver(name, cls):
    _REGISTRY[name] = cls
    return cls


def SolverFactory(name, **kwds):
    """``pyomo.opt.SolverFactory`` stand-in for the engine's solvers (``spopt.py:884``)."""
    if name not in _REGISTRY:
        raise ValueError(f"unknown solver {name!r} (known: {sorted(_REGISTRY)})")
    return _REGISTRY[name](**kwds)


try:   # pragma: no cover -- Pyomo is not importable on the build container / GPU box
    from pyomo.opt import SolverFactory as _PyomoSolverFactory
    _PyomoSolverFactory.register("phg", doc="batched PDHG on MI355X (mpisppy_amd)")(PHGSolver)
except Exception:
    pass
