"""The ``phg`` solver plugin: a per-model (or per-batch) LP / QP solve through the C ABI, with the
plugin surface ``SPOpt`` uses on its solvers (``mpisppy/spopt.py:876-913`` creation, ``:150-231`` use):

* ``SolverFactory("phg")`` -> :class:`PHGSolver` (``spopt.py:884``); :func:`register_solver` adds
  names, and on import the plugin registers itself with Pyomo's ``SolverFactory`` when Pyomo is
  importable (parity unpinned: Pyomo is absent here);
* ``options`` dict (``spopt.py:171-172``): ``pdhg_eps`` (relative KKT tolerance, default 1e-9),
  ``pdhg_max_iter``, ``pdhg_check_every``, ``pdhg_layout``;
* ``solve(model, tee=False, load_solutions=True, save_results=False)`` (``:185-187``) -> a results
  object with ``.solver.status``, ``.solver.termination_condition``, ``len(.solution)``,
  ``.solution(0).status`` (``sputils.py:29-34``) and ``.Problem[0].Lower_bound / Upper_bound``
  (``spopt.py:225-230``: the PDHG dual bound and primal objective, in the model's sense);
* the persistent calls ``set_instance`` (``:933-960``), ``set_objective``, ``update_var``
  (``:625-777``: re-read at the next solve), ``load_vars`` (``:219``);
* ``solve_batch(models)``: every model of ONE sparsity pattern in one launch -- the engine's own
  path (what ``PHBase.solve_loop`` does for all local scenarios at once).

The batch needs no scenario tree for a plain solve: a model without ``_mpisppy_node_list`` gets a
one-column ROOT node whose PH terms are switched off (w_on = prox_on = 0), so the solve is the
model's own LP.  A model whose objective has a DIAGONAL quadratic part (``extract.qdiag``) -- the
reference PH's subproblem from iteration 1 on, ``f(x) + W.x + rho/2 (x - xbar)^2``
(``phbase.py:724-750``) as ``SPOpt.solve_one`` hands it to its plugin (``spopt.py:147-231``) --
is solved as the C ABI's prox-QP: the batch's nonants are the quadratic columns, rho = the
min-form diagonal, xbar = 0, W off (the linear part, W.x - rho xbar.x included, is already in c),
prox on.  A concave (min-form negative) diagonal raises.  The GPU engine is the only solver: there
is no CPU fallback (the library loads or the plugin raises).

Reported bounds (``Problem[0].Lower_bound`` of a min problem) are weak-duality certificates of the
solve's dual iterate (``phg_opts.safe_bound``), valid also at ``maxIterations``.
"""
import numpy as np

from ..engine import BatchArrays, Engine
from ..model import LinearModel, VarData
from ..scenario_tree import ScenarioNode
from .. import _lib
from .extract import as_scenario_model, load_values


class _Status:
    ok, warning, error = "ok", "warning", "error"


class _Termination:
    optimal, maxIterations, error = "optimal", "maxIterations", "error"


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
    def __init__(self, status, x):
        self.status = status
        self.x = x


class Results:
    """Pyomo-results-like object of one solve."""

    def __init__(self, st, iters, kkt, obj, bound, sense, x):
        tc = {0: _Termination.optimal, 1: _Termination.maxIterations}.get(int(st), _Termination.error)
        status = {0: _Status.ok, 1: _Status.warning}.get(int(st), _Status.error)
        self.solver = _SolverInfo(status, tc, int(iters), float(kkt))
        # bounds in the model's sense: a min problem's dual bound is the lower bound
        self.Problem = [_Problem(float(bound), float(obj), sense)]
        self.problem = self.Problem
        self._solutions = [_Solution("optimal" if st == 0 else "feasible", x)] if st in (0, 1) else []

    @property
    def solution(self):
        res = self

        class _SolList(list):
            def __call__(self, i):
                return self[i]

        return _SolList(res._solutions)


class _PluginScenario:
    """The plugin's view of one model: its standard form (attributes forwarded) with the batch's own
    tree -- the quadratic columns as ROOT nonants -- and unit probability coefficients, without
    touching the caller's model."""

    def __init__(self, lm, nodes):
        self._lm = lm
        self._mpisppy_node_list = nodes
        self._mpisppy_data = type("MpisppyData", (), {})()
        self._mpisppy_data.prob_coeff = {nd.name: 1.0 for nd in nodes}
        self._mpisppy_data.has_variable_probability = False

    def __getattr__(self, k):
        return getattr(self._lm, k)


class PHGSolver:
    """Persistent-style plugin over libphg (one engine per instance, rebuilt when the model or the
    batch shape changes)."""

    name = "phg"

    def __init__(self, **kwds):
        self.options = dict(kwds.get("options", {}))
        self._models = None
        self._lms = None
        self._engine = None
        self._dirty = True

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
        self._dirty = True

    def update_var(self, var=None):
        self._dirty = True

    def solve(self, model=None, tee=False, load_solutions=True, save_results=False, **kwds):
        if model is not None and (self._models is None or len(self._models) != 1 or self._models[0] is not model):
            self._set([model])
        if self._models is None:
            raise RuntimeError("PHGSolver.solve: no model (call set_instance or pass one)")
        return self._solve(tee, load_solutions)[0]

    def solve_batch(self, models, tee=False, load_solutions=True):
        self._set(list(models))
        return self._solve(tee, load_solutions)

    def load_vars(self, vars_to_load=None):
        if self._engine is None:
            raise RuntimeError("PHGSolver.load_vars: nothing solved yet")
        self._load()

    def close(self):
        if self._engine is not None:
            self._engine.close()
            self._engine = None

    # ------------------------------------------------------------------ internals
    def _set(self, models):
        self._models = models
        self._dirty = True

    def _build(self):
        import torch
        lms = []
        for md in self._models:
            lm = as_scenario_model(md)
            if not isinstance(lm, LinearModel) or lm.n == 0:
                raise ValueError("PHGSolver: empty model")
            lms.append(lm)
        S = len(lms)
        # min-form diagonal of each model's quadratic objective; the batch's nonants are the columns
        # quadratic in any model (one shared column list), else the dummy column 0 with PH terms off
        qmin = []
        for lm in lms:
            q = getattr(lm, "_qdiag", None)
            q = np.zeros(lm.n) if q is None else lm.sense * np.asarray(q, np.float64)
            if (q < 0).any():
                raise ValueError(f"PHGSolver: model {lm.name}: the quadratic objective is not convex "
                                 "(min-form diagonal < 0)")
            qmin.append(q)
        qcols = sorted(set(int(j) for q in qmin for j in np.nonzero(q)[0]))
        self._quadratic = bool(qcols)
        cols = qcols or [0]
        views = []
        for lm in lms:
            names = lm.column_names()
            nodes = [ScenarioNode("ROOT", 1.0, 1, None, [VarData(lm, j, names[j]) for j in cols], lm)]
            views.append(_PluginScenario(lm, nodes))
        batch = BatchArrays(views, ["ROOT"], [1.0 / S] * S, 0, S, 1)
        if self._engine is not None:
            self._engine.close()
        dev = torch.cuda.current_device()
        self._engine = Engine(batch, device=dev, layout=self.options.get("pdhg_layout", "auto"))
        if self._quadratic:
            # prox term rho/2 (x - xbar)^2 with xbar = 0: exactly the diagonal quadratic
            self._engine.set(_lib.F_RHO, np.stack([q[cols] for q in qmin]).ravel())
            self._engine.set(_lib.F_XBAR, np.zeros(len(cols)))
        self._lms = lms
        self._dirty = False

    def _solve(self, tee, load_solutions):
        if self._dirty or self._engine is None:
            self._build()
        eng = self._engine
        eng.solve(0, 1 if self._quadratic else 0, eps=float(self.options.get("pdhg_eps", 1e-9)),
                  max_iter=int(self.options.get("pdhg_max_iter", 200000)),
                  check_every=int(self.options.get("pdhg_check_every", 32)), warm_start=0, safe_bound=True)
        eng.sync()
        st = eng.get_i32(_lib.I_STATUS)
        it = eng.get_i32(_lib.I_ITERS)
        kkt = eng.get(_lib.F_KKT)
        obj = eng.get(_lib.F_OBJ)
        bnd = eng.get(_lib.F_BOUND)
        X = eng.get(_lib.F_X).reshape(eng.S, -1)
        sense = self._lms[0].sense
        out = [Results(st[s], it[s], kkt[s], obj[s], bnd[s], sense, X[s]) for s in range(eng.S)]
        if tee:
            for s, r in enumerate(out):
                print(f"[phg] {getattr(self._lms[s], 'name', s)}: {r.solver.termination_condition} "
                      f"obj={r.Problem[0].Upper_bound if sense == 1 else r.Problem[0].Lower_bound} "
                      f"iters={r.solver.iterations} kkt={r.solver.kkt:.2e}")
        if load_solutions:
            self._load(X)
        return out

    def _load(self, X=None):
        if X is None:
            X = self._engine.get(_lib.F_X).reshape(self._engine.S, -1)
        for lm, x in zip(self._lms, X):
            load_values(lm, x)


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
