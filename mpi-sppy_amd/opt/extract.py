"""Standard-form extraction: a model -> ``min/max c^T x + c0  s.t.  row_lo <= A x <= row_hi,
col_lo <= x <= col_hi`` in CSR, the arrays ``phg_load_batch`` takes (include/phg.h).

The reference hands each scenario's Pyomo model to a solver plugin, which writes it out for the
external solver (``spopt.py:184-231``).  Here the same model is read ONCE into standard form and
then lives in the batch.  Three sources:

* :class:`~mpisppy_amd.model.LinearModel` -- already standard form;
* any model following the duck-typed protocol below (what a modelling layer, or a test, supplies);
* a Pyomo ``ConcreteModel`` when Pyomo is importable: the active variables, the active linear
  constraints and the single active objective, through ``pyomo.repn.generate_standard_repn``.
  Pyomo is absent on the build container and on the GPU box, so this path is written against
  Pyomo's public API and is PARITY UNPINNED (never executed here); a nonlinear constraint body, or
  an objective with off-diagonal quadratic terms, raises.

The objective may carry a DIAGONAL quadratic part -- what the reference's PH puts on every scenario
at iteration >= 1: ``W_on * sum W_i x_i + prox_on * sum rho_i/2 (x_i^2 - 2 xbar_i x_i + xbar_i^2)``
(``phbase.py:724-750``, ``ProxExpr``), expanded by ``generate_standard_repn`` into linear terms plus
``rho_i/2 x_i^2``.  It is kept as ``qdiag`` (objective = c^T x + 1/2 sum_j qdiag_j x_j^2 + c0); the
plugin (``opt/phg.py``) maps it onto the C ABI's prox term (rho = qdiag, xbar = 0).

Duck-typed protocol (``extract`` checks for ``variables``):
  ``model.variables()``   -> sequence of variable objects (``.name``, ``.lb``, ``.ub`` with None = unbounded,
                             optional ``.fixed`` / ``.value``: a fixed variable gets lb = ub = value)
  ``model.constraints()`` -> sequence of rows (``.name``, ``.terms`` = [(variable, coef), ...],
                             ``.lower`` / ``.upper`` with None = unbounded, optional ``.constant`` moved
                             to the bounds)
  ``model.objective()``   -> object with ``.terms``, optional ``.constant``, ``.sense`` (1 min, -1 max),
                             optional ``.quadratic`` = [(variable, variable, coef), ...] for coef * x * y
                             (diagonal only: both the same variable)
"""
import numpy as np

from ..model import INF, LinearModel, VarData
from ..scenario_tree import ScenarioNode


class StandardForm:
    """CSR standard form of one model; ``variables`` are the source objects in column order."""

    def __init__(self, name, variables, names, c, c0, sense, rowptr, colidx, vals, row_lo, row_hi, row_names,
                 col_lo, col_hi, qdiag=None):
        self.name = name
        # objective = c^T x + 1/2 sum_j qdiag_j x_j^2 + c0 (model sense)
        self.qdiag = np.zeros(len(c)) if qdiag is None else np.asarray(qdiag, np.float64)
        self.variables = variables
        self.names = names
        self.c, self.c0, self.sense = c, c0, sense
        self.rowptr, self.colidx, self.vals = rowptr, colidx, vals
        self.row_lo, self.row_hi, self.row_names = row_lo, row_hi, row_names
        self.col_lo, self.col_hi = col_lo, col_hi
        self.col_of = {id(v): j for j, v in enumerate(variables)}

    @property
    def n(self):
        return len(self.c)

    @property
    def m(self):
        return len(self.row_lo)


def _bound(v, default):
    return default if v is None else float(v)


def _csr(rows, n):
    """rows: list of dict col -> coef -> (rowptr, colidx, vals), columns sorted in each row."""
    rowptr = np.zeros(len(rows) + 1, np.int32)
    cols, vals = [], []
    for i, d in enumerate(rows):
        for j in sorted(d):
            cols.append(j)
            vals.append(d[j])
        rowptr[i + 1] = len(cols)
    return rowptr, np.array(cols, np.int32), np.array(vals, np.float64)


def _from_linear_model(m):
    a = m.arrays()
    cols = [VarData(m, j, nm) for j, nm in enumerate(m.column_names())]
    sf = StandardForm(m.name, cols, m.column_names(), a["c"], m.obj_offset, m.sense, a["rowptr"], a["colidx"],
                      a["vals"], a["row_lo"], a["row_hi"], [r[3] for r in m._rows], a["col_lo"], a["col_hi"],
                      qdiag=getattr(m, "_qdiag", None))
    sf.col_of = {}   # LinearModel variables map by column index (VarData objects are made on demand)
    return sf


def _duck_bounds(variables):
    n = len(variables)
    lo = np.empty(n)
    hi = np.empty(n)
    for j, v in enumerate(variables):
        if getattr(v, "fixed", False):
            lo[j] = hi[j] = float(v.value)
        else:
            lo[j], hi[j] = _bound(v.lb, -INF), _bound(v.ub, INF)
    return lo, hi


def _duck_objective(ob, col, n, name):
    c = np.zeros(n)
    for v, a in ob.terms:
        c[col[id(v)]] += float(a)
    q = _qdiag(((col[id(v1)], col[id(v2)], a) for v1, v2, a in (getattr(ob, "quadratic", None) or [])), n, name)
    return c, q, float(getattr(ob, "constant", 0.0) or 0.0), int(getattr(ob, "sense", 1))


def _from_duck(model):
    variables = list(model.variables())
    col = {id(v): j for j, v in enumerate(variables)}
    n = len(variables)
    lo, hi = _duck_bounds(variables)
    rows, rlo, rhi, rnames = [], [], [], []
    for r in model.constraints():
        d = {}
        for v, a in r.terms:
            j = col[id(v)]
            d[j] = d.get(j, 0.0) + float(a)
        k = float(getattr(r, "constant", 0.0) or 0.0)
        rows.append(d)
        rlo.append(_bound(r.lower, -INF) - k)
        rhi.append(_bound(r.upper, INF) - k)
        rnames.append(getattr(r, "name", f"r{len(rows) - 1}"))
    c, q, c0, sense = _duck_objective(model.objective(), col, n, getattr(model, "name", ""))
    rp, ci, vals = _csr(rows, n)
    return StandardForm(getattr(model, "name", ""), variables, [getattr(v, "name", f"x{j}") for j, v in enumerate(variables)],
                        c, c0, sense, rp, ci, vals, np.array(rlo), np.array(rhi), rnames, lo, hi, qdiag=q)


def _qdiag(terms, n, name):
    """coef * x_j * x_k terms -> qdiag (objective 1/2 sum qdiag_j x_j^2): diagonal only."""
    q = np.zeros(n)
    for j, k, a in terms:
        if j != k:
            raise ValueError(f"model {name}: off-diagonal quadratic objective term (columns {j}, {k}); "
                             "the engine solves diagonal quadratics (PH's prox term) only")
        q[j] += 2.0 * float(a)
    return q


def _pyomo_bounds(variables):   # parity unpinned (module docstring)
    import pyomo.environ as pyo
    n = len(variables)
    lo, hi = np.empty(n), np.empty(n)
    for j, v in enumerate(variables):
        if v.fixed:
            lo[j] = hi[j] = float(pyo.value(v))
        else:
            lo[j], hi[j] = _bound(v.lb, -INF), _bound(v.ub, INF)
    return lo, hi


def _pyomo_objective(model, col, n, obj=None):   # parity unpinned (module docstring)
    import pyomo.environ as pyo
    from pyomo.repn import generate_standard_repn
    if obj is None:
        objs = list(model.component_data_objects(pyo.Objective, active=True, descend_into=True))
        if len(objs) != 1:
            raise ValueError(f"expected one active objective, found {len(objs)}")
        obj = objs[0]
    # linear, or quadratic with diagonal terms only: PH's W and prox terms (phbase.py:724-750); the
    # mutable Params (W, xbars, rho, W_on, prox_on) enter with their CURRENT values
    repn = generate_standard_repn(obj.expr, compute_values=True, quadratic=True)
    if repn.nonlinear_expr is not None:
        raise ValueError("the objective has a nonlinear part; only linear + diagonal quadratic is supported")
    c = np.zeros(n)
    for v, a in zip(repn.linear_vars, repn.linear_coefs):
        c[col[id(v)]] += float(a)
    q = _qdiag(((col[id(v1)], col[id(v2)], a) for (v1, v2), a in
                zip(repn.quadratic_vars or [], repn.quadratic_coefs or [])), n, model.name)
    return c, q, float(repn.constant), 1 if obj.sense == pyo.minimize else -1


def _from_pyomo(model):   # parity unpinned: Pyomo is not importable here (module docstring)
    import pyomo.environ as pyo
    from pyomo.repn import generate_standard_repn
    variables = list(model.component_data_objects(pyo.Var, active=True, descend_into=True))
    col = {id(v): j for j, v in enumerate(variables)}
    n = len(variables)
    lo, hi = _pyomo_bounds(variables)
    rows, rlo, rhi, rnames = [], [], [], []
    for con in model.component_data_objects(pyo.Constraint, active=True, descend_into=True):
        repn = generate_standard_repn(con.body, compute_values=True)
        if not repn.is_linear():
            raise ValueError(f"constraint {con.name}: only linear constraints are supported")
        d = {}
        for v, a in zip(repn.linear_vars, repn.linear_coefs):
            d[col[id(v)]] = d.get(col[id(v)], 0.0) + float(a)
        k = float(repn.constant)
        rows.append(d)
        rlo.append(-INF if con.lower is None else float(pyo.value(con.lower)) - k)
        rhi.append(INF if con.upper is None else float(pyo.value(con.upper)) - k)
        rnames.append(con.name)
    c, q, c0, sense = _pyomo_objective(model, col, n)
    rp, ci, vals = _csr(rows, n)
    return StandardForm(model.name, variables, [v.name for v in variables], c, c0, sense, rp, ci,
                        vals, np.array(rlo), np.array(rhi), rnames, lo, hi, qdiag=q)


def extract(model):
    """Standard form of ``model`` (LinearModel, duck-typed model, or Pyomo model)."""
    if isinstance(model, LinearModel):
        return _from_linear_model(model)
    if hasattr(model, "variables") and hasattr(model, "constraints"):
        return _from_duck(model)
    if hasattr(model, "component_data_objects"):
        return _from_pyomo(model)
    raise TypeError(f"cannot extract a standard form from {type(model).__name__}")


def objective_of(model, sf, obj=None):
    """The objective of ``model`` as it stands NOW, over ``sf``'s columns: (c, qdiag, c0, sense).

    What a solver plugin must re-read before every solve of a model the caller mutates in place:
    the reference's PH keeps ONE model per scenario and changes the mutable Params W, xbars, rho,
    W_on, prox_on between solves (``phbase.py:621-638, 716-760``), so the objective's linear part,
    diagonal and constant change while the constraint matrix does not.  ``obj`` (Pyomo only) is the
    objective ``set_objective`` was handed (``spopt.py:147-160``)."""
    if isinstance(model, LinearModel):
        q = getattr(model, "_qdiag", None)
        return (np.array(model._cost, np.float64), np.zeros(model.n) if q is None else np.asarray(q, np.float64).copy(),
                float(model.obj_offset), int(model.sense))
    if hasattr(model, "variables") and hasattr(model, "constraints"):
        return _duck_objective(model.objective(), sf.col_of, sf.n, getattr(model, "name", ""))
    if hasattr(model, "component_data_objects"):
        return _pyomo_objective(model, sf.col_of, sf.n, obj)
    raise TypeError(f"cannot read an objective from {type(model).__name__}")


def column_bounds_of(model, sf):
    """The column bounds of ``model`` as they stand NOW (a fixed variable: lo = hi = its value), over
    ``sf``'s columns -- ``_fix_nonants`` / ``_restore_nonants`` fix and free variables in place
    (``spopt.py:590-640``)."""
    if isinstance(model, LinearModel):
        return np.array(model._lo, np.float64), np.array(model._hi, np.float64)
    if hasattr(model, "variables") and hasattr(model, "constraints"):
        return _duck_bounds(sf.variables)
    if hasattr(model, "component_data_objects"):
        return _pyomo_bounds(sf.variables)
    raise TypeError(f"cannot read column bounds from {type(model).__name__}")


def to_linear_model(sf, name=None):
    """The engine's model object for a standard form (one column per source variable, in order)."""
    m = LinearModel(name or sf.name)
    for j, nm in enumerate(sf.names):
        col = m._new_col(str(nm))
        m._lo[col], m._hi[col], m._cost[col] = float(sf.col_lo[j]), float(sf.col_hi[j]), float(sf.c[j])
    for i in range(sf.m):
        d = {int(sf.colidx[q]): float(sf.vals[q]) for q in range(sf.rowptr[i], sf.rowptr[i + 1])}
        m._rows.append((d, float(sf.row_lo[i]), float(sf.row_hi[i]), str(sf.row_names[i])))
    m.sense = sf.sense
    m.obj_offset = float(sf.c0)
    m._qdiag = np.asarray(sf.qdiag, np.float64).copy()   # diagonal quadratic objective (opt/phg.py)
    return m


def as_scenario_model(model):
    """A scenario model the batch can take: LinearModel as is; otherwise its standard form as a
    LinearModel whose ``_mpisppy_node_list`` maps each node's nonant variables (source objects) to
    columns, keeping names, probabilities and the source (``_source``, ``_source_vars``) so that
    solutions can be written back (:func:`load_values`)."""
    if isinstance(model, LinearModel):
        return model
    sf = extract(model)
    lm = to_linear_model(sf, getattr(model, "name", None))
    nodes = []
    for nd in getattr(model, "_mpisppy_node_list", []):
        vl = [VarData(lm, sf.col_of[id(v)], sf.names[sf.col_of[id(v)]]) for v in nd.nonant_vardata_list]
        nodes.append(ScenarioNode(nd.name, nd.cond_prob, nd.stage, None, vl, lm, parent_name=getattr(nd, "parent_name", None)))
    if nodes:
        lm._mpisppy_node_list = nodes
    if hasattr(model, "_mpisppy_probability"):
        lm._mpisppy_probability = model._mpisppy_probability
    lm._source = model
    lm._source_vars = sf.variables
    lm._source_sf = sf        # column map for re-reading the objective / bounds (objective_of)
    return lm


def load_values(lm, x, vars_to_load=None):
    """Write column values ``x`` back into the model's variables (``load_vars``; ``vars_to_load``: only
    those source variables)."""
    lm._solution = np.asarray(x, np.float64).copy()
    src = getattr(lm, "_source_vars", None)
    if src is None:
        return
    only = None if vars_to_load is None else {id(v) for v in vars_to_load}
    for v, xv in zip(src, lm._solution):
        if only is not None and id(v) not in only:
            continue
        if hasattr(v, "set_value"):
            v.set_value(float(xv))
        else:
            v.value = float(xv)
