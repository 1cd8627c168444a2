"""TEST INFRASTRUCTURE (oracle): one HiGHS solve per scenario subproblem.

Stands in for the external-solver boundary of the reference,
``SPOpt.solve_one`` -> ``s._solver_plugin.solve(...)`` (``mpisppy/spopt.py:184-231``), using the
HiGHS 1.8.0 copy bundled inside scipy 1.15.3 (LP and diagonal-Hessian QP through the private
``scipy.optimize._highspy._core._Highs`` binding).  Results are returned as plain numbers: primal
x, objective (min-form, including the objective offset), and a status string.
"""
import numpy as np
from scipy.optimize._highspy import _core as _hc

INF = float("inf")


class SolveResult:
    __slots__ = ("status", "x", "obj", "row_dual", "col_dual")

    def __init__(self, status, x, obj, row_dual=None, col_dual=None):
        self.status = status
        self.x = x
        self.obj = obj
        self.row_dual = row_dual
        self.col_dual = col_dual

    @property
    def ok(self):
        return self.status == "Optimal"


def _finite(v):
    v = np.asarray(v, dtype=np.float64)
    return np.where(np.isfinite(v), v, np.where(v > 0, _hc.kHighsInf, -_hc.kHighsInf))


def solve(c, rowptr, colidx, vals, row_lo, row_hi, col_lo, col_hi, qdiag=None, offset=0.0,
          threads=1, tol=1e-10, presolve=None, do_polish=True, time_limit=None):
    """min c^T x + 1/2 x^T diag(qdiag) x + offset  s.t. row_lo <= A x <= row_hi, col_lo <= x <= col_hi.

    A is given in CSR (rowptr[m+1], colidx[nnz], vals[nnz]).
    """
    c = np.asarray(c, dtype=np.float64)
    n = c.shape[0]
    m = len(rowptr) - 1
    if qdiag is not None and np.any(np.asarray(qdiag) != 0) and n > 1000 and do_polish:
        # large prox-QPs (netdes: 2940 columns, 1470 quadratic terms): HiGHS 1.8's active-set QP
        # solver can take minutes; the interior-point oracle certifies them in seconds
        from . import ipm
        r = ipm.solve_qp(c, rowptr, colidx, vals, row_lo, row_hi, col_lo, col_hi, qdiag=qdiag, offset=offset)
        if r.ok:
            return SolveResult("Optimal", r.x, r.obj)
    h = _hc._Highs()
    h.setOptionValue("output_flag", False)
    h.setOptionValue("threads", int(threads))
    if presolve is not None:
        h.setOptionValue("presolve", presolve)
    if time_limit is not None:   # bounded CPU-baseline samples (bench.py): a cut-off solve is not counted
        h.setOptionValue("time_limit", float(max(time_limit, 0.01)))
    h.setOptionValue("primal_feasibility_tolerance", tol)
    h.setOptionValue("dual_feasibility_tolerance", tol)
    lp = _hc.HighsLp()
    lp.num_col_ = n
    lp.num_row_ = m
    lp.col_cost_ = c
    lp.col_lower_ = _finite(col_lo)
    lp.col_upper_ = _finite(col_hi)
    lp.row_lower_ = _finite(row_lo)
    lp.row_upper_ = _finite(row_hi)
    lp.offset_ = float(offset)
    mat = _hc.HighsSparseMatrix()
    mat.format_ = _hc.MatrixFormat.kRowwise
    mat.num_col_ = n
    mat.num_row_ = m
    mat.start_ = np.asarray(rowptr, dtype=np.int32)
    mat.index_ = np.asarray(colidx, dtype=np.int32)
    mat.value_ = np.asarray(vals, dtype=np.float64)
    lp.a_matrix_ = mat
    model = _hc.HighsModel()
    model.lp_ = lp
    if qdiag is not None and np.any(np.asarray(qdiag) != 0):
        qd = np.asarray(qdiag, dtype=np.float64)
        nzc = np.nonzero(qd)[0]
        hess = _hc.HighsHessian()
        hess.dim_ = n
        hess.format_ = _hc.HessianFormat.kTriangular
        start = np.zeros(n + 1, dtype=np.int32)
        for j in nzc:
            start[j + 1] = 1
        hess.start_ = np.cumsum(start).astype(np.int32)
        hess.index_ = nzc.astype(np.int32)
        hess.value_ = qd[nzc]
        model.hessian_ = hess
    h.passModel(model)
    h.run()
    st = h.modelStatusToString(h.getModelStatus())
    sol = h.getSolution()
    x = np.array(sol.col_value, dtype=np.float64)
    obj = float(h.getInfo().objective_function_value)
    rd = np.array(sol.row_dual, dtype=np.float64) if sol.dual_valid else None
    cd = np.array(sol.col_dual, dtype=np.float64) if sol.dual_valid else None
    if qdiag is not None and np.any(np.asarray(qdiag) != 0) and st != "Optimal" and do_polish and time_limit is None:
        # HiGHS 1.8's QP solver occasionally ends in "Solve error" on a prox-QP that is plainly
        # feasible and bounded (farmer cm=10 deep in a PH run, LP part solved by the same HiGHS):
        # retry with the infinite column bounds capped far outside the data (the cap must be
        # inactive at the solution), then the usual certify / polish / IPM chain; else the IPM alone
        cu = np.asarray(col_hi, dtype=np.float64)
        if not np.all(np.isfinite(cu)):
            fin_ = np.abs(np.concatenate([np.asarray(v, float)[np.isfinite(v)] for v in
                                          (col_lo, col_hi, row_lo, row_hi)] + [np.zeros(1)]))
            cap = 1e3 * max(1.0, float(fin_.max()))
            r = solve(c, rowptr, colidx, vals, row_lo, row_hi, col_lo, np.where(np.isfinite(cu), cu, cap),
                      qdiag=qdiag, offset=offset, threads=threads, tol=tol, presolve=presolve,
                      do_polish=do_polish)
            if r.ok and np.all(np.abs(r.x[~np.isfinite(cu)]) < 0.5 * cap):
                return r
        from . import ipm
        r = ipm.solve_qp(c, rowptr, colidx, vals, row_lo, row_hi, col_lo, col_hi, qdiag=qdiag, offset=offset)
        if r.ok:
            return SolveResult("Optimal", r.x, r.obj)
    if qdiag is not None and st == "Optimal" and do_polish:
        # 1. HiGHS's own point, when its duals certify it (relative KKT <= 1e-9);
        # 2. else the exact active-set polish (small subproblems: dense KKT solves);
        # 3. else the interior-point oracle (LP-dominated, degenerate prox-QPs such as sslp defeat
        #    the single-swap polish)
        ok = rd is not None and cd is not None and \
            kkt_certify(c, qdiag, rowptr, colidx, vals, row_lo, row_hi, col_lo, col_hi, x, rd, cd) <= 1e-9
        xp = x
        if not ok and n <= 400:
            xp, ok = polish(c, qdiag, rowptr, colidx, vals, row_lo, row_hi, col_lo, col_hi, x)
        if not ok:
            from . import ipm
            r = ipm.solve_qp(c, rowptr, colidx, vals, row_lo, row_hi, col_lo, col_hi, qdiag=qdiag,
                             offset=offset)
            if not r.ok:
                raise RuntimeError("oracle QP: HiGHS, the active-set polish and the IPM all failed to "
                                   "certify optimality")
            xp = r.x
        x = xp
        qd = np.asarray(qdiag, dtype=np.float64)
        obj = float(c @ x + 0.5 * np.sum(qd * x * x) + offset)
    return SolveResult(st, x, obj, rd, cd)


def kkt_certify(c, qdiag, rowptr, colidx, vals, row_lo, row_hi, col_lo, col_hi, x, row_dual, col_dual):
    """Relative KKT error of (x, duals) for the min-form QP (HiGHS sign convention: col_dual =
    c + Q x - A^T row_dual; a positive dual means the lower bound is active)."""
    c = np.asarray(c, float)
    n = c.shape[0]
    m = len(rowptr) - 1
    ax = np.zeros(m)
    aty = np.zeros(n)
    for i in range(m):
        for p in range(rowptr[i], rowptr[i + 1]):
            ax[i] += vals[p] * x[colidx[p]]
            aty[colidx[p]] += vals[p] * row_dual[i]
    q = np.zeros(n) if qdiag is None else np.asarray(qdiag, float)
    sc = 1.0 + np.abs(c).max(initial=0.0)
    stat = np.abs(c + q * x - aty - col_dual).max(initial=0.0) / sc
    xs = 1.0 + np.abs(x).max(initial=0.0)
    axs = 1.0 + np.abs(ax).max(initial=0.0)
    pr = max(np.maximum(np.asarray(col_lo) - x, x - np.asarray(col_hi)).max(initial=0.0) / xs,
             np.maximum(np.asarray(row_lo) - ax, ax - np.asarray(row_hi)).max(initial=0.0) / axs, 0.0)
    # complementarity: dual sign must match an active bound; measure |dual| * distance
    with np.errstate(invalid="ignore"):   # 0 * inf in the unselected branch of np.where
        dl = np.where(col_dual > 0, col_dual * (x - np.where(np.isfinite(col_lo), col_lo, -np.inf)), 0.0)
        du = np.where(col_dual < 0, -col_dual * (np.where(np.isfinite(col_hi), col_hi, np.inf) - x), 0.0)
        rl_ = np.where(row_dual > 0, row_dual * (ax - np.where(np.isfinite(row_lo), row_lo, -np.inf)), 0.0)
        ru_ = np.where(row_dual < 0, -row_dual * (np.where(np.isfinite(row_hi), row_hi, np.inf) - ax), 0.0)
    comp = max(np.abs(dl).max(initial=0), np.abs(du).max(initial=0), np.abs(rl_).max(initial=0),
               np.abs(ru_).max(initial=0)) / (sc * max(xs, axs))
    val = max(stat, pr, comp)
    return val if np.isfinite(val) else np.inf


def _dense(rowptr, colidx, vals, m, n):
    A = np.zeros((m, n))
    for i in range(m):
        for p in range(rowptr[i], rowptr[i + 1]):
            A[i, colidx[p]] += vals[p]
    return A


def polish(c, qdiag, rowptr, colidx, vals, row_lo, row_hi, col_lo, col_hi, x0, tol=1e-9,
           max_rounds=50):
    """Exact KKT solve on the active set of an approximate solution (primal-dual active set).

    HiGHS 1.8's QP solver stops with reduced-gradient errors of ~1e-2 on the prox-augmented
    farmer subproblems (measured: a feasible descent direction with slope -7.7e-3 remains at its
    'Optimal' point).  The reference fixtures were produced by CPLEX/Gurobi/Xpress, which solve
    these QPs to ~1e-9, so the oracle polishes: guess the active set from x0, solve the equality
    KKT system of that face exactly, then add violated / drop wrong-signed constraints until
    primal and dual feasibility hold to ``tol`` (relative).  Returns (x, ok).
    """
    c = np.asarray(c, float)
    n = c.shape[0]
    m = len(rowptr) - 1
    A = _dense(rowptr, colidx, vals, m, n)
    q = np.zeros(n) if qdiag is None else np.asarray(qdiag, float)
    rlo, rhi = np.asarray(row_lo, float), np.asarray(row_hi, float)
    clo, chi = np.asarray(col_lo, float), np.asarray(col_hi, float)
    x0 = np.asarray(x0, float)
    ax = A @ x0
    sc_r = np.maximum(1.0, np.abs(ax))
    sc_c = np.maximum(1.0, np.abs(x0))
    # active sets: +1 at upper, -1 at lower, 2 equality/fixed
    ract = np.zeros(m, int)
    cact = np.zeros(n, int)
    atol = 1e-6
    for i in range(m):
        if rlo[i] == rhi[i]:
            ract[i] = 2
        elif np.isfinite(rlo[i]) and abs(ax[i] - rlo[i]) <= atol * sc_r[i]:
            ract[i] = -1
        elif np.isfinite(rhi[i]) and abs(ax[i] - rhi[i]) <= atol * sc_r[i]:
            ract[i] = 1
    for j in range(n):
        if clo[j] == chi[j]:
            cact[j] = 2
        elif np.isfinite(clo[j]) and abs(x0[j] - clo[j]) <= atol * sc_c[j]:
            cact[j] = -1
        elif np.isfinite(chi[j]) and abs(x0[j] - chi[j]) <= atol * sc_c[j]:
            cact[j] = 1
    x = x0.copy()
    for _ in range(max_rounds):
        R = np.nonzero(ract)[0]
        C = np.nonzero(cact)[0]
        F = np.nonzero(cact == 0)[0]
        xc = np.where(cact == 1, chi, clo)
        xc = np.where(cact == 2, clo, xc)
        bR = np.where(ract[R] == 1, rhi[R], rlo[R])
        nF, nR = len(F), len(R)
        K = np.zeros((nF + nR, nF + nR))
        K[:nF, :nF] = np.diag(q[F])
        K[:nF, nF:] = -A[np.ix_(R, F)].T
        K[nF:, :nF] = A[np.ix_(R, F)]
        rhs = np.concatenate([-c[F], bR - A[np.ix_(R, C)] @ xc[C]])
        sol, *_ = np.linalg.lstsq(K, rhs, rcond=None)
        x = xc.copy()
        x[F] = sol[:nF]
        y = np.zeros(m)
        y[R] = sol[nF:]
        z = q * x + c - A.T @ y
        # primal check
        ax = A @ x
        viol_r = np.maximum(rlo - ax, ax - rhi) / np.maximum(1.0, np.abs(ax))
        viol_r[ract != 0] = 0.0
        viol_c = np.maximum(clo - x, x - chi) / np.maximum(1.0, np.abs(x))
        viol_c[cact != 0] = 0.0
        # dual sign checks (Qx + c - A^T y - z = 0; z>=0 at lower, y>=0 at row lower)
        dscale = max(1.0, float(np.max(np.abs(c))))
        bad_r = np.where(ract == -1, -y, np.where(ract == 1, y, 0.0)) / dscale
        bad_c = np.where(cact == -1, -z, np.where(cact == 1, z, 0.0)) / dscale
        zfree = np.abs(z[F]) / dscale if nF else np.zeros(0)
        worst = max(viol_r.max(initial=0), viol_c.max(initial=0), bad_r.max(initial=0),
                    bad_c.max(initial=0))
        if worst <= tol and (zfree.max(initial=0) <= 1e-7):
            return x, True
        # fix the worst offender
        cand = [(viol_r.max(initial=0), "vr"), (viol_c.max(initial=0), "vc"),
                (bad_r.max(initial=0), "br"), (bad_c.max(initial=0), "bc")]
        _, kind = max(cand)
        if kind == "vr":
            i = int(np.argmax(viol_r))
            ract[i] = -1 if ax[i] < rlo[i] else 1
        elif kind == "vc":
            j = int(np.argmax(viol_c))
            cact[j] = -1 if x[j] < clo[j] else 1
        elif kind == "br":
            ract[int(np.argmax(bad_r))] = 0
        else:
            cact[int(np.argmax(bad_c))] = 0
    return x, False
