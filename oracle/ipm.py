"""TEST INFRASTRUCTURE (oracle): primal-dual interior-point method for the PH subproblems.

    min c^T x + 1/2 x^T diag(q) x   s.t.  row_lo <= A x <= row_hi,  col_lo <= x <= col_hi

Mehrotra predictor-corrector on the bound-split form: every finite bound gets a slack and a dual,
range / inequality rows get a row variable w (A x - w = 0, row_lo <= w <= row_hi), equality rows
stay equalities.  Newton steps use the normal equations A (Q + D)^-1 A^T, dense Cholesky (the
subproblems here have m <= a few thousand).  Used where HiGHS 1.8's QP solver plus the active-set
polish of ``oracle.highs`` cannot certify optimality (LP-dominated prox-QPs such as sslp: many
degenerate bounds, few quadratic terms).  Converges to a relative KKT error ~1e-11.
"""
import numpy as np
import scipy.linalg as sla
import scipy.sparse as sp


class IpmResult:
    def __init__(self, x, obj, ok, iters, kkt):
        self.x, self.obj, self.ok, self.iters, self.kkt = x, obj, ok, iters, kkt


def solve_qp(c, rowptr, colidx, vals, row_lo, row_hi, col_lo, col_hi, qdiag=None, offset=0.0,
             tol=1e-10, max_iter=200):
    c = np.asarray(c, float)
    n = c.shape[0]
    m = len(rowptr) - 1
    A = sp.csr_matrix((np.asarray(vals, float), np.asarray(colidx), np.asarray(rowptr)), shape=(m, n))
    q = np.zeros(n) if qdiag is None else np.asarray(qdiag, float)
    rl, ru = np.asarray(row_lo, float), np.asarray(row_hi, float)
    cl, cu = np.asarray(col_lo, float), np.asarray(col_hi, float)
    # fixed columns are substituted out
    fixed = np.isfinite(cl) & np.isfinite(cu) & (cl == cu)
    xfix = np.where(fixed, cl, 0.0)
    keep = ~fixed
    shift = A @ xfix
    A = A[:, keep]
    cK, qK, clK, cuK = c[keep], q[keep], cl[keep], cu[keep]
    rl, ru = rl - shift, ru - shift
    eq = np.isfinite(rl) & np.isfinite(ru) & (rl == ru)
    ineq = ~eq
    nI = int(ineq.sum())
    # z = (x, w): A x - E w = b, with E selecting the inequality rows
    E = sp.csr_matrix((np.ones(nI), (np.nonzero(ineq)[0], np.arange(nI))), shape=(m, nI))
    M = sp.hstack([A, -E]).tocsr()
    b = np.where(eq, rl, 0.0)
    nz = A.shape[1] + nI
    cz = np.concatenate([cK, np.zeros(nI)])
    qz = np.concatenate([qK, np.zeros(nI)])
    lz = np.concatenate([clK, rl[ineq]])
    uz = np.concatenate([cuK, ru[ineq]])
    hl, hu = np.isfinite(lz), np.isfinite(uz)
    # starting point: inside the bounds
    z = np.zeros(nz)
    z = np.where(hl & hu, 0.5 * (lz + uz), z)
    z = np.where(hl & ~hu, np.maximum(z, lz + 1.0), z)
    z = np.where(~hl & hu, np.minimum(z, uz - 1.0), z)
    sl = np.where(hl, np.maximum(z - lz, 1.0), 0.0)
    su = np.where(hu, np.maximum(uz - z, 1.0), 0.0)
    vl = np.where(hl, 1.0, 0.0)
    vu = np.where(hu, 1.0, 0.0)
    lam = np.zeros(m)
    bn = 1.0 + np.linalg.norm(b) + np.linalg.norm(np.where(hl, lz, 0)) + np.linalg.norm(np.where(hu, uz, 0))
    cn = 1.0 + np.linalg.norm(cz)
    reg = 1e-12
    ok = False
    kkt = np.inf
    for it in range(max_iter):
        rd = qz * z + cz - M.T @ lam - vl + vu                 # dual residual
        rp = M @ z - b                                         # primal residual
        rbl = np.where(hl, z - lz - sl, 0.0)
        rbu = np.where(hu, uz - z - su, 0.0)
        nb = hl.sum() + hu.sum()
        mu = (sl @ vl + su @ vu) / max(nb, 1)
        pobj = cz @ z + 0.5 * qz @ (z * z)
        kkt = max(np.linalg.norm(rp) / bn, np.linalg.norm(rd) / cn, mu / (1.0 + abs(pobj)))
        if kkt < tol:
            ok = True
            break
        if not np.isfinite(kkt):
            break
        with np.errstate(divide="ignore", invalid="ignore"):
            dl = np.where(hl, vl / np.maximum(np.where(hl, sl, 1.0), 1e-150), 0.0)
            du = np.where(hu, vu / np.maximum(np.where(hu, su, 1.0), 1e-150), 0.0)
        H = qz + dl + du + reg
        Hi = 1.0 / H
        N = (M.multiply(Hi) @ M.T).toarray()
        N[np.diag_indices_from(N)] += 1e-14 * (1.0 + np.abs(np.diag(N)).max())
        try:
            fac = sla.cho_factor(N, lower=True, check_finite=False)
            solveN = lambda r: sla.cho_solve(fac, r, check_finite=False)
        except np.linalg.LinAlgError:
            lu = sla.lu_factor(N, check_finite=False)
            solveN = lambda r: sla.lu_solve(lu, r, check_finite=False)

        def newton(rcl, rcu):
            # complementarity targets: sl vl = rcl-part, su vu = rcu-part
            with np.errstate(divide="ignore", invalid="ignore"):
                gl = np.where(hl, (rcl - vl * rbl) / np.where(hl, sl, 1.0), 0.0)
                gu = np.where(hu, (rcu - vu * rbu) / np.where(hu, su, 1.0), 0.0)
            r1 = -rd + gl - gu
            dlam = solveN(-rp - M @ (Hi * r1))
            dz = Hi * (r1 + M.T @ dlam)
            dsl = np.where(hl, dz + rbl, 0.0)
            dsu = np.where(hu, -dz + rbu, 0.0)
            with np.errstate(divide="ignore", invalid="ignore"):
                dvl = np.where(hl, (rcl - vl * dsl) / np.where(hl, sl, 1.0), 0.0)
                dvu = np.where(hu, (rcu - vu * dsu) / np.where(hu, su, 1.0), 0.0)
            return dz, dlam, dsl, dsu, dvl, dvu

        def steplen(s, ds, mask):
            neg = mask & (ds < 0)
            return min(1.0, float(np.min(-s[neg] / ds[neg]))) if neg.any() else 1.0

        # predictor
        dz, dlam, dsl, dsu, dvl, dvu = newton(np.where(hl, -sl * vl, 0.0), np.where(hu, -su * vu, 0.0))
        ap = min(steplen(sl, dsl, hl), steplen(su, dsu, hu))
        ad = min(steplen(vl, dvl, hl), steplen(vu, dvu, hu))
        mu_aff = ((sl + ap * dsl) @ (vl + ad * dvl) + (su + ap * dsu) @ (vu + ad * dvu)) / max(nb, 1)
        sigma = (mu_aff / mu) ** 3 if mu > 0 else 0.0
        # corrector
        rcl = np.where(hl, sigma * mu - sl * vl - dsl * dvl, 0.0)
        rcu = np.where(hu, sigma * mu - su * vu - dsu * dvu, 0.0)
        dz, dlam, dsl, dsu, dvl, dvu = newton(rcl, rcu)
        ap = 0.995 * min(steplen(sl, dsl, hl), steplen(su, dsu, hu))
        ad = 0.995 * min(steplen(vl, dvl, hl), steplen(vu, dvu, hu))
        ap, ad = min(ap, 1.0), min(ad, 1.0)
        z += ap * dz
        sl += ap * dsl
        su += ap * dsu
        lam += ad * dlam
        vl += ad * dvl
        vu += ad * dvu
    ok = ok or kkt < 1e-9
    x = xfix.copy()
    x[keep] = z[:A.shape[1]]
    obj = float(c @ x + 0.5 * q @ (x * x) + offset)
    return IpmResult(x, obj, ok, it, kkt)
