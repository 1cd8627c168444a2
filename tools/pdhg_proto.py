"""Design prototype (NOT the product, NOT the oracle): batched restarted PDHG for scenario LP/QPs,
vectorised over scenarios with numpy/scipy.sparse.  Used to tune the algorithm (scaling, restarts,
step sizes, tolerances) on CPU before writing it as the gfx950 kernel in
``mpi-sppy_amd/csrc/pdhg.hip``.

Per scenario s:  min c^T x + 1/2 x^T diag(q) x   s.t.  rl <= A x <= ru,  cl <= x <= cu.
"""
import numpy as np
import scipy.sparse as sp


class Batch:
    def __init__(self, scen_arrays):
        """scen_arrays: list of dicts (c,rowptr,colidx,vals,row_lo,row_hi,col_lo,col_hi)."""
        self.S = len(scen_arrays)
        blocks = []
        self.n = np.array([len(a["c"]) for a in scen_arrays])
        self.m = np.array([len(a["rowptr"]) - 1 for a in scen_arrays])
        for a in scen_arrays:
            A = sp.csr_matrix((a["vals"], a["colidx"], a["rowptr"]),
                              shape=(len(a["rowptr"]) - 1, len(a["c"])))
            blocks.append(A)
        self.A = sp.block_diag(blocks, format="csr")
        self.cat = lambda key: np.concatenate([a[key] for a in scen_arrays])
        self.c = self.cat("c")
        self.rl, self.ru = self.cat("row_lo"), self.cat("row_hi")
        self.cl, self.cu = self.cat("col_lo"), self.cat("col_hi")
        self.sc = np.repeat(np.arange(self.S), self.n)     # scenario id per column
        self.sr = np.repeat(np.arange(self.S), self.m)     # scenario id per row


def seg_sum(v, sid, S):
    return np.bincount(sid, weights=v, minlength=S)


def seg_max(v, sid, S):
    out = np.zeros(S)
    np.maximum.at(out, sid, v)
    return out


class PDHG:
    def __init__(self, b, ruiz_iters=10, pock=True, eps=1e-9, check_every=64,
                 max_iter=200000, verbose=False):
        self.b = b
        S = b.S
        A = b.A.tocsr().astype(float)
        # --- Ruiz equilibration + Pock-Chambolle (alpha=1) ------------------------------------
        dr = np.ones(A.shape[0])
        dc = np.ones(A.shape[1])
        for _ in range(ruiz_iters):
            Aa = abs(A)
            rmax = Aa.max(axis=1).toarray().ravel()
            cmax = Aa.max(axis=0).toarray().ravel()
            rs = 1.0 / np.sqrt(np.where(rmax > 0, rmax, 1.0))
            cs = 1.0 / np.sqrt(np.where(cmax > 0, cmax, 1.0))
            A = sp.diags(rs) @ A @ sp.diags(cs)
            dr *= rs
            dc *= cs
        if pock:
            Aa = abs(A)
            rs = 1.0 / np.sqrt(np.maximum(np.asarray(Aa.sum(axis=1)).ravel(), 1e-300))
            cs = 1.0 / np.sqrt(np.maximum(np.asarray(Aa.sum(axis=0)).ravel(), 1e-300))
            A = sp.diags(rs) @ A @ sp.diags(cs)
            dr *= rs
            dc *= cs
        self.A = A.tocsr()
        self.AT = self.A.T.tocsr()
        self.dr, self.dc = dr, dc
        # spectral norm per scenario by power iteration
        v = np.ones(A.shape[1])
        for _ in range(60):
            w = self.AT @ (self.A @ v)
            nrm = np.sqrt(seg_sum(w * w, b.sc, S))
            v = w / np.maximum(nrm[b.sc], 1e-300)
        w = self.A @ v
        self.anorm = np.sqrt(np.sqrt(seg_sum((self.AT @ w) ** 2, b.sc, S)))
        self.eps = eps
        self.check_every = check_every
        self.max_iter = max_iter
        self.verbose = verbose

    def solve(self, c, q, x0=None, y0=None, omega0=None):
        """Solve all scenarios; c, q are unscaled (length total n).  Returns x, y (unscaled),
        iterations per scenario."""
        b = self.b
        S = b.S
        dc, dr = self.dc, self.dr
        cs = c * dc
        qs = q * dc * dc
        cl = b.cl / dc
        cu = b.cu / dc
        rl = b.rl * dr
        ru = b.ru * dr
        A, AT = self.A, self.AT
        x = np.zeros_like(cs) if x0 is None else np.clip(x0 / dc, cl, cu)
        y = np.zeros(A.shape[0]) if y0 is None else y0 / dr
        eta = 0.998 / self.anorm
        # primal weight init: ||c|| / ||b||
        cn = np.sqrt(seg_sum(cs * cs, b.sc, S))
        bf = np.where(np.isfinite(rl), rl, 0.0) ** 2 + np.where(np.isfinite(ru), ru, 0.0) ** 2
        bn = np.sqrt(seg_sum(bf, b.sr, S))
        omega = np.where((cn > 1e-10) & (bn > 1e-10), cn / np.maximum(bn, 1e-300), 1.0) \
            if omega0 is None else omega0.copy()
        done = np.zeros(S, bool)
        iters = np.zeros(S, int)
        # restart bookkeeping
        xs, ys = x.copy(), y.copy()           # last restart point
        xa, ya = np.zeros_like(x), np.zeros_like(y)
        na = np.zeros(S)                      # number averaged
        kkt_restart = self.kkt(x, y, cs, qs, cl, cu, rl, ru, omega) if getattr(self, "init_kkt", False) else None
        kkt_prev_cand = np.full(S, np.inf)
        since = np.zeros(S, int)
        total = 0
        Ax = A @ x
        ATy = AT @ y
        while total < self.max_iter and not done.all():
            act_c = ~done[b.sc]
            act_r = ~done[b.sr]
            tau = (eta / omega)[b.sc]
            sig = (eta * omega)[b.sr]
            for _ in range(self.check_every):
                xn = (x - tau * (cs - ATy)) / (1.0 + tau * qs)
                xn = np.clip(xn, cl, cu)
                xn = np.where(act_c, xn, x)
                Axn = A @ xn
                g = y - sig * (2.0 * Axn - Ax)
                yn = np.maximum(g + sig * rl, 0.0) + np.minimum(g + sig * ru, 0.0)
                yn = np.where(act_r, yn, y)
                x, y, Ax = xn, yn, Axn
                ATy = AT @ y
                xa += np.where(act_c, x, 0.0)
                ya += np.where(act_r, y, 0.0)
                na += ~done
            total += self.check_every
            iters += self.check_every * (~done)
            since += self.check_every * (~done)
            # KKT of current and average
            xav = xa / np.maximum(na, 1)[b.sc]
            yav = ya / np.maximum(na, 1)[b.sr]
            k_cur = self.kkt(x, y, cs, qs, cl, cu, rl, ru, omega)
            k_avg = self.kkt(xav, yav, cs, qs, cl, cu, rl, ru, omega)
            use_avg = k_avg < k_cur
            cand = np.where(use_avg, k_avg, k_cur)
            if kkt_restart is None:
                kkt_restart = cand.copy()
            # termination test on unscaled relative KKT
            rel = self.rel_kkt(x, y, cs, qs, cl, cu, rl, ru)
            newly = (rel < self.eps) & ~done
            done |= newly
            # restart decision
            restart = ((cand <= 0.2 * kkt_restart) |
                       ((cand <= 0.8 * kkt_restart) & (cand > kkt_prev_cand)) |
                       (since >= 0.36 * iters)) & ~done
            kkt_prev_cand = cand
            if restart.any():
                rc = restart[b.sc]
                rr = restart[b.sr]
                xc = np.where(use_avg[b.sc], xav, x)
                yc = np.where(use_avg[b.sr], yav, y)
                dx = np.sqrt(seg_sum((xc - xs) ** 2, b.sc, S))
                dy = np.sqrt(seg_sum((yc - ys) ** 2, b.sr, S))
                ok = restart & (dx > 1e-10) & (dy > 1e-10)
                omega = np.where(ok, np.exp(0.5 * np.log(np.maximum(dy, 1e-300) / np.maximum(dx, 1e-300))
                                            + 0.5 * np.log(omega)), omega)
                x = np.where(rc, xc, x)
                y = np.where(rr, yc, y)
                xs = np.where(rc, x, xs)
                ys = np.where(rr, y, ys)
                xa = np.where(rc, 0.0, xa)
                ya = np.where(rr, 0.0, ya)
                na = np.where(restart, 0, na)
                kkt_restart = np.where(restart, cand, kkt_restart)
                kkt_prev_cand = np.where(restart, np.inf, kkt_prev_cand)
                since = np.where(restart, 0, since)
                Ax = A @ x
                ATy = AT @ y
                tau = (eta / omega)[b.sc]
                sig = (eta * omega)[b.sr]
            if self.verbose:
                print(total, "done", done.sum(), "rel max", rel[~done].max() if (~done).any() else 0)
        return x * dc, y * dr, iters, omega

    def _parts(self, x, y, cs, qs, cl, cu, rl, ru):
        b = self.b
        Ax = self.A @ x
        pr = Ax - np.clip(Ax, rl, ru)
        r = cs + qs * x - self.AT @ y
        # dual residual: r_j may be >0 only if cl finite, <0 only if cu finite
        dres = np.where(np.isfinite(cl), 0.0, np.maximum(r, 0.0)) + \
            np.where(np.isfinite(cu), 0.0, np.minimum(r, 0.0))
        pobj = seg_sum(cs * x + 0.5 * qs * x * x, b.sc, b.S)
        rp = np.maximum(r, 0.0)
        rn = np.minimum(r, 0.0)
        dcol = np.where(np.isfinite(cl), cl, 0.0) * rp + np.where(np.isfinite(cu), cu, 0.0) * rn
        yp = np.maximum(y, 0.0)
        yn = np.minimum(y, 0.0)
        drow = np.where(np.isfinite(rl), rl, 0.0) * yp + np.where(np.isfinite(ru), ru, 0.0) * yn
        dobj = seg_sum(dcol - 0.5 * qs * x * x, b.sc, b.S) + seg_sum(drow, b.sr, b.S)
        return pr, dres, pobj, dobj

    def kkt(self, x, y, cs, qs, cl, cu, rl, ru, omega):
        b = self.b
        pr, dres, pobj, dobj = self._parts(x, y, cs, qs, cl, cu, rl, ru)
        return np.sqrt(omega ** 2 * seg_sum(pr * pr, b.sr, b.S) + seg_sum(dres * dres, b.sc, b.S) / omega ** 2
                       + (pobj - dobj) ** 2)

    def rel_kkt(self, x, y, cs, qs, cl, cu, rl, ru):
        """Relative KKT error on the UNSCALED problem (max of the three PDLP ratios)."""
        b = self.b
        dc, dr = self.dc, self.dr
        pr, dres, pobj, dobj = self._parts(x, y, cs, qs, cl, cu, rl, ru)
        pr_u = pr / dr
        dr_u = dres / dc
        bnorm = np.sqrt(seg_sum(np.where(np.isfinite(rl), rl / dr, 0) ** 2 +
                                np.where(np.isfinite(ru), ru / dr, 0) ** 2, b.sr, b.S))
        cnorm = np.sqrt(seg_sum((cs / dc) ** 2, b.sc, b.S))
        p = np.sqrt(seg_sum(pr_u ** 2, b.sr, b.S)) / (1.0 + bnorm)
        d = np.sqrt(seg_sum(dr_u ** 2, b.sc, b.S)) / (1.0 + cnorm)
        g = np.abs(pobj - dobj) / (1.0 + np.abs(pobj) + np.abs(dobj))
        return np.maximum(np.maximum(p, d), g)
