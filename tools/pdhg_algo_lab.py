"""Algorithm lab (NOT the product, NOT the oracle): PDHG variants inside a mini PH loop on CPU.

Compares PDHG iterations per scenario solve, warm-started across PH iterations exactly like the
engine, for
  * "ra"  : restarted average PDHG (PDLP restarts, the kernels' current algorithm), and
  * "hal" : reflected restarted Halpern PDHG (Lu & Yang 2024; cuPDLPx): z+ = k+1/k+2 ((1+g) T(z) -
            g z) + 1/k+2 z0, restarts on the fixed-point residual, restart to T(z).
Usage: python tools/pdhg_algo_lab.py [S] [cm] [ph_iters] [variant ...]
(LAB_PRESOLVE=1: fold singleton rows into bounds first, as phg_load_batch does.)

Findings kept for the record (farmer cm=10, 100 scenarios, 30 PH iterations, eps 1e-9):
  * singleton-row presolve: 594 -> 369 mean PDHG iterations per solve (adopted);
  * primal weight smoothing theta 0.5 -> 0.8: 369 -> 322 (adopted, confirmed on MI355X);
  * carrying the primal weight across PH iterations (keepw=1): 322 -> 257 here, but on the GPU
    the 10k-scenario PH then stalls (conv 4e-4 after 2 489 PH iterations vs converged at 5 185 in
    1.4 s): not adopted;
  * restart to the current iterate only (noavg=1): +2 % iterations here, but 136 of 10 000
    scenarios hit the iteration cap late in a long PH run on the GPU: not adopted;
  * Halpern / reflected Halpern ("hal"): 20-110 % more iterations: not adopted;
  * extrapolated warm start x_k + a (x_k - x_{k-1}) (and y), "ex=a": 276.3 / 275.4 / 279.4 mean
    iterations per solve at a = 0 / 0.5 / 1 (40 PH iterations, 100 scenarios, presolved, the
    kernels' settings): no gain, not adopted.
"""
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from pdhg_proto import Batch, seg_sum  # noqa: E402


class Lab:
    def __init__(self, b, ruiz=10, eps=1e-9, check=64, max_iter=100000):
        self.b = b
        S = b.S
        A = b.A.tocsr().astype(float)
        dr = np.ones(A.shape[0])
        dc = np.ones(A.shape[1])
        for _ in range(ruiz):
            Aa = abs(A)
            rs = 1.0 / np.sqrt(np.where((m := Aa.max(axis=1).toarray().ravel()) > 0, m, 1.0))
            cs = 1.0 / np.sqrt(np.where((m := Aa.max(axis=0).toarray().ravel()) > 0, m, 1.0))
            A = sp.diags(rs) @ A @ sp.diags(cs)
            dr *= rs
            dc *= cs
        Aa = abs(A)
        rs = 1.0 / np.sqrt(np.maximum(np.asarray(Aa.sum(axis=1)).ravel(), 1e-300))
        cs = 1.0 / np.sqrt(np.maximum(np.asarray(Aa.sum(axis=0)).ravel(), 1e-300))
        A = sp.diags(rs) @ A @ sp.diags(cs)
        dr *= rs
        dc *= cs
        self.A, self.AT, self.dr, self.dc = A.tocsr(), A.T.tocsr(), dr, dc
        v = np.ones(A.shape[1])
        for _ in range(60):
            w = self.AT @ (self.A @ v)
            nrm = np.sqrt(seg_sum(w * w, b.sc, S))
            v = w / np.maximum(nrm[b.sc], 1e-300)
        w = self.A @ v
        self.anorm = np.sqrt(np.sqrt(seg_sum((self.AT @ w) ** 2, b.sc, S)))
        self.eps, self.check, self.max_iter = eps, check, max_iter

    # ------------------------------------------------------------------ residuals
    def parts(self, x, y, cs, qs, cl, cu, rl, ru, Ax=None, ATy=None):
        b = self.b
        Ax = self.A @ x if Ax is None else Ax
        ATy = self.AT @ y if ATy is None else ATy
        pr = Ax - np.clip(Ax, rl, ru)
        r = cs + qs * x - ATy
        dres = np.where(np.isfinite(cl), 0.0, np.maximum(r, 0.0)) + np.where(np.isfinite(cu), 0.0, np.minimum(r, 0.0))
        pobj = seg_sum(cs * x + 0.5 * qs * x * x, b.sc, b.S)
        dcol = np.where(np.isfinite(cl), cl, 0.0) * np.maximum(r, 0) + np.where(np.isfinite(cu), cu, 0.0) * np.minimum(r, 0)
        drow = np.where(np.isfinite(rl), rl, 0.0) * np.maximum(y, 0) + np.where(np.isfinite(ru), ru, 0.0) * np.minimum(y, 0)
        dobj = seg_sum(dcol - 0.5 * qs * x * x, b.sc, b.S) + seg_sum(drow, b.sr, b.S)
        return pr, dres, pobj, dobj

    def rel(self, x, y, cs, qs, cl, cu, rl, ru, Ax=None, ATy=None):
        b = self.b
        pr, dres, pobj, dobj = self.parts(x, y, cs, qs, cl, cu, rl, ru, Ax, ATy)
        bnorm = np.sqrt(seg_sum(np.where(np.isfinite(rl), rl / self.dr, 0) ** 2 +
                                np.where(np.isfinite(ru), ru / self.dr, 0) ** 2, b.sr, b.S))
        cnorm = np.sqrt(seg_sum((cs / self.dc) ** 2, b.sc, b.S))
        p = np.sqrt(seg_sum((pr / self.dr) ** 2, b.sr, b.S)) / (1 + bnorm)
        d = np.sqrt(seg_sum((dres / self.dc) ** 2, b.sc, b.S)) / (1 + cnorm)
        g = np.abs(pobj - dobj) / (1 + np.abs(pobj) + np.abs(dobj))
        return np.maximum(np.maximum(p, d), g), (pr, dres, pobj, dobj)

    def wkkt(self, parts, omega):
        b = self.b
        pr, dres, pobj, dobj = parts
        return np.sqrt(omega ** 2 * seg_sum(pr * pr, b.sr, b.S) + seg_sum(dres * dres, b.sc, b.S) / omega ** 2
                       + (pobj - dobj) ** 2)

    # ------------------------------------------------------------------ one solve
    def solve(self, c, q, x0, y0, variant="ra", gamma=1.0, bs=0.2, bnec=0.8, ba=0.36, th=0.5, noavg=0.0,
              keepw=0.0):
        b = self.b
        S = b.S
        dc, dr = self.dc, self.dr
        cs, qs = c * dc, q * dc * dc
        cl, cu = b.cl / dc, b.cu / dc
        rl, ru = b.rl * dr, b.ru * dr
        A, AT = self.A, self.AT
        x = np.clip(x0 / dc, cl, cu)
        y = y0 / dr
        y = np.where(np.isfinite(rl), y, np.minimum(y, 0))
        y = np.where(np.isfinite(ru), y, np.maximum(y, 0))
        eta = 0.99 / self.anorm
        cn = np.sqrt(seg_sum(cs * cs, b.sc, S))
        bn = np.sqrt(seg_sum(np.where(np.isfinite(rl), rl, 0) ** 2 + np.where(np.isfinite(ru), ru, 0) ** 2, b.sr, S))
        omega = np.where((cn > 1e-10) & (bn > 1e-10), cn / np.maximum(bn, 1e-300), 1.0)
        if keepw and getattr(self, "_omega_prev", None) is not None:
            omega = self._omega_prev if keepw == 1.0 else np.sqrt(self._omega_prev * omega)
        done = np.zeros(S, bool)
        iters = np.zeros(S, int)
        xr, yr = x.copy(), y.copy()
        xa, ya = np.zeros_like(x), np.zeros_like(y)
        na = np.zeros(S)
        Ax, ATy = A @ x, AT @ y
        krst = self.wkkt(self.rel(x, y, cs, qs, cl, cu, rl, ru, Ax, ATy)[1], omega)
        kprev = np.full(S, np.inf)
        since = np.zeros(S, int)
        k_h = np.zeros(S)                      # Halpern counter since restart
        xout, yout = x.copy(), y.copy()
        total = 0
        while total < self.max_iter and not done.all():
            tau = (eta / omega)[b.sc]
            sig = (eta * omega)[b.sr]
            ac, ar = ~done[b.sc], ~done[b.sr]
            for _ in range(self.check):
                xh = np.clip((x - tau * (cs - ATy)) / (1 + tau * qs), cl, cu)
                Axh = A @ xh
                g = y - sig * (2 * Axh - Ax)
                yh = np.maximum(g + sig * rl, 0) + np.minimum(g + sig * ru, 0)
                if variant == "ra":
                    xn, yn, Axn = xh, yh, Axh
                    xa += np.where(ac, xn, 0)
                    ya += np.where(ar, yn, 0)
                    na += ~done
                else:
                    lam = ((k_h + 1) / (k_h + 2))
                    lc, lr = lam[b.sc], lam[b.sr]
                    xn = lc * ((1 + gamma) * xh - gamma * x) + (1 - lc) * xr
                    yn = lr * ((1 + gamma) * yh - gamma * y) + (1 - lr) * yr
                    Axn = A @ xn
                    k_h += ~done
                    self._last_h = (xh, yh, Axh)
                x = np.where(ac, xn, x)
                y = np.where(ar, yn, y)
                Ax = np.where(ar, Axn, Ax)
                ATy = AT @ y
            total += self.check
            iters += self.check * (~done)
            since += self.check * (~done)
            if variant == "ra":
                inv = 1 / np.maximum(na, 1)
                xav, yav = xa * inv[b.sc], ya * inv[b.sr]
                rc_, pc = self.rel(x, y, cs, qs, cl, cu, rl, ru, Ax, ATy)
                ra_, pa = self.rel(xav, yav, cs, qs, cl, cu, rl, ru)
                kc, ka = self.wkkt(pc, omega), self.wkkt(pa, omega)
                ua = (ka < kc) & (noavg == 0.0)
                if noavg:
                    ra_ = np.full_like(rc_, np.inf)
                cand = np.where(ua, ka, kc)
                fin_ = (np.minimum(rc_, ra_) <= self.eps) & ~done
                xf = np.where(ua[b.sc] & (ra_ < rc_)[b.sc], xav, x)
                yf = np.where(ua[b.sr] & (ra_ < rc_)[b.sr], yav, y)
                xtgt = np.where(ua[b.sc], xav, x)
                ytgt = np.where(ua[b.sr], yav, y)
            else:
                xh, yh, Axh = self._last_h
                rc_, pc = self.rel(xh, yh, cs, qs, cl, cu, rl, ru, Axh, None)
                # fixed-point residual ||z - T(z)|| in the primal-weighted norm
                fx = seg_sum((x - xh) ** 2, b.sc, S)
                fy = seg_sum((y - yh) ** 2, b.sr, S)
                cand = np.sqrt(omega * fx + fy / omega)
                fin_ = (rc_ <= self.eps) & ~done
                xf, yf = xh, yh
                xtgt, ytgt = xh, yh
            xout = np.where((fin_)[b.sc], xf, xout)
            yout = np.where((fin_)[b.sr], yf, yout)
            done |= fin_
            restart = ((cand <= bs * krst) | ((cand <= bnec * krst) & (cand > kprev)) | (since >= ba * iters)) & ~done
            kprev = cand
            if restart.any():
                rc, rr = restart[b.sc], restart[b.sr]
                dx = np.sqrt(seg_sum((xtgt - xr) ** 2, b.sc, S))
                dy = np.sqrt(seg_sum((ytgt - yr) ** 2, b.sr, S))
                ok = restart & (dx > 1e-10) & (dy > 1e-10)
                omega = np.where(ok, np.exp(th * np.log(np.maximum(dy, 1e-300) / np.maximum(dx, 1e-300))
                                            + (1 - th) * np.log(omega)), omega)
                x = np.where(rc, xtgt, x)
                y = np.where(rr, ytgt, y)
                xr = np.where(rc, x, xr)
                yr = np.where(rr, y, yr)
                xa = np.where(rc, 0, xa)
                ya = np.where(rr, 0, ya)
                na = np.where(restart, 0, na)
                k_h = np.where(restart, 0, k_h)
                krst = np.where(restart, cand, krst)
                kprev = np.where(restart, np.inf, kprev)
                since = np.where(restart, 0, since)
                Ax, ATy = A @ x, AT @ y
        xout = np.where(done[b.sc], xout, x)
        yout = np.where(done[b.sr], yout, y)
        self._omega_prev = omega
        return xout * dc, yout * dr, iters


def singleton_rows_to_bounds(a, keep_cols):
    """Rows with one nonzero on a non-nonant column become bounds on that column."""
    rp, ci, v = a["rowptr"], a["colidx"], a["vals"]
    cl, cu = a["col_lo"].copy(), a["col_hi"].copy()
    keep = []
    for i in range(len(rp) - 1):
        if rp[i + 1] - rp[i] == 1 and ci[rp[i]] not in keep_cols and v[rp[i]] != 0:
            j, aa = ci[rp[i]], v[rp[i]]
            lo, hi = a["row_lo"][i] / aa, a["row_hi"][i] / aa
            if aa < 0:
                lo, hi = hi, lo
            cl[j], cu[j] = max(cl[j], lo), min(cu[j], hi)
        else:
            keep.append(i)
    rows = [(ci[rp[i]:rp[i + 1]], v[rp[i]:rp[i + 1]]) for i in keep]
    nrp = np.concatenate([[0], np.cumsum([len(r[0]) for r in rows])]).astype(np.int32)
    return dict(a, rowptr=nrp, colidx=np.concatenate([r[0] for r in rows]), vals=np.concatenate([r[1] for r in rows]),
                row_lo=a["row_lo"][keep], row_hi=a["row_hi"][keep], col_lo=cl, col_hi=cu)


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    cm = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    variants = sys.argv[4:] or ["ra", "hal:1.0", "hal:0.0"]
    from oracle import models as om
    scens = [om.farmer(nm, crops_multiplier=cm, num_scens=S) for nm in om.farmer_names(S)]
    arrs = [s.arrays() for s in scens]
    if os.environ.get("LAB_PRESOLVE"):
        arrs = [singleton_rows_to_bounds(a, set(scens[0].nonant_cols())) for a in arrs]
        print("presolve: m", len(arrs[0]["row_lo"]), flush=True)
    b = Batch(arrs)
    cols = np.array(scens[0].nonant_cols())
    N = len(cols)
    n = len(arrs[0]["c"])
    lab = Lab(b)
    c0 = b.c.copy()
    p = 1.0 / S
    for var in variants:
        name, _, opt = var.partition(":")
        kw = {}
        for item in filter(None, opt.split(",")):
            k_, _, v_ = item.partition("=")
            if k_ == "chk":
                lab.check = int(v_)
            else:
                kw[k_ if v_ else "gamma"] = float(v_ if v_ else k_)
        lab.check = int(kw.pop("chk", lab.check)) if "chk" in kw else lab.check
        ex = kw.pop("ex", 0.0)          # extrapolated warm start x + ex (x - x_prev)
        W = np.zeros((S, N))
        xbar = np.zeros(N)
        x = np.zeros(b.A.shape[1])
        y = np.zeros(b.A.shape[0])
        its = []
        xp, yp = None, None
        t0 = time.perf_counter()
        for k in range(K + 1):
            c = c0.copy().reshape(S, n)
            q = np.zeros((S, n))
            if k > 0:
                c[:, cols] += W - 1.0 * xbar
                q[:, cols] = 1.0
            x0, y0 = x, y
            if ex and xp is not None and k > 1:
                x0, y0 = x + ex * (x - xp), y + ex * (y - yp)
            xp, yp = x, y
            x, y, it = lab.solve(c.ravel(), q.ravel(), x0, y0, variant=name, **kw)
            if k > 0:
                its.append(it.mean())
            xn = x.reshape(S, n)[:, cols]
            xbar = p * xn.sum(axis=0)
            W += 1.0 * (xn - xbar)
            conv = np.abs(xn - xbar).mean()
        lab.check = 64
        print(f"{var:24s} mean iters/solve over {K} PH iters: {np.mean(its):8.1f}  last {its[-1]:7.1f} "
              f"conv {conv:.3e}  ({time.perf_counter() - t0:.1f}s)", flush=True)


if __name__ == "__main__":
    main()
