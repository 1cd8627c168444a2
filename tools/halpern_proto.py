"""CPU prototype: PDHG iterations per prox-QP solve on farmer PH subproblems, the kernels' restarted
averaged PDHG (PDLP restarts on the average / current iterate) against reflected restarted Halpern
PDHG (restarts on the fixed-point residual, no running averages).  A design study, not a product
path: numpy, dense matrices, one scenario at a time.

Usage: python tools/halpern_proto.py [S] [cm] [ph_iters] [rho_reflect ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkg  # noqa: E402

_pkg.load()
from mpisppy_amd.engine import BatchArrays  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402
from mpisppy_amd.ph import PH  # noqa: E402

EPS, CHK, BSUF, BNEC, BART, THETA = 1e-9, 32, 0.2, 0.8, 0.25, 0.8


def scenarios(S, cm):
    o = {"solver_name": "phg", "PHIterLimit": 2, "defaultPHrho": 1.0, "convthresh": 0.0, "verbose": False,
         "display_progress": False}
    ph = PH(o, farmer.scenario_names_creator(S), farmer.scenario_creator,
            scenario_creator_kwargs={"crops_multiplier": cm, "num_scens": S})
    models = [ph.local_scenarios[n] for n in ph.local_scenario_names]
    b = BatchArrays(models, ph.all_nodenames, [m._mpisppy_probability for m in models], ph.scen_global0, S, 1)
    out = []
    vals = np.asarray(b.vals).reshape(S, -1)
    for s in range(S):
        A = np.zeros((b.m, b.n))
        for i in range(b.m):
            for p in range(b.rowptr[i], b.rowptr[i + 1]):
                A[i, b.colidx[p]] = vals[s, p]
        sl = lambda v, k: np.asarray(v).reshape(S, -1)[s].copy()  # noqa: E731
        out.append(dict(A=A, c=sl(b.c, b.n), cl=sl(b.cl, b.n), cu=sl(b.cu, b.n), rl=sl(b.rl, b.m),
                        ru=sl(b.ru, b.m)))
    return out, np.asarray(b.nonant_col), b.sense


def precondition(A):
    m, n = A.shape
    dr, dc = np.ones(m), np.ones(n)
    Ah = A.copy()
    for it in range(11):
        pock = it == 10
        rn = np.abs(Ah).sum(1) if pock else np.abs(Ah).max(1)
        cn = np.abs(Ah).sum(0) if pock else np.abs(Ah).max(0)
        rs = np.where(rn > 0, 1 / np.sqrt(np.where(rn > 0, rn, 1)), 1.0)
        cs = np.where(cn > 0, 1 / np.sqrt(np.where(cn > 0, cn, 1)), 1.0)
        Ah = rs[:, None] * Ah * cs[None, :]
        dr *= rs
        dc *= cs
    return Ah, dr, dc, 0.99 / np.linalg.norm(Ah, 2)


class Prob:
    """min c x + q/2 x^2, rl <= A x <= ru, cl <= x <= cu in the scaled space x = dc xh, y = dr yh."""

    def __init__(self, d, c, q):
        self.Ah, self.dr, self.dc, self.eta = precondition(d["A"])
        self.A = d["A"]
        self.c, self.q = c * self.dc, q * self.dc ** 2
        self.lo, self.hi = d["cl"] / self.dc, d["cu"] / self.dc
        self.rlo, self.rhi = d["rl"] * self.dr, d["ru"] * self.dr
        fin = lambda v: np.where(np.abs(v) < 1e300, v, 0.0)  # noqa: E731
        self.bnorm = np.sqrt((fin(d["rl"]) ** 2).sum() + (fin(d["ru"]) ** 2).sum())
        self.cnorm = np.linalg.norm(c)
        bh = np.sqrt((fin(self.rlo) ** 2).sum() + (fin(self.rhi) ** 2).sum())
        cn = np.linalg.norm(self.c)
        self.omega0 = cn / bh if cn > 1e-10 and bh > 1e-10 else 1.0

    def T(self, x, y, aty, ax, tau, sig):
        xn = np.clip((x - tau * (self.c - aty)) / (1 + tau * self.q), self.lo, self.hi)
        axn = self.Ah @ xn
        g = y - sig * (2 * axn - ax)
        yn = np.maximum(g + sig * self.rlo, 0) + np.minimum(g + sig * self.rhi, 0)
        return xn, yn, axn, self.Ah.T @ yn

    def kkt(self, x, y, ax, aty):
        pr = ax - np.clip(ax, self.rlo, self.rhi)
        rc = self.c + self.q * x - aty
        fl, fh = np.abs(self.lo) < 1e300, np.abs(self.hi) < 1e300
        dres = np.where(~fl & (rc > 0), rc, 0) + np.where(~fh & (rc < 0), rc, 0)
        pu, du = pr / self.dr, dres / self.dc
        pobj = self.c @ x + 0.5 * (self.q * x * x).sum()
        frl, frh = np.abs(self.rlo) < 1e300, np.abs(self.rhi) < 1e300
        dobj = (np.where(frl, self.rlo, 0) * np.maximum(y, 0)).sum() + (np.where(frh, self.rhi, 0) * np.minimum(y, 0)).sum()
        dobj += (np.where(fl, self.lo, 0) * np.maximum(rc, 0)).sum() + (np.where(fh, self.hi, 0) * np.minimum(rc, 0)).sum()
        dobj -= 0.5 * (self.q * x * x).sum()
        rel = max(np.linalg.norm(pu) / (1 + self.bnorm), np.linalg.norm(du) / (1 + self.cnorm),
                  abs(pobj - dobj) / (1 + abs(pobj) + abs(dobj)))
        return (pr @ pr, dres @ dres, pobj - dobj), rel


def wkkt(o, w):
    return np.sqrt(w * w * o[0] + o[1] / (w * w) + o[2] ** 2)


def new_omega(w, dx, dy):
    if dx > 1e-10 and dy > 1e-10:
        return np.exp(THETA * np.log(dy / dx) + (1 - THETA) * np.log(w))
    return w


def solve_avg(P, x, y, omega, max_iter=200000):
    """The kernels' scheme: restarted averaged PDHG, PDLP restart rule, checks every CHK."""
    tau, sig = P.eta / omega, P.eta * omega
    ax, aty = P.Ah @ x, P.Ah.T @ y
    o, _ = P.kkt(x, y, ax, aty)
    krst, kprev = wkkt(o, omega), np.inf
    xr, yr = x.copy(), y.copy()
    xs, ys = np.zeros_like(x), np.zeros_like(y)
    it = since = cnt = 0
    while True:
        for _ in range(CHK):
            x, y, ax, aty = P.T(x, y, aty, ax, tau, sig)
            xs += x
            ys += y
        it += CHK
        since += CHK
        cnt += CHK
        xa, ya = xs / cnt, ys / cnt
        axa, atya = P.Ah @ xa, P.Ah.T @ ya
        oc, rc = P.kkt(x, y, ax, aty)
        oa, ra = P.kkt(xa, ya, axa, atya)
        if min(rc, ra) <= EPS or it >= max_iter:
            return (xa, ya, omega, it) if ra < rc else (x, y, omega, it)
        kc, ka = wkkt(oc, omega), wkkt(oa, omega)
        ua = ka < kc
        cand = min(kc, ka)
        if cand <= BSUF * krst or (cand <= BNEC * krst and cand > kprev) or since >= BART * it:
            if ua:
                x, y, ax, aty = xa, ya, axa, atya
            omega = new_omega(omega, np.linalg.norm(x - xr), np.linalg.norm(y - yr))
            tau, sig = P.eta / omega, P.eta * omega
            xr, yr = x.copy(), y.copy()
            xs[:], ys[:] = 0, 0
            cnt = since = 0
            krst, kprev = cand, np.inf
        else:
            kprev = cand


def solve_halpern(P, x, y, omega, refl, max_iter=200000):
    """Reflected restarted Halpern PDHG: z+ = (k+1)/(k+2) ((1+r) T(z) - r z) + 1/(k+2) z0; the
    restart test on the fixed-point residual ||z - T(z)|| (weighted by omega), restart to T(z)."""
    tau, sig = P.eta / omega, P.eta * omega
    ax, aty = P.Ah @ x, P.Ah.T @ y
    x0, y0, ax0, aty0 = x.copy(), y.copy(), ax.copy(), aty.copy()
    r0, rprev = None, np.inf
    it = k = 0
    while True:
        for kk in range(CHK):
            xt, yt, axt, atyt = P.T(x, y, aty, ax, tau, sig)
            if k == 0 and r0 is None:   # the epoch's reference: the residual at its start point
                r0 = np.sqrt(omega * ((xt - x) @ (xt - x)) + ((yt - y) @ (yt - y)) / omega)
            if kk == CHK - 1:
                break
            lam = (k + 1) / (k + 2)
            x = lam * ((1 + refl) * xt - refl * x) + (1 - lam) * x0
            y = lam * ((1 + refl) * yt - refl * y) + (1 - lam) * y0
            ax = lam * ((1 + refl) * axt - refl * ax) + (1 - lam) * ax0
            aty = lam * ((1 + refl) * atyt - refl * aty) + (1 - lam) * aty0
            k += 1
        it += CHK
        _, rt = P.kkt(xt, yt, axt, atyt)
        if rt <= EPS or it >= max_iter:
            return xt, yt, omega, it
        res = np.sqrt(omega * ((xt - x) @ (xt - x)) + ((yt - y) @ (yt - y)) / omega)
        restart = res <= BSUF * r0 or (res <= BNEC * r0 and res > rprev) or k >= BART * it
        rprev = res
        lam = (k + 1) / (k + 2)
        if restart:
            omega = new_omega(omega, np.linalg.norm(xt - x0), np.linalg.norm(yt - y0))
            tau, sig = P.eta / omega, P.eta * omega
            x, y, ax, aty = xt, yt, axt, atyt
            x0, y0, ax0, aty0 = x.copy(), y.copy(), ax.copy(), aty.copy()
            k = 0
            r0, rprev = None, np.inf
        else:
            x = lam * ((1 + refl) * xt - refl * x) + (1 - lam) * x0
            y = lam * ((1 + refl) * yt - refl * y) + (1 - lam) * y0
            ax = lam * ((1 + refl) * axt - refl * ax) + (1 - lam) * ax0
            aty = lam * ((1 + refl) * atyt - refl * aty) + (1 - lam) * aty0
            k += 1


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    cm = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 6
    refls = [float(v) for v in sys.argv[4:]] or [0.0, 0.5, 1.0]
    scen, ncol, sense = scenarios(S, cm)
    rho = 1.0
    n = scen[0]["A"].shape[1]
    W = np.zeros((S, len(ncol)))
    xbar = np.zeros(len(ncol))
    state = [dict(x=np.zeros(n), y=np.zeros(scen[0]["A"].shape[0]), omega=None) for _ in range(S)]
    methods = ["avg"] + [f"halpern{r}" for r in refls]
    for ph_it in range(K):
        tot = {mth: 0 for mth in methods}
        xs = []
        for s in range(S):
            c = sense * scen[s]["c"].copy()
            q = np.zeros(n)
            if ph_it > 0:
                c[ncol] += W[s] - rho * xbar
                q[ncol] = rho
            P = Prob(scen[s], c, q)
            st = state[s]
            om = P.omega0 if st["omega"] is None else np.sqrt(P.omega0 * st["omega"])
            x0 = np.clip(st["x"], P.lo, P.hi)
            y0 = st["y"]
            for mth in methods:
                if mth == "avg":
                    x, y, w, its = solve_avg(P, x0.copy(), y0.copy(), om)
                    keep = (x, y, w)
                else:
                    _, _, _, its = solve_halpern(P, x0.copy(), y0.copy(), om, float(mth[7:]))
                tot[mth] += its
            st["x"], st["y"], st["omega"] = keep
            xs.append((keep[0] * P.dc)[ncol])
        xs = np.array(xs)
        xbar = xs.mean(0)
        W += rho * (xs - xbar)
        print(f"PH iter {ph_it}: PDHG iterations per solve " +
              ", ".join(f"{mth} {tot[mth] / S:.0f}" for mth in methods), flush=True)


if __name__ == "__main__":
    main()
