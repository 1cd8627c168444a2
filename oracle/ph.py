"""TEST INFRASTRUCTURE (oracle): numpy restatement of the reference PH hot path.

Follows, statement by statement where order matters for floating point:

* ``_Compute_Xbar``          -- ``mpisppy/phbase.py:32-112`` (per-rank accumulation in local
  scenario order, then a SUM over ranks standing in for ``comms[node].Allreduce``)
* ``Update_W``               -- ``mpisppy/phbase.py:301-326``
* ``convergence_diff``       -- ``mpisppy/phbase.py:349-371`` (mean over ranks of per-rank means)
* ``Iter0`` / ``iterk_loop`` -- ``mpisppy/phbase.py:829-1061``; ``PH.ph_main`` ``mpisppy/opt/ph.py:31-76``
* ``solve_one`` contract     -- ``mpisppy/spopt.py:99-247`` (HiGHS via ``oracle.highs``)
* ``Ebound``/``Eobjective``/``_update_E1``/``feas_prob`` -- ``mpisppy/spopt.py:344-470``
* rank slices                -- ``_ScenTree.scen_names_to_ranks``, ``mpisppy/utils/sputils.py:790-826``
* node probabilities         -- ``mpisppy/spbase.py:382-395`` (prob_coeff = p_s / uncond_prob)
* default probability        -- ``mpisppy/spbase.py:509-526`` (1/S)

Scenario subproblem in min-form (``phbase.py:670-760``)::

    min sg*c^T x + W_on * sum_k W_k x_k + prox_on * sum_k rho_k/2 (x_k^2 - 2 xbar_k x_k + xbar_k^2)

(sg = -1 for a maximisation model; the reported objective is then negated back.)
"""
import math
import time

import numpy as np

from . import highs


def rank_slices(S, n_proc):
    """``sputils.py:819-826``: contiguous ``range(int(i*avg), int((i+1)*avg))``, avg = S/n_proc."""
    if n_proc == 1:
        return [list(range(S))]
    avg = S / n_proc
    return [list(range(int(i * avg), int((i + 1) * avg))) for i in range(n_proc)]


class OraclePH:
    def __init__(self, options, all_scenario_names, scenario_creator, scenario_creator_kwargs=None,
                 n_proc=1, scenarios=None, threads=1, variable_probability=None):
        self.options = dict(options)
        self.names = list(all_scenario_names)
        kw = scenario_creator_kwargs or {}
        if scenarios is None:
            scenarios = [scenario_creator(nm, **kw) for nm in self.names]
        self.scen = scenarios
        self.S = len(self.scen)
        self.n_proc = n_proc
        self.slices = rank_slices(self.S, n_proc)
        self.threads = threads
        self.is_minimizing = self.scen[0].sense == 1
        # probabilities (spbase.py:509-526)
        self.prob = np.array([s.prob if s.prob is not None else 1.0 / self.S for s in self.scen])
        # node bookkeeping: nonant keys (ndn, i) in node-list order (spbase.py:297-306)
        self.keys = []
        self.prob_coeff = []          # per scenario: list per nonant of prob_coeff[node]
        for s, p in zip(self.scen, self.prob):
            uncond = 1.0
            keys = []
            pc = []
            for depth, nd in enumerate(s.nodes):
                if depth > 0:
                    uncond = uncond * nd["cond_prob"]
                for i in range(len(nd["cols"])):
                    keys.append((nd["name"], i))
                    pc.append(p / uncond)
            self.keys.append(keys)
            self.prob_coeff.append(np.array(pc))
        self.N = len(self.keys[0])
        # variable_probability (spbase.py:398-438): callable(OScen) -> [(column, prob)]
        self.prob0_mask = np.ones((self.S, self.N))
        self.has_varprob = variable_probability is not None
        if variable_probability is not None:
            for k, s in enumerate(self.scen):
                pos = {col: i for i, col in enumerate(s.nonant_cols())}
                for col, pr in variable_probability(s):
                    self.prob_coeff[k][pos[col]] = pr
                    if pr == 0:
                        self.prob0_mask[k, pos[col]] = 0.0
        self.cols = np.array([s.nonant_cols() for s in self.scen], dtype=np.int64)
        self.arr = [s.arrays() for s in self.scen]
        rho0 = float(self.options["defaultPHrho"])
        self.rho = np.full((self.S, self.N), rho0)
        self.W = np.zeros((self.S, self.N))
        # smoothed PH (phbase.py:641-655): z = 0, p = defaultPHp, beta = defaultPHbeta
        self.smoothed = int(self.options.get("smoothed", 0))
        self.z = np.zeros((self.S, self.N))
        self.p = np.full((self.S, self.N), float(self.options.get("defaultPHp", 0.0)))
        self.beta = np.full((self.S, self.N), float(self.options.get("defaultPHbeta", 0.0)))
        self.xbar = np.zeros((self.S, self.N))
        self.xsqbar = np.zeros((self.S, self.N))
        self.x = [None] * self.S
        self.obj = np.zeros(self.S)
        self.outer = np.zeros(self.S)
        self.feasible = np.ones(self.S, dtype=bool)
        self.W_on = 0
        self.prox_on = 0
        self._PHIter = 0
        self.conv = None
        self.solve_count = 0
        self.solve_time = 0.0

    # ------------------------------------------------------------------------------- solves
    def nonants(self, k):
        return self.x[k][self.cols[k]]

    def solve_one(self, k):
        """``spopt.py:99-247`` for one scenario, min-form with W/prox terms."""
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
            if self.smoothed:   # phbase.py:743-755: + p/2 (x^2 - 2 z x + z^2)
                p_, z = self.p[k], self.z[k]
                np.add.at(c, cols, -p_ * z)
                np.add.at(q, cols, p_)
                off += float(np.sum(p_ / 2.0 * z * z))
        t0 = time.perf_counter()
        r = highs.solve(c, a["rowptr"], a["colidx"], a["vals"], a["row_lo"], a["row_hi"],
                        a["col_lo"], a["col_hi"], qdiag=q, offset=off, threads=self.threads)
        self.solve_time += time.perf_counter() - t0
        self.solve_count += 1
        if not r.ok:
            self.feasible[k] = False
            import os
            if os.environ.get("ORACLE_DUMP"):
                np.savez(os.environ["ORACLE_DUMP"], cost=c, q=q if q is not None else np.zeros(0), off=off,
                         **{kk: np.asarray(v) for kk, v in a.items()})
            raise RuntimeError(f"[oracle] Solve failed for scenario {self.names[k]}: {r.status}")
        self.feasible[k] = True
        self.x[k] = r.x
        self.obj[k] = sg * r.obj
        self.outer[k] = sg * r.obj        # LP/QP solved to optimality: Lower_bound == objective
        return r

    def solve_loop(self):
        for k in range(self.S):
            self.solve_one(k)

    # ------------------------------------------------------------------------------- PH update
    def Compute_Xbar(self):
        """``phbase.py:32-112``: per node, per rank accumulate p*x and p*x^2, SUM over ranks."""
        # node -> (rank -> local concat)
        node_len = {}
        for k in range(self.S):
            for (ndn, i) in self.keys[k]:
                node_len[ndn] = max(node_len.get(ndn, 0), i + 1)
        glob = {nd: np.zeros(2 * L) for nd, L in node_len.items()}
        for sl in self.slices:
            loc = {}
            for k in sl:
                xs = self.nonants(k)
                pos = 0
                for nd in self.scen[k].nodes:
                    ndn = nd["name"]
                    nlen = len(nd["cols"])
                    if ndn not in loc:
                        loc[ndn] = np.zeros(2 * nlen)
                    arr = xs[pos:pos + nlen]
                    probs = self.prob_coeff[k][pos:pos + nlen]
                    loc[ndn][:nlen] += probs * arr
                    loc[ndn][nlen:] += probs * arr ** 2
                    pos += nlen
            for ndn, v in loc.items():
                glob[ndn] = glob[ndn] + v
        for k in range(self.S):
            pos = 0
            for nd in self.scen[k].nodes:
                ndn = nd["name"]
                nlen = len(nd["cols"])
                self.xbar[k, pos:pos + nlen] = glob[ndn][:nlen]
                self.xsqbar[k, pos:pos + nlen] = glob[ndn][nlen:]
                pos += nlen
        self.node_xbar = {nd: v[:len(v) // 2].copy() for nd, v in glob.items()}

    def Update_W(self):
        """``phbase.py:301-326``."""
        for k in range(self.S):
            xs = self.nonants(k)
            self.W[k] += self.rho[k] * (xs - self.xbar[k])
            if self.has_varprob:
                self.W[k] *= self.prob0_mask[k]

    def Update_z(self):
        """``phbase.py:329-346``: z += beta (x - z)."""
        for k in range(self.S):
            xs = self.nonants(k)
            self.z[k] += self.beta[k] * (xs - self.z[k])

    def convergence_diff(self):
        """``phbase.py:349-371``."""
        tot = 0.0
        for sl in self.slices:
            local = 0.0
            cnt = 0
            for k in sl:
                xs = self.nonants(k)
                for i in range(self.N):
                    local += abs(xs[i] - self.xbar[k, i])
                    cnt += 1
            local /= cnt
            tot += local
        return tot / self.n_proc

    # ------------------------------------------------------------------------------- expectations
    def _rank_fsum(self, vals):
        out = 0.0
        for sl in self.slices:
            out += math.fsum(vals[k] for k in sl)
        return out

    def Ebound(self):
        """``spopt.py:377-422``."""
        return self._rank_fsum([self.prob[k] * float(self.outer[k]) for k in range(self.S)])

    def scenario_objective(self, k, W_on=None, prox_on=None):
        """pyo.value(objfct) with the current Params (``spopt.py:365``)."""
        W_on = self.W_on if W_on is None else W_on
        prox_on = self.prox_on if prox_on is None else prox_on
        a = self.arr[k]
        sg = 1.0 if self.scen[k].sense == 1 else -1.0
        f = float(a["c"] @ self.x[k])
        xs = self.nonants(k)
        term = 0.0
        if W_on:
            term += float(np.sum(self.W[k] * xs))
        if prox_on:
            term += float(np.sum(self.rho[k] / 2.0 * (xs * xs - 2.0 * self.xbar[k] * xs + self.xbar[k] ** 2)))
            if self.smoothed:
                term += float(np.sum(self.p[k] / 2.0 * (xs * xs - 2.0 * self.z[k] * xs + self.z[k] ** 2)))
        return f + sg * term

    def Eobjective(self, W_on=None, prox_on=None):
        """``spopt.py:344-374``."""
        vals = [self.prob[k] * self.scenario_objective(k, W_on, prox_on) for k in range(self.S)]
        out = 0.0
        for sl in self.slices:
            out += math.fsum(vals[k] for k in sl)
        return out

    def _update_E1(self):
        self.E1 = float(sum(sum(self.prob[k] for k in sl) for sl in self.slices))

    def feas_prob(self):
        return float(sum(sum(self.prob[k] for k in sl if self.feasible[k]) for sl in self.slices))

    # ------------------------------------------------------------------------------- PH loop
    def Iter0(self):
        """``phbase.py:829-946``."""
        self._PHIter = 0
        self.W_on = 0
        self.prox_on = 0
        self.solve_loop()
        self._update_E1()
        if abs(1 - self.E1) > 1e-5:
            raise RuntimeError(f"Total probability of scenarios was {self.E1}")
        feasP = self.feas_prob()
        if feasP != self.E1:
            raise RuntimeError(f"Infeasibility detected; E_feas={feasP}, E1={self.E1}")
        if self.smoothed == 2:   # phbase.py:918-922
            self.p = self.p * self.rho
        self.conv = None
        self.trivial_bound = self.Ebound()
        self.W_on = 1
        self.prox_on = 1
        return self.trivial_bound

    def iterk_loop(self, callback=None):
        """``phbase.py:949-1061``."""
        max_iterations = int(self.options["PHIterLimit"])
        self.conv = None
        self.history = []
        for self._PHIter in range(1, max_iterations + 1):
            self.Compute_Xbar()
            self.Update_W()
            if self.smoothed:
                self.Update_z()
            self.conv = self.convergence_diff()
            self.history.append(self.conv)
            if callback is not None:
                callback(self)
            if self.conv is not None and self.conv < self.options["convthresh"]:
                break
            self.solve_loop()

    def ph_main(self, finalize=True, callback=None):
        """``opt/ph.py:31-76``: returns (conv, Eobj, trivial_bound)."""
        tb = self.Iter0()
        self.iterk_loop(callback)
        Eobj = self.Eobjective() if finalize else None
        return self.conv, Eobj, tb

    # ------------------------------------------------------------------------------- bounds
    def lagrangian_bound(self, W):
        """Lagrangian outer bound with the given W, prox off (``lagrangian_bounder.py:13-44``)."""
        saveW, save_on, save_prox = self.W.copy(), self.W_on, self.prox_on
        savex, saveobj, saveouter = list(self.x), self.obj.copy(), self.outer.copy()
        self.W = np.array(W, dtype=float).reshape(self.S, self.N)
        self.W_on, self.prox_on = 1, 0
        self.solve_loop()
        b = self.Ebound()
        self.W, self.W_on, self.prox_on = saveW, save_on, save_prox
        self.x, self.obj, self.outer = savex, saveobj, saveouter
        return b

    def xhat_eval(self, xhat):
        """Inner bound of a two-stage candidate (``xhat_eval.py:102-170``, ``xhatbase.py:42-235``):
        fix every scenario's nonants to ``xhat``, solve with W and prox off; sum_s p_s obj_s if every
        scenario is feasible, else None."""
        vals = []
        for k in range(self.S):
            a = self.arr[k]
            lo, hi = a["col_lo"].copy(), a["col_hi"].copy()
            lo[self.cols[k]] = xhat
            hi[self.cols[k]] = xhat
            sg = 1.0 if self.scen[k].sense == 1 else -1.0
            # feasibility tolerance 1e-6: a candidate from a first-order solve (PDHG, eps 1e-9 relative)
            # meets first-stage rows to ~1e-9 relative (5e-7 on the farmer acreage row), not 1e-10 absolute
            r = highs.solve(sg * a["c"], a["rowptr"], a["colidx"], a["vals"], a["row_lo"], a["row_hi"], lo, hi,
                            tol=1e-6)
            if not r.ok:
                return None
            vals.append(self.prob[k] * sg * r.obj)
        out = 0.0
        for sl in self.slices:
            out += math.fsum(vals[k] for k in sl)
        return out


def ef_solve(scenarios, probs=None):
    """Extensive form (``mpisppy/utils/sputils.py:143-357`` create_EF): block-diagonal scenario
    LPs, objective sum_s p_s f_s, plus equality rows x_{s,node,i} = x_{first scen of node,i}.
    Returns (objective in the model's sense, per-scenario nonant values)."""
    S = len(scenarios)
    if probs is None:
        probs = [s.prob if s.prob is not None else 1.0 / S for s in scenarios]
    arrs = [s.arrays() for s in scenarios]
    offs = np.cumsum([0] + [s.n for s in scenarios])
    sense = scenarios[0].sense
    sg = 1.0 if sense == 1 else -1.0
    c = np.concatenate([sg * p * a["c"] for p, a in zip(probs, arrs)])
    rp, ci, vv, rlo, rhi = [0], [], [], [], []
    for k, a in enumerate(arrs):
        for i in range(len(a["rowptr"]) - 1):
            for p in range(a["rowptr"][i], a["rowptr"][i + 1]):
                ci.append(offs[k] + a["colidx"][p])
                vv.append(a["vals"][p])
            rp.append(len(ci))
        rlo.extend(a["row_lo"])
        rhi.extend(a["row_hi"])
    first = {}
    for k, s in enumerate(scenarios):
        for nd in s.nodes:
            for i, col in enumerate(nd["cols"]):
                key = (nd["name"], i)
                if key not in first:
                    first[key] = offs[k] + col
                else:
                    ci.extend([offs[k] + col, first[key]])
                    vv.extend([1.0, -1.0])
                    rp.append(len(ci))
                    rlo.append(0.0)
                    rhi.append(0.0)
    clo = np.concatenate([a["col_lo"] for a in arrs])
    chi = np.concatenate([a["col_hi"] for a in arrs])
    r = highs.solve(c, np.array(rp), np.array(ci), np.array(vv), np.array(rlo), np.array(rhi),
                    clo, chi)
    if not r.ok:
        raise RuntimeError(f"EF solve failed: {r.status}")
    xs = [r.x[offs[k] + np.array(s.nonant_cols(), dtype=int)] for k, s in enumerate(scenarios)]
    return sg * r.obj, xs
