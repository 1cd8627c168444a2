"""TEST INFRASTRUCTURE (oracle): Pyomo-free restatements of the reference example generators.

Each generator returns an ``OScen`` holding one scenario's LP in standard form

    min/max  c^T x     s.t.  row_lo <= A x <= row_hi,   col_lo <= x <= col_hi

with A in CSR, plus the scenario-tree node list (name, cond_prob, stage, nonant column indices in
the reference's nonant order) and the probability (None -> SPBase default 1/S,
``mpisppy/spbase.py:509-526``).

This module is written independently of the product's generators in ``mpi-sppy_amd/examples``;
``tests/test_models.py`` checks the two bit-for-bit.
"""
import os
import re

import numpy as np

INF = float("inf")


class OScen:
    def __init__(self, name):
        self.name = name
        self.colnames = []
        self.lo = []
        self.hi = []
        self.cost = []
        self.rows = []          # list of (dict col->coef, lo, hi, name)
        self.sense = 1          # 1 = minimize, -1 = maximize
        self.nodes = []         # list of dict(name, cond_prob, stage, cols)
        self.prob = None

    def var(self, name, lo=0.0, hi=INF, cost=0.0):
        self.colnames.append(name)
        self.lo.append(lo)
        self.hi.append(hi)
        self.cost.append(cost)
        return len(self.colnames) - 1

    def row(self, coefs, lo, hi, name=""):
        self.rows.append((dict(coefs), lo, hi, name))

    # dense/CSR views ----------------------------------------------------------------------------
    def csr(self):
        rowptr = [0]
        colidx = []
        vals = []
        for coefs, _, _, _ in self.rows:
            for j in sorted(coefs):
                colidx.append(j)
                vals.append(coefs[j])
            rowptr.append(len(colidx))
        return (np.array(rowptr, np.int32), np.array(colidx, np.int32), np.array(vals, np.float64))

    @property
    def n(self):
        return len(self.colnames)

    @property
    def m(self):
        return len(self.rows)

    def arrays(self):
        rp, ci, v = self.csr()
        return dict(
            c=np.array(self.cost, np.float64),
            rowptr=rp, colidx=ci, vals=v,
            row_lo=np.array([r[1] for r in self.rows], np.float64),
            row_hi=np.array([r[2] for r in self.rows], np.float64),
            col_lo=np.array(self.lo, np.float64),
            col_hi=np.array(self.hi, np.float64),
        )

    def nonant_cols(self):
        out = []
        for nd in self.nodes:
            out.extend(nd["cols"])
        return out


def extract_num(s):
    """``mpisppy/utils/sputils.py:497-506``."""
    return int(re.compile(r"(\d+)$").search(s).group(1))


# ------------------------------------------------------------------------------------------------
# farmer: examples/farmer/farmer.py:31-230 (== mpisppy/tests/examples/farmer.py:31-230)
# ------------------------------------------------------------------------------------------------
_FARMER_BASE = ("WHEAT", "CORN", "SUGAR_BEETS")
_PRICE_QUOTA = {"WHEAT": 100000.0, "CORN": 100000.0, "SUGAR_BEETS": 6000.0}
_SUB_PRICE = {"WHEAT": 170.0, "CORN": 150.0, "SUGAR_BEETS": 36.0}
_SUPER_PRICE = {"WHEAT": 0.0, "CORN": 0.0, "SUGAR_BEETS": 10.0}
_CATTLE = {"WHEAT": 200.0, "CORN": 240.0, "SUGAR_BEETS": 0.0}
_PURCHASE = {"WHEAT": 238.0, "CORN": 210.0, "SUGAR_BEETS": 100000.0}
_PLANT = {"WHEAT": 150.0, "CORN": 230.0, "SUGAR_BEETS": 260.0}
_YIELD = {
    "BelowAverageScenario": {"WHEAT": 2.0, "CORN": 2.4, "SUGAR_BEETS": 16.0},
    "AverageScenario": {"WHEAT": 2.5, "CORN": 3.0, "SUGAR_BEETS": 20.0},
    "AboveAverageScenario": {"WHEAT": 3.0, "CORN": 3.6, "SUGAR_BEETS": 24.0},
}
_FARMER_STREAM = np.random.RandomState()


def farmer(scenario_name, crops_multiplier=1, num_scens=None, seedoffset=0, sense=1):
    scennum = extract_num(scenario_name)
    basenames = ["BelowAverageScenario", "AverageScenario", "AboveAverageScenario"]
    base = basenames[scennum % 3]
    group = scennum // 3
    _FARMER_STREAM.seed(scennum + seedoffset)               # farmer.py:66
    crops = []
    for i in range(crops_multiplier):                       # farmer.py:105-113 (insertion order)
        for cb in _FARMER_BASE:
            crops.append((cb + str(i), cb))
    yields = {}
    for cname, cb in crops:                                  # farmer.py:157-163
        if group != 0:
            yields[cname] = _YIELD[base][cb] + _FARMER_STREAM.rand()
        else:
            yields[cname] = _YIELD[base][cb]
    total = 500.0 * crops_multiplier
    s = OScen(scenario_name)
    s.sense = sense
    sg = 1.0 if sense == 1 else -1.0
    da = {cn: s.var(f"DevotedAcreage[{cn}]", 0.0, total, sg * _PLANT[cb]) for cn, cb in crops}
    qsub = {cn: s.var(f"QuantitySubQuotaSold[{cn}]", 0.0, INF, -sg * _SUB_PRICE[cb]) for cn, cb in crops}
    qsup = {cn: s.var(f"QuantitySuperQuotaSold[{cn}]", 0.0, INF, -sg * _SUPER_PRICE[cb]) for cn, cb in crops}
    qp = {cn: s.var(f"QuantityPurchased[{cn}]", 0.0, INF, sg * _PURCHASE[cb]) for cn, cb in crops}
    s.row({da[cn]: 1.0 for cn, _ in crops}, -INF, total, "ConstrainTotalAcreage")
    for cn, cb in crops:
        s.row({da[cn]: yields[cn], qp[cn]: 1.0, qsub[cn]: -1.0, qsup[cn]: -1.0}, _CATTLE[cb], INF,
              f"EnforceCattleFeedRequirement[{cn}]")
    for cn, cb in crops:
        s.row({qsub[cn]: 1.0, qsup[cn]: 1.0, da[cn]: -yields[cn]}, -INF, 0.0, f"LimitAmountSold[{cn}]")
    for cn, cb in crops:
        s.row({qsub[cn]: 1.0}, 0.0, _PRICE_QUOTA[cb], f"EnforceQuotas[{cn}]")
    # nonant order: sorted DevotedAcreage keys (scenario_tree.py:45-46)
    s.nodes = [dict(name="ROOT", cond_prob=1.0, stage=1, cols=[da[k] for k in sorted(da)])]
    if num_scens is not None:
        s.prob = 1.0 / num_scens
    s.yields = yields
    return s


def farmer_names(num_scens, start=0):
    return [f"scen{i}" for i in range(start, start + num_scens)]


# ------------------------------------------------------------------------------------------------
# hydro: examples/hydro/hydro.py:79-241 with PySP/scenariodata/Scen{1..9}.dat
# ------------------------------------------------------------------------------------------------
_HYDRO_A2 = (10.0, 50.0, 90.0)
_HYDRO_A3 = (40.0, 50.0, 60.0)


def hydro(scenario_name, branching_factors=(3, 3), inflow=None):
    """3-stage hydro.  ``inflow`` overrides (A2, A3); default = the Scen{1..9}.dat values."""
    snum = extract_num(scenario_name)
    if inflow is None:
        a2 = _HYDRO_A2[(snum - 1) // 3]
        a3 = _HYDRO_A3[(snum - 1) % 3]
    else:
        a2, a3 = inflow
    A = {1: 50.0, 2: a2, 3: a3}
    D = {1: 90.0, 2: 160.0, 3: 110.0}
    u = {1: 0.6048, 2: 0.6048, 3: 1.2096}
    dur = {1: 168.0, 2: 168.0, 3: 336.0}
    T = 8760.0
    V0 = 60.48
    betaGt, betaGh, betaDns = 1.0, 0.0, 10.0
    r = {t: (1 / 1.1) ** (dur[t] / T) for t in (1, 2, 3)}
    s = OScen(scenario_name)
    pgt = {t: s.var(f"Pgt[{t}]", 0.0, 100.0) for t in (1, 2, 3)}
    pgh = {t: s.var(f"Pgh[{t}]", 0.0, 100.0) for t in (1, 2, 3)}
    pdns = {t: s.var(f"PDns[{t}]", 0.0, D[t]) for t in (1, 2, 3)}
    vol = {t: s.var(f"Vol[{t}]", 0.0, 100.0) for t in (1, 2, 3)}
    sl = s.var("sl", 0.0, INF)
    sc = {t: s.var(f"StageCost[{t}]", -INF, INF, 1.0) for t in (1, 2, 3)}
    for t in (1, 2, 3):   # StageCost[t] - r (..) [- sl] == 0
        co = {sc[t]: 1.0, pgt[t]: -r[t] * betaGt, pgh[t]: -r[t] * betaGh, pdns[t]: -r[t] * betaDns}
        if t == 3:
            co[sl] = -1.0
        s.row(co, 0.0, 0.0, f"StageCostConstraint[{t}]")
    for t in (1, 2, 3):
        s.row({pgt[t]: 1.0, pgh[t]: 1.0, pdns[t]: 1.0}, D[t], D[t], f"demand[{t}]")
    for t in (1, 2, 3):   # Vol[t] - Vol[t-1] + u A... :  Vol[t]-Vol[t-1]+u*Pgh[t] <= u*A[t]
        co = {vol[t]: 1.0, pgh[t]: u[t]}
        rhs = u[t] * A[t]
        if t == 1:
            rhs = rhs + V0
        else:
            co[vol[t - 1]] = -1.0
        s.row(co, -INF, rhs, f"conserv[{t}]")
    s.row({sl: 1.0, vol[3]: 4166.67}, 4166.67 * V0, INF, "fcfe")
    bf = branching_factors
    ndn = "ROOT_" + str((snum - 1) // bf[1])
    s.nodes = [
        dict(name="ROOT", cond_prob=1.0, stage=1, cols=[pgt[1], pgh[1], pdns[1], vol[1]]),
        dict(name=ndn, cond_prob=1.0 / bf[0], stage=2, cols=[pgt[2], pgh[2], pdns[2], vol[2]]),
    ]
    s.prob = None   # "uniform" -> 1/S
    return s


def hydro_tree(scenario_name, fanouts=(50, 150, 300), seed=1134):
    """Non-uniform 3-stage hydro tree: stage-2 node b has fanouts[b] leaves, cond.
    prob 1/B; inflow A2 ~ U[10,90] per node, A3 ~ U[40,60] per leaf, ``default_rng(seed)`` drawing the
    B node values then the leaf values (ranges: ``PySP/scenariodata/Scen1.dat:30-33``)."""
    rng = np.random.default_rng(seed)
    B = len(fanouts)
    a2 = rng.uniform(10.0, 90.0, size=B)
    a3 = rng.uniform(40.0, 60.0, size=int(sum(fanouts)))
    k = extract_num(scenario_name) - 1
    b = int(np.searchsorted(np.cumsum(fanouts), k, side="right"))
    s = hydro(scenario_name, inflow=(float(a2[b]), float(a3[k])))
    s.nodes[1]["name"] = f"ROOT_{b}"
    s.nodes[1]["cond_prob"] = 1.0 / B
    s.prob = (1.0 / B) / fanouts[b]
    return s


def hydro_names(num_scens=9):
    return [f"Scen{i}" for i in range(1, num_scens + 1)]


# ------------------------------------------------------------------------------------------------
# sslp LP relaxation: examples/sslp/model/ReferenceModel.py + examples/sslp/sslp.py:26-46, data
# sslp_15_45_10 (npz extract of the reference .dat files, tools/make_example_data.py)
# ------------------------------------------------------------------------------------------------
_EXDATA = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-sppy_amd",
                       "examples", "data")


def _npz(name):
    z = np.load(os.path.join(_EXDATA, name))
    return {k: z[k] for k in z.files}


def sslp(scenario_name, penalty=1000.0, instance="sslp_15_45_10"):
    k = extract_num(scenario_name)
    d = _npz(f"{instance}.npz")
    P = d["client_present"]
    if 1 <= k <= P.shape[0]:
        present = P[k - 1].astype(float)
    else:   # synthetic scale-up: Bernoulli(mean presence), default_rng([1134, k])
        present = (np.random.default_rng([1134, k]).random(P.shape[1]) < P.mean(axis=0)).astype(float)
    ns, nc = d["fixed_cost"].shape[0], d["revenue"].shape[0]
    s = OScen(scenario_name)
    # columns in the reference's component order: FacilityOpen, Allocation, Dummy
    fo = {j: s.var(f"FacilityOpen[{j}]", 0.0, 1.0, float(d["fixed_cost"][j - 1])) for j in range(1, ns + 1)}
    al = {}
    for i in range(1, nc + 1):
        for j in range(1, ns + 1):
            al[i, j] = s.var(f"Allocation[({i}, {j})]", 0.0, 1.0, -float(d["revenue"][i - 1, j - 1]))
    du = {j: s.var(f"Dummy[{j}]", 0.0, INF, penalty) for j in range(1, ns + 1)}
    cap = float(d["capacity"])
    for j in range(1, ns + 1):   # Demand . Allocation - Dummy <= Capacity FacilityOpen
        co = {al[i, j]: float(d["demand"][i - 1, j - 1]) for i in range(1, nc + 1)
              if d["demand"][i - 1, j - 1] != 0.0}
        co[du[j]] = -1.0
        co[fo[j]] = -cap
        s.row(co, -INF, 0.0, f"DemandConstraint[{j}]")
    for i in range(1, nc + 1):
        s.row({al[i, j]: 1.0 for j in range(1, ns + 1)}, present[i - 1], present[i - 1], f"ClientConstraint[{i}]")
    s.nodes = [dict(name="ROOT", cond_prob=1.0, stage=1, cols=[fo[j] for j in range(1, ns + 1)])]
    s.prob = None
    return s


def sslp_names(num_scens, start=1):
    return [f"Scenario{i}" for i in range(start, start + num_scens)]


# ------------------------------------------------------------------------------------------------
# netdes LP relaxation: examples/netdes/netdes.py:39-80 + parse.py, instance network-50-30-H-01
# ------------------------------------------------------------------------------------------------
def netdes(scenario_name, num_scens=None, instance="network-50-30-H-01"):
    k = extract_num(scenario_name)
    d = _npz(f"{instance}.npz")
    K = d["p"].shape[0]
    base = k % K
    dk, uk, bk = d["d"][base].copy(), d["u"][base].copy(), d["b"][base]
    if k >= K:   # synthetic scale-up (documented in mpi-sppy_amd/examples/netdes.py)
        rng = np.random.default_rng([1134, k])
        dk = dk * rng.uniform(0.9, 1.1, dk.shape[0])
        uk = uk * rng.uniform(1.0, 1.1, uk.shape[0])
    E = [tuple(int(v) for v in e) for e in d["edges"]]
    s = OScen(scenario_name)
    x = [s.var(f"x[{e}]", 0.0, 1.0, float(d["c"][t])) for t, e in enumerate(E)]
    y = [s.var(f"y[{e}]", 0.0, INF, float(dk[t])) for t, e in enumerate(E)]
    for t in range(len(E)):
        s.row({y[t]: 1.0, x[t]: -float(uk[t])}, -INF, 0.0, f"vubs[{t + 1}]")
    for i in range(int(d["N"])):
        co = {}
        for t, (a, b) in enumerate(E):
            if a == i:
                co[y[t]] = co.get(y[t], 0.0) + 1.0
            if b == i:
                co[y[t]] = co.get(y[t], 0.0) - 1.0
        s.row(co, float(bk[i]), float(bk[i]), f"bals[{i + 1}]")
    s.nodes = [dict(name="ROOT", cond_prob=1.0, stage=1, cols=list(x))]
    s.prob = float(d["p"][base]) if (num_scens is None or num_scens == K) and k < K else 1.0 / num_scens
    return s


def netdes_names(num_scens, start=0):
    return [f"Scenario{i}" for i in range(start, start + num_scens)]


# ------------------------------------------------------------------------------------------------
# uc: synthetic UC-shaped LP relaxation (the reference's examples/uc needs egret,
# absent) -- restated independently of mpi-sppy_amd/examples/uc.py from the same formulas
# ------------------------------------------------------------------------------------------------
def uc(scenario_name, num_gens=85, num_periods=48, num_scens=None):
    k = extract_num(scenario_name)
    G, T = int(num_gens), int(num_periods)
    rng = np.random.default_rng(1134)
    pmax = rng.uniform(50.0, 400.0, G)
    mc = rng.uniform(10.0, 60.0, G)
    sc = rng.uniform(200.0, 2000.0, G)
    u0 = (np.arange(G) % 2 == 0).astype(float)
    tt = np.arange(T)
    dbase = 0.6 * pmax.sum() * (0.8 + 0.2 * np.sin(2.0 * np.pi * tt / T))
    srng = np.random.default_rng([1134, k])
    dem = dbase * (1.0 + 0.05 * srng.standard_normal(T))
    avail = np.where(srng.random((G, T)) < 0.05, 0.8, 1.0)
    pmin, ramp, nl = 0.3 * pmax, 0.5 * pmax, 0.1 * mc * pmax
    s = OScen(scenario_name)
    idx = [(g, t) for g in range(G) for t in range(T)]
    u = {gt: s.var(f"UnitOn[{gt}]", 0.0, 1.0, nl[gt[0]]) for gt in idx}
    p = {gt: s.var(f"PowerGenerated[{gt}]", 0.0, INF, mc[gt[0]]) for gt in idx}
    su = {gt: s.var(f"StartUp[{gt}]", 0.0, 1.0, sc[gt[0]]) for gt in idx}
    sd = {gt: s.var(f"ShutDown[{gt}]", 0.0, 1.0, 0.0) for gt in idx}
    r = {gt: s.var(f"Reserve[{gt}]", 0.0, INF, 0.0) for gt in idx}
    for g, t in idx:
        s.row({p[(g, t)]: 1.0, r[(g, t)]: 1.0, u[(g, t)]: -avail[g, t] * pmax[g]}, -INF, 0.0)
    for g, t in idx:
        s.row({p[(g, t)]: 1.0, u[(g, t)]: -pmin[g]}, 0.0, INF)
    for g, t in idx:
        co = {u[(g, t)]: 1.0, su[(g, t)]: -1.0, sd[(g, t)]: 1.0}
        if t > 0:
            co[u[(g, t - 1)]] = -1.0
            s.row(co, 0.0, 0.0)
        else:
            s.row(co, u0[g], u0[g])
    for g, t in idx:
        if t > 0:
            s.row({p[(g, t)]: 1.0, p[(g, t - 1)]: -1.0}, -INF, ramp[g])
    for g, t in idx:
        if t > 0:
            s.row({p[(g, t - 1)]: 1.0, p[(g, t)]: -1.0}, -INF, ramp[g])
    for t in range(T):
        s.row({p[(g, t)]: 1.0 for g in range(G)}, dem[t], dem[t])
    for t in range(T):
        s.row({r[(g, t)]: 1.0 for g in range(G)}, 0.03 * dem[t], INF)
    s.nodes = [dict(name="ROOT", cond_prob=1.0, stage=1, cols=[u[k2] for k2 in sorted(u)])]
    if num_scens is not None:
        s.prob = 1.0 / num_scens
    return s


def uc_names(num_scens, start=1):
    return [f"Scenario{i}" for i in range(start, start + num_scens)]
