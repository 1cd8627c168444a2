"""3-stage hydro (restates ``examples/hydro/hydro.py:79-241`` with the data of
``examples/hydro/PySP/scenariodata/Scen{1..9}.dat``).

``scenario_creator(scenario_name, branching_factors, inflows=None)``: scenario ``Scen<k>``
(1-based); the stage-2 node is ``ROOT_{(k-1)//BF[1]}`` with cond. prob 1/BF[0]
(``hydro.py:187-215``); probability "uniform".  The nine data files differ only in the inflows
A[2] in {10,50,90} (by (k-1)//3) and A[3] in {40,50,60} (by (k-1)%3); ``inflows`` overrides (A2, A3)
for the synthetic non-uniform trees of BASELINE M3 (``synthetic_scenario_creator``).
"""
import functools

import numpy as np

from .. import model as lm
from ..scenario_tree import ScenarioNode
from .farmer import extract_num

_A2 = (10.0, 50.0, 90.0)
_A3 = (40.0, 50.0, 60.0)


def scenario_creator(scenario_name, branching_factors=None, data_path=None, inflows=None,
                     node_name=None, cond_prob=None):
    if branching_factors is None:
        raise ValueError("Hydro scenario_creator requires branching_factors")
    snum = extract_num(scenario_name)
    if inflows is None:
        a2, a3 = _A2[(snum - 1) // 3], _A3[(snum - 1) % 3]
    else:
        a2, a3 = inflows
    m = _instance(scenario_name, {1: 50.0, 2: a2, 3: a3})
    ndn = node_name if node_name is not None else "ROOT_" + str((snum - 1) // branching_factors[1])
    cp = cond_prob if cond_prob is not None else 1.0 / branching_factors[0]
    m._mpisppy_node_list = [
        ScenarioNode("ROOT", 1.0, 1, None, [m.Pgt[1], m.Pgh[1], m.PDns[1], m.Vol[1]], m),
        ScenarioNode(ndn, cp, 2, None, [m.Pgt[2], m.Pgh[2], m.PDns[2], m.Vol[2]], m,
                     parent_name="ROOT"),
    ]
    m._mpisppy_probability = "uniform"
    return m


def _instance(name, A):
    T = (1, 2, 3)
    D = {1: 90.0, 2: 160.0, 3: 110.0}
    u = {1: 0.6048, 2: 0.6048, 3: 1.2096}
    dur = {1: 168.0, 2: 168.0, 3: 336.0}
    V0, Tyear = 60.48, 8760.0
    betaGt, betaGh, betaDns = 1.0, 0.0, 10.0
    r = {t: (1 / 1.1) ** (dur[t] / Tyear) for t in T}
    m = lm.LinearModel(name)
    pgt = m.add_var("Pgt", T, (0.0, 100.0))
    pgh = m.add_var("Pgh", T, (0.0, 100.0))
    pdns = m.add_var("PDns", T, lambda v: (0.0, D[int(v.name[-2])]))
    vol = m.add_var("Vol", T, (0.0, 100.0))
    sl = m.add_var("sl", None, (0.0, None))
    sc = m.add_var("StageCost", T, (None, None))
    for t in T:
        row = [(sc[t], 1.0), (pgt[t], -r[t] * betaGt), (pgh[t], -r[t] * betaGh), (pdns[t], -r[t] * betaDns)]
        if t == 3:
            row.append((sl[None], -1.0))
        m.add_row(row, 0.0, 0.0, f"StageCostConstraint[{t}]")
    for t in T:
        m.add_row([(pgt[t], 1.0), (pgh[t], 1.0), (pdns[t], 1.0)], D[t], D[t], f"demand[{t}]")
    for t in T:
        row = [(vol[t], 1.0), (pgh[t], u[t])]
        rhs = u[t] * A[t]
        if t == 1:
            rhs += V0
        else:
            row.append((vol[t - 1], -1.0))
        m.add_row(row, None, rhs, f"conserv[{t}]")
    m.add_row([(sl[None], 1.0), (vol[3], 4166.67)], 4166.67 * V0, None, "fcfe")
    m.set_objective([(sc[t], 1.0) for t in T], lm.minimize)
    return m


@functools.lru_cache(maxsize=8)
def _synthetic_tree(fanouts, seed):
    """Inflows of a non-uniform 3-stage tree: A[2] ~ U[10, 90] per stage-2 node,
    A[3] ~ U[40, 60] per leaf (the ranges of the commented ``B`` table in
    ``examples/hydro/PySP/scenariodata/Scen1.dat:30-33``), numpy ``default_rng(seed)``, node draws
    first.  Leaves are numbered 1.. in node order."""
    rng = np.random.default_rng(seed)
    a2 = rng.uniform(10.0, 90.0, size=len(fanouts))
    a3 = rng.uniform(40.0, 60.0, size=int(sum(fanouts)))
    node_of = np.repeat(np.arange(len(fanouts)), fanouts)
    return a2, a3, node_of


def synthetic_fanouts(num_scens):
    """Stage-2 fan-outs 10 % / 30 % / 60 % of the leaves: 500 -> (50, 150, 300), 2000 -> (200, 600, 1200)."""
    f1, f2 = num_scens // 10, (3 * num_scens) // 10
    return (f1, f2, num_scens - f1 - f2)


def synthetic_scenario_creator(scenario_name, fanouts=(50, 150, 300), seed=1134):
    """Leaf ``Scen<k>`` of the non-uniform tree: stage-2 node ``ROOT_b`` (cond. prob 1/B), scenario
    probability (1/B)/fanouts[b]; same model as ``scenario_creator`` with that leaf's inflows."""
    fanouts = tuple(int(f) for f in fanouts)
    a2, a3, node_of = _synthetic_tree(fanouts, seed)
    k = extract_num(scenario_name) - 1
    b = int(node_of[k])
    B = len(fanouts)
    m = scenario_creator(scenario_name, branching_factors=[B, 1], inflows=(float(a2[b]), float(a3[k])),
                         node_name=f"ROOT_{b}", cond_prob=1.0 / B)
    m._mpisppy_probability = (1.0 / B) / fanouts[b]
    return m


def synthetic_nodenames(fanouts):
    return ["ROOT"] + [f"ROOT_{b}" for b in range(len(fanouts))]


def scenario_names_creator(num_scens, start=None):
    start = 1 if start is None else start
    return [f"Scen{i}" for i in range(start, start + num_scens)]


def scenario_denouement(rank, scenario_name, scenario):
    pass
