"""UC-shaped scenario LP: a seeded synthetic stand-in for ``examples/uc``.

The reference's unit-commitment example (``examples/uc/uc_funcs.py:22-24``) builds its scenario
models with egret, which is not installed here or on the GPU box, so its data cannot be read.  What
the hot path needs from it is its SHAPE: ~2e4 columns and rows per scenario, ~8e4 nonzeros, and
N = 4 080 nonanticipative commitment variables (``examples/test_data/uca_baseline/uc_funcs.npy``
holds 4 080 first-stage values).  This generator builds a unit-commitment LP relaxation of that
shape -- G = 85 generators x T = 48 periods -- from seeded synthetic data (parity unpinned against
the reference: only the oracle restatement ``oracle.models.uc`` checks it).

Per generator g and period t: UnitOn u in [0, 1] (the nonant, ROOT), Power p >= 0, StartUp and
ShutDown in [0, 1], Reserve r >= 0; cost  mc_g p + nl_g u + sc_g StartUp.
Rows: capacity  p + r - avail_{s,g,t} Pmax_g u <= 0;  minimum output  p - Pmin_g u >= 0;
commitment logic  u_t - u_{t-1} - StartUp_t + ShutDown_t = 0  (= u0_g at t = 0);
ramping  |p_t - p_{t-1}| <= R_g;  per period: demand  sum_g p = D_{s,t},
reserve  sum_g r >= 0.03 D_{s,t}.
Per scenario: demand (right-hand side) and a 5 % chance of a 20 % derate per (g, t) (matrix
entries) -- the scenario matrices differ, so the solver streams each scenario's values.
Generator data: ``numpy.random.default_rng(1134)``; scenario k: ``default_rng([1134, k])``.
"""
import re

import numpy as np

from .. import model as lm
from ..scenario_tree import ScenarioNode


def _gen_data(G, T):
    rng = np.random.default_rng(1134)
    pmax = rng.uniform(50.0, 400.0, G)
    mc = rng.uniform(10.0, 60.0, G)
    sc = rng.uniform(200.0, 2000.0, G)
    u0 = (np.arange(G) % 2 == 0).astype(float)
    t = np.arange(T)
    dbase = 0.6 * pmax.sum() * (0.8 + 0.2 * np.sin(2.0 * np.pi * t / T))
    return pmax, mc, sc, u0, dbase


def _scen_data(k, G, T, dbase):
    rng = np.random.default_rng([1134, k])
    dem = dbase * (1.0 + 0.05 * rng.standard_normal(T))
    avail = np.where(rng.random((G, T)) < 0.05, 0.8, 1.0)
    return dem, avail


def scenario_creator(scenario_name, num_gens=85, num_periods=48, num_scens=None):
    k = int(re.search(r"(\d+)$", scenario_name).group(1))
    G, T = int(num_gens), int(num_periods)
    pmax, mc, sc, u0, dbase = _gen_data(G, T)
    dem, avail = _scen_data(k, G, T, dbase)
    pmin = 0.3 * pmax
    ramp = 0.5 * pmax
    nl = 0.1 * mc * pmax
    idx = [(g, t) for g in range(G) for t in range(T)]
    m = lm.LinearModel(scenario_name)
    u = m.add_var("UnitOn", idx, (0.0, 1.0))
    p = m.add_var("PowerGenerated", idx, (0.0, None))
    su = m.add_var("StartUp", idx, (0.0, 1.0))
    sd = m.add_var("ShutDown", idx, (0.0, 1.0))
    r = m.add_var("Reserve", idx, (0.0, None))
    for g, t in idx:
        m.add_row([(p[(g, t)], 1.0), (r[(g, t)], 1.0), (u[(g, t)], -avail[g, t] * pmax[g])], None, 0.0,
                  f"Capacity[{g},{t}]")
    for g, t in idx:
        m.add_row([(p[(g, t)], 1.0), (u[(g, t)], -pmin[g])], 0.0, None, f"MinOutput[{g},{t}]")
    for g, t in idx:
        co = [(u[(g, t)], 1.0), (su[(g, t)], -1.0), (sd[(g, t)], 1.0)]
        if t > 0:
            co.append((u[(g, t - 1)], -1.0))
            m.add_row(co, 0.0, 0.0, f"Logic[{g},{t}]")
        else:
            m.add_row(co, u0[g], u0[g], f"Logic[{g},{t}]")
    for g, t in idx:
        if t > 0:
            m.add_row([(p[(g, t)], 1.0), (p[(g, t - 1)], -1.0)], None, ramp[g], f"RampUp[{g},{t}]")
    for g, t in idx:
        if t > 0:
            m.add_row([(p[(g, t - 1)], 1.0), (p[(g, t)], -1.0)], None, ramp[g], f"RampDown[{g},{t}]")
    for t in range(T):
        m.add_row([(p[(g, t)], 1.0) for g in range(G)], dem[t], dem[t], f"Demand[{t}]")
    for t in range(T):
        m.add_row([(r[(g, t)], 1.0) for g in range(G)], 0.03 * dem[t], None, f"ReserveReq[{t}]")
    obj = [(p[(g, t)], mc[g]) for g, t in idx] + [(u[(g, t)], nl[g]) for g, t in idx] + \
          [(su[(g, t)], sc[g]) for g, t in idx]
    m.set_objective(obj, lm.minimize)
    m._mpisppy_node_list = [ScenarioNode("ROOT", 1.0, 1, None, [m.UnitOn], m)]
    m._uc_shape = (G, T)
    m._mpisppy_probability = 1.0 / num_scens if num_scens else "uniform"
    return m


def scenario_rhos(scenario_instance, rho_scale_factor=0.1):
    """The reference UC's cost-based rho (``examples/uc/uc_funcs.py:112-132``, the setter
    ``uc_cylinders.py:93`` passes to PH): rho of UnitOn[g,t] = rho_scale_factor x the cost of running
    unit g at the midpoint of its output range -- egret's ComputeProductionCosts(avg_power) +
    MinimumProductionCost there, this model's mc_g avg_power + nl_g here."""
    G, T = scenario_instance._uc_shape
    pmax, mc, _, _, _ = _gen_data(G, T)
    pmin = 0.3 * pmax
    nl = 0.1 * mc * pmax
    avg_power = pmin + (pmax - pmin) / 2.0
    return [(scenario_instance.UnitOn[(g, t)], rho_scale_factor * (mc[g] * avg_power[g] + nl[g]))
            for t in range(T) for g in range(G)]


def rho_setter(scenario_instance, **kwargs):
    """``uc_funcs._rho_setter`` (``uc_funcs.py:112-114``)."""
    return scenario_rhos(scenario_instance, **kwargs)


def scenario_names_creator(num_scens, start=None):
    start = 1 if start is None else start
    return [f"Scenario{i}" for i in range(start, start + num_scens)]


def scenario_denouement(rank, scenario_name, scenario):
    pass
