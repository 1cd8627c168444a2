"""SSLP (stochastic server location) LP relaxation, restating ``examples/sslp/sslp.py:26-46`` and
``examples/sslp/model/ReferenceModel.py`` with the sslp_15_45_10 data
(``examples/sslp/data/sslp_15_45_10/scenariodata/Scenario{1..10}.dat``, extracted to
``examples/data/sslp_15_45_10.npz`` by ``tools/make_example_data.py``) or, with
``instance="sslp_5_25_50"`` (or the reference's ``data_dir`` naming it), the held-out 5-server,
25-client, 50-scenario instance.

Model (integrality relaxed -- the batched engine solves LP/QP subproblems; the reference's own
PH on sslp solves MIPs, so LP-relaxation parity is pinned by the CPU oracle only):
    min  sum_j FixedCost_j FacilityOpen_j + Penalty sum_j Dummy_j - sum_ij Revenue_ij Allocation_ij
    s.t. sum_i Demand_ij Allocation_ij - Dummy_j - Capacity FacilityOpen_j <= 0     (per server j)
         sum_j Allocation_ij = ClientPresent_i                                      (per client i)
         0 <= FacilityOpen, Allocation <= 1,  Dummy >= 0
Nonants: FacilityOpen[1..NumServers] (ROOT).  Scenario ``Scenario<k>``: k <= 10 uses the file's
ClientPresent; k > (the instance's scenario files) (synthetic scale-up) draws ClientPresent_i ~
Bernoulli(mean over the 10 files) from ``numpy.random.default_rng([1134, k])`` -- per scenario, so
every rank builds its own scenarios independently.  Probability: uniform (1/S).
"""
import os
import re

import numpy as np

from .. import model as lm
from ..scenario_tree import ScenarioNode

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
DEFAULT_INSTANCE = "sslp_15_45_10"
_CACHE = {}


def _data(instance=None):
    """The instance's data (``instance``: sslp_15_45_10, or the held-out sslp_5_25_50 --
    examples/sslp/data/<instance>; the reference picks it by ``data_dir``)."""
    inst = instance or DEFAULT_INSTANCE
    if inst not in _CACHE:
        z = np.load(os.path.join(_DIR, f"{inst}.npz"))
        _CACHE[inst] = {k: z[k] for k in z.files}
    return _CACHE[inst]


def _instance_of(data_dir, instance):
    if instance:
        return instance
    if data_dir:   # the reference's data_dir, e.g. .../sslp/data/sslp_5_25_50/scenariodata
        for part in reversed(os.path.normpath(data_dir).split(os.sep)):
            if part.startswith("sslp_"):
                return part
    return DEFAULT_INSTANCE


def client_present(k, instance=None):
    d = _data(instance)
    P = d["client_present"]
    if 1 <= k <= P.shape[0]:
        return P[k - 1].astype(float)
    rng = np.random.default_rng([1134, k])
    return (rng.random(P.shape[1]) < P.mean(axis=0)).astype(float)


def scenario_creator(scenario_name, data_dir=None, penalty=1000.0, instance=None):
    k = int(re.search(r"(\d+)$", scenario_name).group(1))
    inst = _instance_of(data_dir, instance)
    d = _data(inst)
    ns, nc = d["fixed_cost"].shape[0], d["revenue"].shape[0]
    servers = range(1, ns + 1)
    clients = range(1, nc + 1)
    present = client_present(k, inst)
    m = lm.LinearModel(scenario_name)
    fo = m.add_var("FacilityOpen", list(servers), (0.0, 1.0))
    al = m.add_var("Allocation", [(i, j) for i in clients for j in servers], (0.0, 1.0))
    du = m.add_var("Dummy", list(servers), (0.0, None))
    cap = float(d["capacity"])
    for j in servers:
        co = [(al[(i, j)], float(d["demand"][i - 1, j - 1])) for i in clients if d["demand"][i - 1, j - 1] != 0.0]
        co += [(du[j], -1.0), (fo[j], -cap)]
        m.add_row(co, None, 0.0, f"DemandConstraint[{j}]")
    for i in clients:
        m.add_row([(al[(i, j)], 1.0) for j in servers], present[i - 1], present[i - 1], f"ClientConstraint[{i}]")
    obj = [(fo[j], float(d["fixed_cost"][j - 1])) for j in servers]
    obj += [(du[j], penalty) for j in servers]
    obj += [(al[(i, j)], -float(d["revenue"][i - 1, j - 1])) for i in clients for j in servers
            if d["revenue"][i - 1, j - 1] != 0.0]
    m.set_objective(obj, lm.minimize)
    m._mpisppy_node_list = [ScenarioNode("ROOT", 1.0, 1, None, [m.FacilityOpen], m)]
    m._mpisppy_probability = "uniform"
    return m


def scenario_names_creator(num_scens, start=None):
    start = 1 if start is None else start
    return [f"Scenario{i}" for i in range(start, start + num_scens)]


def scenario_denouement(rank, scenario_name, scenario):
    pass
