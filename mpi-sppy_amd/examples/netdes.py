"""Network design (fixed-charge multicommodity-free flow) LP relaxation, restating
``examples/netdes/netdes.py:24-80`` with the network-50-30-H-01 instance (``instance=
"network-10-20-H-01"`` or a reference ``path`` naming it: the held-out 10-node, 20-scenario one)
(``examples/netdes/data/network-50-30-H-01.dat``, extracted per edge to
``examples/data/network-50-30-H-01.npz`` by ``tools/make_example_data.py``).

    min  sum_e c_e x_e + sum_e d_e y_e
    s.t. y_e - u_e x_e <= 0                                    (vubs, per edge, edge order)
         sum_{(i,j)} y_ij - sum_{(j,i)} y_ji = b_i               (bals, per node)
         0 <= x_e <= 1 (binary relaxed),  y_e >= 0
Nonants: x over all edges (ROOT), edge order = row-major np.where(A > 0).  Scenario
``Scenario<k>`` (zero-based): k < K (the file's scenarios: 30) uses the file's d, u, b and
probability p_k (nonuniform); k >= K (synthetic scale-up) takes scenario k mod 30 with d x U[0.9, 1.1] and
u x U[1.0, 1.1] from ``numpy.random.default_rng([1134, k])`` and b unchanged (the flow balance must
keep sum b = 0; capacities only grow so the relaxation stays feasible).  ``num_scens`` other than
30 gives uniform probabilities 1/num_scens.
"""
import os
import re

import numpy as np

from .. import model as lm
from ..scenario_tree import attach_root_node

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
DEFAULT_INSTANCE = "network-50-30-H-01"
_CACHE = {}


def _data(instance=None):
    """The instance's data (``instance``: network-50-30-H-01, or the held-out network-10-20-H-01 --
    examples/netdes/data/<instance>.dat; the reference passes the file's ``path``)."""
    inst = instance or DEFAULT_INSTANCE
    if inst not in _CACHE:
        z = np.load(os.path.join(_DIR, f"{inst}.npz"))
        _CACHE[inst] = {k: z[k] for k in z.files}
    return _CACHE[inst]


def _instance_of(path, instance):
    if instance:
        return instance
    if path:
        return os.path.splitext(os.path.basename(path))[0]
    return DEFAULT_INSTANCE


def scenario_data(k, instance=None):
    d = _data(instance)
    K = d["p"].shape[0]
    base = k % K
    dk, uk, bk = d["d"][base].copy(), d["u"][base].copy(), d["b"][base].copy()
    if k >= K:
        rng = np.random.default_rng([1134, k])
        dk *= rng.uniform(0.9, 1.1, dk.shape[0])
        uk *= rng.uniform(1.0, 1.1, uk.shape[0])
    return dk, uk, bk, float(d["p"][base])


def scenario_creator(scenario_name, path=None, num_scens=None, instance=None):
    k = int(re.search(r"(\d+)$", scenario_name).group(1))
    inst = _instance_of(path, instance)
    d = _data(inst)
    edges = [(int(a), int(b)) for a, b in d["edges"]]
    N = int(d["N"])
    dk, uk, bk, pk = scenario_data(k, inst)
    m = lm.LinearModel(scenario_name)
    x = m.add_var("x", edges, (0.0, 1.0))
    y = m.add_var("y", edges, (0.0, None))
    for e, (i, j) in enumerate(edges):
        m.add_row([(y[(i, j)], 1.0), (x[(i, j)], -float(uk[e]))], None, 0.0, f"vubs[{e + 1}]")
    for i in range(N):
        co = [(y[(a, b)], 1.0) for (a, b) in edges if a == i]
        co += [(y[(a, b)], -1.0) for (a, b) in edges if b == i]
        m.add_row(co, float(bk[i]), float(bk[i]), f"bals[{i + 1}]")
    obj = [(x[e], float(d["c"][k_])) for k_, e in enumerate(edges)]
    obj += [(y[e], float(dk[k_])) for k_, e in enumerate(edges)]
    m.set_objective(obj, lm.minimize)
    K = d["p"].shape[0]
    m._mpisppy_probability = pk if (num_scens is None or num_scens == K) and k < K else 1.0 / num_scens
    attach_root_node(m, None, [m.x])
    return m


def scenario_names_creator(num_scens, start=None):
    start = 0 if start is None else start
    return [f"Scenario{i}" for i in range(start, start + num_scens)]


def scenario_denouement(rank, scenario_name, scenario):
    pass
