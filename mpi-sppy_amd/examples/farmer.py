"""Scalable farmer (restates ``examples/farmer/farmer.py:31-230`` and the identical data of
``mpisppy/tests/examples/farmer.py``), returning a :class:`~mpisppy_amd.model.LinearModel`.

Same keyword API: ``scenario_creator(scenario_name, use_integer=False, sense=minimize,
crops_multiplier=1, num_scens=None, seedoffset=0)``; scenario ``scen<k>``: base yields
Below/Average/Above by k % 3, group k // 3; ``RandomState.seed(k + seedoffset)`` and one ``rand()``
per crop in crop insertion order when group != 0 (``farmer.py:66,157-163``).
"""
import re

import numpy as np

from .. import model as lm
from ..scenario_tree import attach_root_node

farmerstream = np.random.RandomState()

_BASE = ("WHEAT", "CORN", "SUGAR_BEETS")
_DATA = dict(
    PriceQuota={"WHEAT": 100000.0, "CORN": 100000.0, "SUGAR_BEETS": 6000.0},
    SubQuotaSellingPrice={"WHEAT": 170.0, "CORN": 150.0, "SUGAR_BEETS": 36.0},
    SuperQuotaSellingPrice={"WHEAT": 0.0, "CORN": 0.0, "SUGAR_BEETS": 10.0},
    CattleFeedRequirement={"WHEAT": 200.0, "CORN": 240.0, "SUGAR_BEETS": 0.0},
    PurchasePrice={"WHEAT": 238.0, "CORN": 210.0, "SUGAR_BEETS": 100000.0},
    PlantingCostPerAcre={"WHEAT": 150.0, "CORN": 230.0, "SUGAR_BEETS": 260.0},
)
_YIELD = {
    "BelowAverageScenario": {"WHEAT": 2.0, "CORN": 2.4, "SUGAR_BEETS": 16.0},
    "AverageScenario": {"WHEAT": 2.5, "CORN": 3.0, "SUGAR_BEETS": 20.0},
    "AboveAverageScenario": {"WHEAT": 3.0, "CORN": 3.6, "SUGAR_BEETS": 24.0},
}


def extract_num(s):
    return int(re.compile(r"(\d+)$").search(s).group(1))


def scenario_creator(scenario_name, use_integer=False, sense=lm.minimize, crops_multiplier=1,
                     num_scens=None, seedoffset=0):
    if use_integer:
        raise NotImplementedError("integer farmer: the batched engine solves LP/QP relaxations only")
    if sense not in (lm.minimize, lm.maximize):
        raise ValueError("Model sense Not recognized")
    scennum = extract_num(scenario_name)
    basenames = ["BelowAverageScenario", "AverageScenario", "AboveAverageScenario"]
    basename = basenames[scennum % 3]
    groupnum = scennum // 3
    farmerstream.seed(scennum + seedoffset)
    model = _instance(basename, groupnum, sense, crops_multiplier)
    attach_root_node(model, None, [model.DevotedAcreage])
    if num_scens is not None:
        model._mpisppy_probability = 1 / num_scens
    return model


def _instance(basename, groupnum, sense, cm):
    crops = []
    for i in range(cm):
        for b in _BASE:
            crops.append(b + str(i))
    base = {c: c.rstrip("0123456789") for c in crops}
    yld = {}
    for c in crops:
        yld[c] = _YIELD[basename][base[c]] + (farmerstream.rand() if groupnum != 0 else 0.0)
    total = 500.0 * cm
    m = lm.LinearModel(f"{basename}{groupnum}")
    m.Yield = yld
    m.TOTAL_ACREAGE = total
    da = m.add_var("DevotedAcreage", crops, (0.0, total))
    qsub = m.add_var("QuantitySubQuotaSold", crops, (0.0, None))
    qsup = m.add_var("QuantitySuperQuotaSold", crops, (0.0, None))
    qp = m.add_var("QuantityPurchased", crops, (0.0, None))
    m.add_row([(da[c], 1.0) for c in crops], None, total, "ConstrainTotalAcreage")
    for c in crops:
        m.add_row([(da[c], yld[c]), (qp[c], 1.0), (qsub[c], -1.0), (qsup[c], -1.0)],
                  _DATA["CattleFeedRequirement"][base[c]], None, f"EnforceCattleFeedRequirement[{c}]")
    for c in crops:
        m.add_row([(qsub[c], 1.0), (qsup[c], 1.0), (da[c], -yld[c])], None, 0.0, f"LimitAmountSold[{c}]")
    for c in crops:
        m.add_row([(qsub[c], 1.0)], 0.0, _DATA["PriceQuota"][base[c]], f"EnforceQuotas[{c}]")
    sg = 1.0 if sense == lm.minimize else -1.0
    obj = []
    for c in crops:
        obj.append((da[c], sg * _DATA["PlantingCostPerAcre"][base[c]]))
        obj.append((qp[c], sg * _DATA["PurchasePrice"][base[c]]))
        obj.append((qsub[c], -sg * _DATA["SubQuotaSellingPrice"][base[c]]))
        obj.append((qsup[c], -sg * _DATA["SuperQuotaSellingPrice"][base[c]]))
    m.set_objective(obj, sense)
    return m


def scenario_names_creator(num_scens, start=None):
    start = 0 if start is None else start
    return [f"scen{i}" for i in range(start, start + num_scens)]


def kw_creator(cfg):
    get = cfg.get if hasattr(cfg, "get") else (lambda k, d=None: getattr(cfg, k, d))
    return {"use_integer": get("farmer_with_integers", False) or False,
            "crops_multiplier": get("crops_multiplier", 1) or 1,
            "num_scens": get("num_scens", None)}


def scenario_denouement(rank, scenario_name, scenario):
    pass
