"""Scenario-tree nodes (restates ``mpisppy/scenario_tree.py:51-103``).

``ScenarioNode(name, cond_prob, stage, cost_expression, nonant_list, scen_model, ...)`` keeps the
reference constructor signature.  ``nonant_list`` entries are :class:`~mpisppy_amd.model.VarBlock`
(expanded over SORTED keys, as ``build_vardatalist`` does at ``scenario_tree.py:45-46``) or single
:class:`~mpisppy_amd.model.VarData`.  ``nonant_vardata_list`` is the ordered VarData list and
``nonant_cols`` the matching column indices (the index map the GPU batch is built from).
"""
from .model import VarBlock, VarData


def build_vardatalist(model, varlist):
    if varlist is None:
        raise RuntimeError("varlist is None in scenario_tree.build_vardatalist")
    if isinstance(varlist, (VarBlock, VarData)):
        varlist = [varlist]
    out = []
    for v in varlist:
        if isinstance(v, VarBlock) and v.is_indexed():
            out.extend(v[k] for k in sorted(v.keys()))
        elif isinstance(v, VarBlock):
            out.append(v[None])
        elif isinstance(v, VarData):
            out.append(v)
        else:
            raise TypeError(f"unsupported nonant entry {v!r}")
    return out


class ScenarioNode:
    def __init__(self, name, cond_prob, stage, cost_expression, nonant_list, scen_model,
                 nonant_ef_suppl_list=None, parent_name=None):
        self.name = name
        self.cond_prob = cond_prob
        self.stage = stage
        self.cost_expression = cost_expression
        self.nonant_list = nonant_list
        self.nonant_ef_suppl_list = nonant_ef_suppl_list
        self.parent_name = parent_name
        self.nonant_vardata_list = build_vardatalist(scen_model, nonant_list) \
            if nonant_list is not None else []
        self.nonant_ef_suppl_vardata_list = build_vardatalist(scen_model, nonant_ef_suppl_list) \
            if nonant_ef_suppl_list is not None else []
        self.uncond_prob = None

    @property
    def nonant_cols(self):
        return [v.col for v in self.nonant_vardata_list]


def attach_root_node(model, firstobj, varlist, nonant_ef_suppl_list=None, do_uniform=True):
    """``mpisppy/utils/sputils.py:860-881``."""
    model._mpisppy_node_list = [ScenarioNode("ROOT", 1.0, 1, firstobj, varlist, model,
                                             nonant_ef_suppl_list=nonant_ef_suppl_list)]
    if do_uniform and not hasattr(model, "_mpisppy_probability"):
        model._mpisppy_probability = "uniform"
