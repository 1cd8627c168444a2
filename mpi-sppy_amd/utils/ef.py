"""Extensive forms of scenario groups as one :class:`~mpisppy_amd.model.LinearModel` -- the
subproblem of a bundle.

Restates ``create_EF`` / ``_create_EF_from_scen_dict`` (``mpisppy/utils/sputils.py:143-354``) on the
engine's standard-form models:

* every scenario's columns and rows are copied into one model (column names prefixed
  ``"<scenario>."``), in scenario order;
* objective = (sum_s p_s f_s) / (sum_s p_s) (``sputils.py:281-291``); offsets alike;
* one reference column per nonant (node name, position): the first scenario's column that carries
  it (``sputils.py:326-331``); every later scenario's copy is tied to it by a row
  ``x_s - x_ref = 0`` named ``_C_EF_[node,i,scenario]`` (``:332-338``), except where the variable is
  fixed (lower == upper) and ``nonant_for_fixed_vars`` is False;
* the EF's probability is the sum of the members' (``:275-284``); uniform members (no
  probability, or ``"uniform"``) get 1 / len(group) first, as the reference does;
* ``ref_vars[(node, i)]`` and ``_nlens`` as in the reference.

Every member must use the same tree-node names (two-stage: ROOT).  The EF carries no
``_mpisppy_node_list``; the bundler attaches one (ROOT over the reference columns).
"""
from ..model import INF, LinearModel, VarData


class _EFVar(VarData):
    __slots__ = ()


def create_EF(scenario_names, scenario_creator, scenario_creator_kwargs=None, EF_name=None,
              suppress_warnings=False, nonant_for_fixed_vars=True):
    """``sputils.create_EF`` (``sputils.py:143-222``) for LinearModel scenarios."""
    kw = scenario_creator_kwargs or {}
    scen_dict = {nm: scenario_creator(nm, **kw) for nm in scenario_names}
    if len(scen_dict) == 0:
        raise RuntimeError("create_EF() received empty scenario list")
    probs = [getattr(s, "_mpisppy_probability", None) for s in scen_dict.values()]
    if any(p is None or p == "uniform" for p in probs):
        if not suppress_warnings and not all(p == "uniform" for p in probs):
            print("WARNING: At least one scenario is missing _mpisppy_probability attribute. "
                  "Assuming equally-likely scenarios...")
        for s in scen_dict.values():
            s._mpisppy_probability = 1.0 / len(scen_dict)
    return create_EF_from_scen_dict(scen_dict, EF_name=EF_name, nonant_for_fixed_vars=nonant_for_fixed_vars)


def create_EF_from_scen_dict(scen_dict, EF_name=None, nonant_for_fixed_vars=True):
    """``sputils._create_EF_from_scen_dict`` (``sputils.py:225-354``)."""
    ef = LinearModel(EF_name or "EF")
    senses = {s.sense for s in scen_dict.values()}
    if len(senses) != 1:
        raise ValueError("Cannot build the extensive form: the scenarios' objective senses differ")
    ef.sense = senses.pop()
    ptot = sum(float(s._mpisppy_probability) for s in scen_dict.values())
    if ptot <= 0.0:
        raise ValueError("create_EF: the scenarios' probabilities sum to zero")
    ef._mpisppy_probability = ptot
    ef.ref_vars = {}
    ef._nlens = {}
    ef.scen_list = list(scen_dict)
    colmap = {}
    for sname, s in scen_dict.items():
        base = ef.n
        colmap[sname] = base
        p = float(s._mpisppy_probability) / ptot
        a = s.arrays()
        for j, nm in enumerate(s.column_names()):
            col = ef._new_col(f"{sname}.{nm}")
            ef._lo[col] = float(a["col_lo"][j])
            ef._hi[col] = float(a["col_hi"][j])
            ef._cost[col] = p * float(a["c"][j])
        ef.obj_offset += p * float(s.obj_offset)
        rp, ci, vals = a["rowptr"], a["colidx"], a["vals"]
        for i in range(s.m):
            d = {base + int(ci[q]): float(vals[q]) for q in range(rp[i], rp[i + 1])}
            ef._rows.append((d, float(a["row_lo"][i]), float(a["row_hi"][i]), f"{sname}.{s._rows[i][3]}"))
    for sname, s in scen_dict.items():
        base = colmap[sname]
        for nd in s._mpisppy_node_list:
            L = len(nd.nonant_vardata_list)
            if ef._nlens.setdefault(nd.name, L) != L:
                raise RuntimeError(f"Number of non-anticipative variables is not consistent at node {nd.name} "
                                   f"in scenario {sname}")
            for i, v in enumerate(nd.nonant_vardata_list):
                col = base + v.col
                fixed = ef._lo[col] == ef._hi[col]
                key = (nd.name, i)
                if key not in ef.ref_vars:
                    if nonant_for_fixed_vars or not fixed:
                        ef.ref_vars[key] = _EFVar(ef, col, ef._colnames[col])
                elif nonant_for_fixed_vars or not fixed:
                    ef._rows.append(({col: 1.0, ef.ref_vars[key].col: -1.0}, 0.0, 0.0,
                                     f"_C_EF_[{nd.name},{i},{sname}]"))
    return ef


def ef_nonants(ef):
    """(node name, i, value) of the reference columns (``sputils.ef_nonants``, ``:403-415``)."""
    for (ndn, i), var in ef.ref_vars.items():
        yield ndn, i, var.value


def ef_objective(ef, x):
    """EF objective at column values ``x`` (the model sense's value of the normalised objective)."""
    return ef.objective_value(x)


__all__ = ["create_EF", "create_EF_from_scen_dict", "ef_nonants", "ef_objective", "INF"]
