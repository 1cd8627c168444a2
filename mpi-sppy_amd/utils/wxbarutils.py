"""W and xbar CSV files (restates ``mpisppy/utils/wxbarutils.py:47-389``).

Formats, as the reference writes and reads them:

* W, one file:      ``scen_name,var_name,value`` per local nonant, gathered to rank 0 and APPENDED
                    (``wxbarutils.py:47-89``);
* W, per scenario:  ``<dir>/<scen_name>_weights.csv`` with ``var_name,value`` rows (overwritten);
* xbar:             ``var_name,value`` for the nonants of the first local scenario, rank 0 only,
                    appended (``:276-296``);
* ROOT xbar npy:    ``numpy.savetxt`` of the ROOT node's xbar (``:378-389``).

Readers skip lines starting with ``#``; variable names may contain commas (everything between the
first and last field).  Values go to / come from the engine's device arrays (W is S x N per rank,
xbar / xsqbar are per tree node), so a file written here loads into the reference and vice versa.
"""
import os

import numpy as np

from .. import _lib


def _nonant_names(scenario):
    return [v.name for nd in scenario._mpisppy_node_list for v in nd.nonant_vardata_list]


def _fmt(val):
    return str(float(val))      # shortest round-trip repr, as the reference's str(pyo.value(.))


# ----------------------------------------------------------------------------------------- W
def write_W_to_file(PHB, fname, sep_files=False):
    W = PHB.Ws()
    if sep_files:
        for k, (sname, s) in enumerate(PHB.local_scenarios.items()):
            with open(os.path.join(fname, sname + "_weights.csv"), "w") as f:
                for vname, val in zip(_nonant_names(s), W[k]):
                    f.write(f"{vname},{_fmt(val)}\n")
        return
    local = [(sname, vname, float(val))
             for k, (sname, s) in enumerate(PHB.local_scenarios.items())
             for vname, val in zip(_nonant_names(s), W[k])]
    allw = PHB.comms["ROOT"].gather_object(local, root=0)
    if PHB.cylinder_rank == 0:
        with open(fname, "a") as f:
            for part in allw:
                for sname, vname, val in part:
                    f.write(f"{sname},{vname},{_fmt(val)}\n")


def _parse_W_csv_single(fname):
    if not os.path.exists(fname):
        raise RuntimeError(f"Could not find file {fname}")
    out = {}
    with open(fname) as f:
        for line in f:
            if line.startswith("#"):
                continue
            parts = line.split(",")
            out[",".join(parts[:-1])] = float(parts[-1])
    return out


def _parse_W_csv(fname, scenario_names_local, scenario_names_global, rank):
    glob = set(scenario_names_global)
    loc = set(scenario_names_local)
    out = {}
    with open(fname) as f:
        for line in f:
            if line.startswith("#"):
                continue
            parts = line.split(",")
            sname, vname, val = parts[0], ",".join(parts[1:-1]), float(parts[-1])
            if sname not in glob:
                if rank == 0:
                    print("WARNING: Ignoring unknown scenario name", sname)
                continue
            if sname in loc:
                out.setdefault(sname, {})[vname] = val
    missing = [s for s in scenario_names_local if s not in out]
    if missing:
        raise RuntimeError(f"rank {rank} could not find the following scenarios in the provided "
                           "weight file: " + ", ".join(missing))
    return out


def _check_W(w_val_dict, PHB, rank):
    """Missing variables raise, unknown ones are dropped with a warning, and the weights must be
    dual feasible: sum_s p_s w_s(var) = 0 within 1e-7 for every variable name (``:224-273``)."""
    for sname, s in PHB.local_scenarios.items():
        vn_model = _nonant_names(s)
        provided = w_val_dict[sname]
        miss = set(vn_model) - set(provided)
        if miss:
            raise RuntimeError(sname + " is missing the following variables: " + ", ".join(sorted(miss)))
        extra = set(provided) - set(vn_model)
        if extra:
            print("Removing unknown variables:", ", ".join(sorted(extra)))
            for v in extra:
                provided.pop(v, None)
    names = set().union(*[_nonant_names(s) for s in PHB.local_scenarios.values()])
    if PHB.n_proc > 1:   # multistage ranks see different nonant names: reduce over their union
        for other in PHB.comms["ROOT"].allgather_object(sorted(names)):
            names.update(other)
    names = sorted(names)
    local = np.array([sum(s._mpisppy_probability * w_val_dict[sn].get(v, 0.0)
                          for sn, s in PHB.local_scenarios.items()) for v in names])
    dual = PHB.comms["ROOT"].allreduce_array(local) if PHB.n_proc > 1 else local
    for v, d in zip(names, dual):
        if abs(d) > 1e-7:
            raise RuntimeError("Provided weights do not satisfy dual feasibility: "
                               "sum_{scenarios} prob(s) * w(s) != 0. Error on variable " + v)


def set_W_from_file(fname, PHB, rank, sep_files=False, disable_check=False):
    local_names = list(PHB.local_scenarios.keys())
    if sep_files:
        wd = {sn: _parse_W_csv_single(os.path.join(fname, sn + "_weights.csv")) for sn in local_names}
    else:
        wd = _parse_W_csv(fname, local_names, PHB.all_scenario_names, rank)
    if not disable_check:
        _check_W(wd, PHB, rank)
    W = PHB.Ws().copy()
    for k, (sname, s) in enumerate(PHB.local_scenarios.items()):
        d = wd.get(sname, {})
        for i, vname in enumerate(_nonant_names(s)):
            if vname in d:
                W[k, i] = d[vname]
    PHB.engine.set(_lib.F_W, W.ravel())


# -------------------------------------------------------------------------------------- xbar
def _scenario_xbar_slots(PHB, k):
    """(offset into the per-node xbar array, var name) for local scenario k's nonants."""
    b = PHB.engine.batch
    s = PHB.local_scenarios[PHB.local_scenario_names[k]]
    slots = []
    for lvl, nd in enumerate(s._mpisppy_node_list):
        off = int(b.node_off[b.scen_node[k, lvl]])
        slots.extend((off + i, v.name) for i, v in enumerate(nd.nonant_vardata_list))
    return slots


def write_xbar_to_file(PHB, fname):
    if PHB.cylinder_rank != 0:
        return
    xb = PHB.xbars()
    with open(fname, "a") as f:
        for off, vname in _scenario_xbar_slots(PHB, 0):
            f.write(f"{vname},{_fmt(xb[off])}\n")


def _parse_xbar_csv(fname):
    out = {}
    with open(fname) as f:
        for line in f:
            if line.startswith("#"):
                continue
            parts = line.split(",")
            out[",".join(parts[:-1])] = float(parts[-1])
    return out


def _check_xbar(xbar_val_dict, PHB):
    names = set(_nonant_names(PHB.local_scenarios[PHB.local_scenario_names[0]]))
    miss = names - set(xbar_val_dict)
    if miss:
        raise RuntimeError("Could not find the following required variable values in the provided "
                           "input file: " + ", ".join(sorted(miss)))
    extra = set(xbar_val_dict) - names
    if extra:
        print("Ignoring the following variables values provided in the input file: "
              + ", ".join(sorted(extra)))


def set_xbar_from_file(fname, PHB):
    """Sets xbar and xsqbar = xbar^2 of every local scenario's nodes (``:298-319``)."""
    vals = _parse_xbar_csv(fname)
    if PHB.cylinder_rank == 0:
        _check_xbar(vals, PHB)
    xb = PHB.engine.get(_lib.F_XBAR)
    for k in range(PHB.engine.S):
        for off, vname in _scenario_xbar_slots(PHB, k):
            if vname not in vals:
                raise RuntimeError(f"xbar file {fname} has no value for {vname}")
            xb[off] = vals[vname]
    PHB.engine.set(_lib.F_XBAR, xb)
    PHB.engine.set(_lib.F_XSQBAR, xb * xb)


def ROOT_xbar_npy_serializer(PHB, fname):
    b = PHB.engine.batch
    g = b.all_nodenames.index("ROOT")
    off = int(b.node_off[g])
    np.savetxt(fname, PHB.xbars()[off:off + int(b.level_len[0])])
