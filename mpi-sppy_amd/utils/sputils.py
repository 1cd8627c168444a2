"""Solution writers (restates ``mpisppy/utils/sputils.py:53-84``) and the hub <-> spoke flat
buffer layout (``mpisppy/cylinders/hub.py:286-290, 379-403, 580-616``; ``spoke.py:220-240``).

Writers take ``(file_name, scenario, bundling)`` like the reference's and read variable values from
the scenario model (``VarData.value``: the solution the engine loaded into it).

Flat buffers: the reference ships W / nonants between cylinders through MPI windows as one float64
array ``[values..., BestOuterBound, BestInnerBound, write_id]`` (hub -> spoke; ``padding=3``) and
``[bound, write_id]`` (spoke -> hub).  On one GPU the engine hands W / nonants over device-to-device
and never builds these arrays; :func:`hub_send_buffer` / :func:`read_spoke_buffer` produce and
consume them for interoperating with MPI-based cylinders (or recording a run in that format).
"""
import os

import numpy as np

from .. import _lib


def _root(scenario):
    root = scenario._mpisppy_node_list[0]
    assert root.name == "ROOT"
    return root


def _strip_bundle(name, bundling):
    if bundling:
        dot = name.find(".")
        assert dot >= 0
        name = name[dot + 1:]
    return name


def first_stage_nonant_npy_serializer(file_name, scenario, bundling):
    """ROOT nonants as a 1-d float array in an ``.npy`` file (``sputils.py:53-58``)."""
    np.save(file_name, np.fromiter((v.value for v in _root(scenario).nonant_vardata_list), float))


def first_stage_nonant_writer(file_name, scenario, bundling):
    """``var_name,value`` per ROOT nonant (``sputils.py:60-70``)."""
    with open(file_name, "w") as f:
        for v in _root(scenario).nonant_vardata_list:
            f.write(f"{_strip_bundle(v.name, bundling)},{v.value}\n")


def _sort_key(k):
    return (0, k) if not isinstance(k, tuple) else (1, k)


def scenario_tree_solution_writer(directory_name, scenario_name, scenario, bundling):
    """``<dir>/<scenario_name>.csv``: ``var_name,value`` for every variable of the scenario, in the
    reference's deterministic order (components by name, then indices sorted; ``sputils.py:72-84``)."""
    with open(os.path.join(directory_name, scenario_name + ".csv"), "w") as f:
        for blk in sorted(scenario._blocks, key=lambda b: b.name):
            keys = list(blk.keys())
            try:
                keys = sorted(keys, key=_sort_key)
            except TypeError:
                pass
            for k in keys:
                v = blk[k]
                f.write(f"{_strip_bundle(v.name, bundling)},{v.value}\n")


# ----------------------------------------------------------------------------- flat buffers
def hub_send_buffer(hub, what="W", write_id=0):
    """``[W or nonants (local scenarios x N)..., BestOuterBound, BestInnerBound, write_id]``."""
    e = hub.opt.engine
    vals = e.get(_lib.F_W if what == "W" else _lib.F_XN)
    buf = np.empty(vals.size + 3)
    buf[:-3] = vals
    buf[-3] = hub.BestOuterBound
    buf[-2] = hub.BestInnerBound
    buf[-1] = write_id
    return buf


def spoke_send_buffer(bound, write_id):
    """``[bound, write_id]`` (``spoke.py:220-240``: a bound spoke's window)."""
    return np.array([bound, float(write_id)])


def read_spoke_buffer(buf, last_write_id):
    """(bound, write_id, is_new): a value is new only if its write_id advanced (``hub.py:405-440``)."""
    wid = int(buf[-1])
    return float(buf[0]), wid, wid > last_write_id
