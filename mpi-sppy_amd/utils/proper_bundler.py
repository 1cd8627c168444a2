"""Proper bundles: scenario groups solved as ONE subproblem (their extensive form).

Restates ``mpisppy/utils/proper_bundler.py:29-122`` for the engine's LinearModel scenarios: a
wrapped model module whose ``scenario_creator`` returns, for a name ``Bundle_<first>_<last>``, the EF
of scenarios first..last (:func:`mpisppy_amd.utils.ef.create_EF`) with a ROOT node over its
reference nonant columns; for a scenario name, the scenario itself.  Two-stage only, as in the
reference ("Multi-stage ... not supported", ``proper_bundler.py:21``).  PH then runs over the
bundles exactly as over scenarios: every bundle of a batch has the same sparsity pattern when the
member scenarios do, so bundles are one more batch for the GPU engine.

Not restated: reading / writing dill-pickled bundles (``pickle_bundle.py``): the engine does not
unpickle model files.
"""
import re

from ..scenario_tree import attach_root_node
from .ef import create_EF


def extract_num(name):
    """Trailing integer of a scenario name (``sputils.extract_num``)."""
    return int(re.compile(r"(\d+)$").search(name).group(1))


class ProperBundler:
    """Wrap a model module (``scenario_creator``, ``scenario_names_creator``, ``kw_creator``) so that
    bundle names create bundles.  ``cfg`` is any mapping with ``num_scens`` and
    ``scenarios_per_bundle``."""

    def __init__(self, module, comm=None):
        self.module = module
        self.comm = comm
        self.original_kwargs = {}

    def scenario_names_creator(self, num_scens, start=None, cfg=None):
        return self.module.scenario_names_creator(num_scens, start=start)

    def bundle_names_creator(self, num_buns, start=None, cfg=None):
        """``proper_bundler.py:51-62``: Bundle_<first>_<last>, numbered like the scenarios."""
        start = 0 if start is None else start
        if cfg is None or cfg.get("num_scens") is None or cfg.get("scenarios_per_bundle") is None:
            raise ValueError("ProperBundler needs cfg with num_scens and scenarios_per_bundle")
        bsize = int(cfg["scenarios_per_bundle"])
        if int(cfg["num_scens"]) % bsize != 0:
            raise ValueError("num_scens must be a multiple of scenarios_per_bundle")
        inum = extract_num(self.module.scenario_names_creator(1)[0])
        return [f"Bundle_{bn * bsize + inum}_{(bn + 1) * bsize - 1 + inum}" for bn in range(start, start + num_buns)]

    def kw_creator(self, cfg):
        kw = self.module.kw_creator(cfg) if hasattr(self.module, "kw_creator") else {}
        self.original_kwargs = dict(kw)
        return dict(kw, cfg=cfg)

    def set_kwargs(self, kwargs):
        """The member scenarios' creator kwargs when no cfg / kw_creator is used."""
        self.original_kwargs = dict(kwargs)

    def scenario_creator(self, sname, **kwargs):
        """``proper_bundler.py:73-122``."""
        kw = {k: v for k, v in kwargs.items() if k != "cfg"}
        if "scen" in sname or "Scen" in sname:
            return self.module.scenario_creator(sname, **{**self.original_kwargs, **kw})
        if "Bundle" not in sname:
            raise RuntimeError(f"Scenario name does not have scen or Bundle: {sname}")
        first, last = (int(t) for t in sname.split("_")[1:3])
        snames = self.module.scenario_names_creator(last - first + 1, first)
        ckw = {**self.original_kwargs, **kw}
        bundle = create_EF(snames, self.module.scenario_creator, scenario_creator_kwargs=ckw, EF_name=sname,
                           suppress_warnings=True, nonant_for_fixed_vars=False)
        nonants = [v for (ndn, _i), v in sorted(bundle.ref_vars.items(), key=lambda t: t[0][1]) if ndn == "ROOT"]
        scen = self.module.scenario_creator(snames[0], **ckw)
        bprob = "uniform" if getattr(scen, "_mpisppy_probability", None) == "uniform" else bundle._mpisppy_probability
        attach_root_node(bundle, 0, nonants)
        bundle._mpisppy_probability = bprob
        return bundle


def bundle_scenarios(names, bundles):
    """Split ``names`` into ``bundles`` contiguous groups (``spbase.py:_assign_bundles``, :223-257:
    group i holds names[int(i * avg): int((i + 1) * avg)], avg = len / bundles)."""
    if bundles > len(names):
        raise RuntimeError("Not enough scenarios to satisfy the bundles_per_rank requirement")
    avg = len(names) / bundles
    return [names[int(i * avg):int((i + 1) * avg)] for i in range(bundles)]
