"""SPBase restated: scenario distribution, index maps and node bookkeeping.

Follows ``mpisppy/spbase.py`` (``SPBase.__init__`` :48-124, ``_calculate_scenario_ranks``
:188-220, ``_attach_nonant_indices`` :297-306, ``_attach_nlens`` :309-324,
``_compute_unconditional_node_probabilities`` :382-395, ``_look_and_leap`` :509-526) and
``_ScenTree.scen_names_to_ranks`` (``mpisppy/utils/sputils.py:790-856``).  The index maps are
bit-exact with the reference: scenario order, rank slices, ``(node_name, i)`` nonant keys in node
list order with sorted Var keys inside a node.
"""
import numpy as np

from .comm import SingleComm


def scen_names_to_ranks_slices(S, n_proc):
    """``sputils.py:819-826``: rank -> contiguous scenario index list."""
    if n_proc == 1:
        return [list(range(S))]
    avg = S / n_proc
    return [list(range(int(i * avg), int((i + 1) * avg))) for i in range(n_proc)]


def create_nodenames_from_branching_factors(bfs):
    """``sputils.py:992-1017``: non-leaf node names of a uniform tree."""
    stage_nodes = ["ROOT"]
    names = ["ROOT"]
    for bf in bfs[:-1]:
        nxt = []
        for nd in stage_nodes:
            for b in range(bf):
                nxt.append(f"{nd}_{b}")
        names.extend(nxt)
        stage_nodes = nxt
    return names


class SPBase:
    def __init__(self, options, all_scenario_names, scenario_creator, scenario_denouement=None,
                 all_nodenames=None, mpicomm=None, scenario_creator_kwargs=None,
                 variable_probability=None, E1_tolerance=1e-5):
        self.options = options
        self.all_scenario_names = list(all_scenario_names)
        self.scenario_creator = scenario_creator
        self.scenario_denouement = scenario_denouement
        self.all_nodenames = list(all_nodenames) if all_nodenames is not None else ["ROOT"]
        self.mpicomm = mpicomm if mpicomm is not None else SingleComm()
        self.comms = {"ROOT": self.mpicomm}
        self.n_proc = self.mpicomm.Get_size()
        self.cylinder_rank = self.mpicomm.Get_rank()
        self.global_rank = self.cylinder_rank
        self.E1_tolerance = E1_tolerance
        self.variable_probability = variable_probability
        self.bundling = bool(options.get("bundles_per_rank", 0))
        if self.bundling:
            self._setup_loose_bundles(scenario_creator, scenario_creator_kwargs or {})
        self._calculate_scenario_ranks()
        self._create_scenarios(scenario_creator_kwargs or {})
        self._look_and_leap()
        self._compute_unconditional_node_probabilities()
        self._attach_nlens()
        self._attach_nonant_indices()
        self._verify_nonant_lengths()
        self._use_variable_probability_setter()
        self._set_sense()
        self._spcomm = None

    # ---------------------------------------------------------------------------------------
    def _calculate_scenario_ranks(self):
        S = len(self.all_scenario_names)
        self._rank_slices = scen_names_to_ranks_slices(S, self.n_proc)
        self._scenario_slices = [r for r, sl in enumerate(self._rank_slices) for _ in sl]
        self.local_scenario_names = [self.all_scenario_names[i] for i in self._rank_slices[self.cylinder_rank]]
        self.scen_global0 = self._rank_slices[self.cylinder_rank][0] if self._rank_slices[self.cylinder_rank] else 0

    def _setup_loose_bundles(self, scenario_creator, kw):
        """``bundles_per_rank`` (``spbase.py:223-257`` _assign_bundles, ``spopt.py:840-873``
        _subproblem_creation): each rank's scenarios are split into that many contiguous groups and
        each group is solved as one subproblem, its extensive form (``utils/ef.py``).  Here the
        bundles then take the scenarios' place in the batch (named ``rank<r>bundle<b>`` as in the
        reference, probability = the members' sum): the members of a bundle share one nonant copy,
        so their W / x-bar updates coincide and PH over the bundles is PH over the scenarios with
        every member's nonants equal.  The reference's convergence metric counts SCENARIOS
        (``phbase.py:349-371`` loops over local_scenarios, not the bundles); weighing each bundle once
        is that count only when the bundles are equal-sized, so unequal bundle sizes are rejected
        (ValueError) rather than silently changing conv and the convthresh stopping iteration.
        Two-stage trees only."""
        from .utils.ef import create_EF_from_scen_dict
        from .utils.proper_bundler import bundle_scenarios
        from .scenario_tree import attach_root_node
        bpr = int(self.options["bundles_per_rank"])
        S = len(self.all_scenario_names)
        if self.n_proc * bpr > S:
            raise RuntimeError("Not enough scenarios to satisfy the bundles_per_rank requirement")
        slices = scen_names_to_ranks_slices(S, self.n_proc)
        self.names_in_bundles = {}
        bundle_names = []
        for r, slc in enumerate(slices):
            groups = bundle_scenarios([self.all_scenario_names[i] for i in slc], bpr)
            self.names_in_bundles[r] = dict(enumerate(groups))
            bundle_names += [f"rank{r}bundle{b}" for b in range(bpr)]
        sizes = {len(g) for r in self.names_in_bundles for g in self.names_in_bundles[r].values()}
        if len(sizes) > 1:
            raise ValueError(f"bundles_per_rank={bpr} over {S} scenarios and {self.n_proc} rank(s) gives "
                             f"bundles of unequal sizes {sorted(sizes)}: the convergence metric would weigh "
                             "them differently from the reference's per-scenario count; choose "
                             "bundles_per_rank * n_proc dividing the scenario count")
        members = {nm: grp for r in range(self.n_proc) for nm, grp in
                   zip(bundle_names[r * bpr:(r + 1) * bpr], self.names_in_bundles[r].values())}
        self.all_scenario_names_unbundled = self.all_scenario_names
        self.all_scenario_names = bundle_names

        def bundle_creator(bname, **ckw):
            sdict = {}
            for sname in members[bname]:
                sc = scenario_creator(sname, **ckw)
                if len(sc._mpisppy_node_list) != 1:
                    raise RuntimeError("bundles_per_rank: two-stage scenario trees only")
                if getattr(sc, "_mpisppy_probability", None) in (None, "uniform"):
                    sc._mpisppy_probability = 1.0 / S
                sdict[sname] = sc
            ef = create_EF_from_scen_dict(sdict, EF_name=bname, nonant_for_fixed_vars=False)
            nonants = [v for (ndn, _i), v in sorted(ef.ref_vars.items(), key=lambda t: t[0][1]) if ndn == "ROOT"]
            attach_root_node(ef, 0, nonants)
            ef._mpisppy_probability = sum(float(sc._mpisppy_probability) for sc in sdict.values())
            return ef

        self.scenario_creator = bundle_creator

    def _create_scenarios(self, kw):
        self.local_scenarios = {}
        for sname in self.local_scenario_names:
            s = self.scenario_creator(sname, **kw)
            self.local_scenarios[sname] = s
        self.local_subproblems = self.local_scenarios
        self.scenarios_constructed = True

    def _look_and_leap(self):
        S = len(self.all_scenario_names)
        for sname, s in self.local_scenarios.items():
            pspec = getattr(s, "_mpisppy_probability", None)
            if pspec is None or pspec == "uniform":
                s._mpisppy_probability = 1.0 / S
            if not hasattr(s, "_mpisppy_node_list"):
                raise RuntimeError(f"_mpisppy_node_list not found on scenario {sname}")
            if not hasattr(s, "_mpisppy_data"):
                s._mpisppy_data = type("MpisppyData", (), {})()

    def _compute_unconditional_node_probabilities(self):
        for s in self.local_scenarios.values():
            nodes = s._mpisppy_node_list
            nodes[0].uncond_prob = 1.0
            for parent, child in zip(nodes[:-1], nodes[1:]):
                child.uncond_prob = parent.uncond_prob * child.cond_prob
            s._mpisppy_data.prob_coeff = {nd.name: s._mpisppy_probability / nd.uncond_prob for nd in nodes}
            s._mpisppy_data.prob0_mask = {nd.name: 1.0 for nd in nodes}
            s._mpisppy_data.has_variable_probability = False

    def _attach_nlens(self):
        for s in self.local_scenarios.values():
            s._mpisppy_data.nlens = {nd.name: len(nd.nonant_vardata_list) for nd in s._mpisppy_node_list}
            s._mpisppy_data.cistart = {}
            sofar = 0
            for ndn, ln in s._mpisppy_data.nlens.items():
                s._mpisppy_data.cistart[ndn] = sofar
                sofar += ln

    def _attach_nonant_indices(self):
        for s in self.local_scenarios.values():
            ni = {}
            for nd in s._mpisppy_node_list:
                for i in range(s._mpisppy_data.nlens[nd.name]):
                    ni[(nd.name, i)] = nd.nonant_vardata_list[i]
            s._mpisppy_data.nonant_indices = ni
            s._mpisppy_data.varid_to_nonant_index = {id(v): k for k, v in ni.items()}
        self.nonant_length = len(ni) if self.local_scenarios else 0

    def _verify_nonant_lengths(self):
        lens = {}
        for s in self.local_scenarios.values():
            for nd in s._mpisppy_node_list:
                L = s._mpisppy_data.nlens[nd.name]
                if lens.setdefault(nd.name, L) != L:
                    raise RuntimeError(f"Tree node {nd.name} has scenarios with different numbers of "
                                       f"non-anticipative variables: {L} vs. {lens[nd.name]}")
        for nd in set().union(*[[n.name for n in s._mpisppy_node_list] for s in self.local_scenarios.values()]):
            if nd not in self.all_nodenames:
                raise RuntimeError(f"Tree node '{nd}' not in all_nodenames list {self.all_nodenames}")

    def _use_variable_probability_setter(self, verbose=False):
        """``spbase.py:398-438``: variable_probability(scenario, **kw) -> [(vardata or id, prob)]
        makes prob_coeff per nonant for the nodes it touches; prob0_mask zeroes W of
        zero-probability variables (phbase.py:323-326)."""
        if self.variable_probability is None:
            for s in self.local_scenarios.values():
                s._mpisppy_data.has_variable_probability = False
            return
        kw = self.options.get("variable_probability_kwargs", {}) or {}
        for s in self.local_scenarios.values():
            s._mpisppy_data.has_variable_probability = True
            for v, prob in self.variable_probability(s, **kw):
                vid = v if isinstance(v, int) else id(v)
                ndn, i = s._mpisppy_data.varid_to_nonant_index[vid]
                if not isinstance(s._mpisppy_data.prob_coeff[ndn], np.ndarray):
                    nl = s._mpisppy_data.nlens[ndn]
                    s._mpisppy_data.prob_coeff[ndn] = np.full(nl, s._mpisppy_data.prob_coeff[ndn], dtype="d")
                    s._mpisppy_data.prob0_mask[ndn] = np.ones(nl, dtype="d")
                s._mpisppy_data.prob_coeff[ndn][i] = prob
                if prob == 0:
                    s._mpisppy_data.prob0_mask[ndn][i] = 0.0
        if not self.options.get("do_not_check_variable_probabilities", False):
            self._check_variable_probabilities_sum(verbose)

    def _check_variable_probabilities_sum(self, verbose=False):
        """``spbase.py:459-500``: per node, the per-variable probabilities must sum to 1 over all
        scenarios (SUM across ranks)."""
        sums = {}
        for s in self.local_scenarios.values():
            for nd in s._mpisppy_node_list:
                v = np.full(s._mpisppy_data.nlens[nd.name], 0.0) + s._mpisppy_data.prob_coeff[nd.name]
                sums[nd.name] = sums.get(nd.name, 0.0) + v
        # ranks own different nodes of a multistage tree: ONE reduction over a vector laid out over
        # the union of every rank's nodes (the reference has one communicator per node instead),
        # so every rank makes the same collective call with the same length
        lens = {k: len(v) for k, v in sums.items()}
        if self.n_proc > 1:
            for d in self.mpicomm.allgather_object(lens):
                lens.update(d)
        names = sorted(lens)
        off = np.concatenate([[0], np.cumsum([lens[k] for k in names])]).astype(int)
        flat = np.zeros(int(off[-1]))
        for i, k in enumerate(names):
            if k in sums:
                flat[off[i]:off[i + 1]] = sums[k]
        if self.n_proc > 1:
            flat = np.asarray(self.mpicomm.allreduce_array(flat))
        for i, ndn in enumerate(names):
            tot = flat[off[i]:off[i + 1]]
            if not np.allclose(tot, 1.0, atol=self.E1_tolerance):
                bad = np.nonzero(~np.isclose(tot, 1.0, atol=self.E1_tolerance))[0]
                raise RuntimeError(f"Node {ndn}, variables indexed {bad.tolist()} have unconditional "
                                   f"probability sums {tot[bad].tolist()}")

    def is_zero_prob(self, scenario_model, var):
        """``spbase.py:442-457``."""
        if self.variable_probability is None:
            return False
        d = scenario_model._mpisppy_data
        ndn, i = d.varid_to_nonant_index[id(var)]
        pc = d.prob_coeff[ndn]
        return isinstance(pc, np.ndarray) and float(pc[i]) == 0.0

    def _set_sense(self):
        senses = {s.sense for s in self.local_scenarios.values()}
        if len(senses) > 1:
            raise RuntimeError("All scenario models must have the same model sense (minimize or maximize)")
        self.is_minimizing = senses.pop() == 1 if senses else True

    @property
    def spcomm(self):
        return self._spcomm

    @spcomm.setter
    def spcomm(self, value):
        self._spcomm = value
