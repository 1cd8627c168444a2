"""PH hub and wheel (restates the PHHub <-> opt contract of ``mpisppy/cylinders/hub.py:29-616``
and ``WheelSpinner`` of ``mpisppy/spin_the_wheel.py:40-164``).

``WheelSpinner(hub_dict, list_of_spoke_dict).spin()`` constructs ``hub_dict["opt_class"]
(**opt_kwargs)``, wraps it in ``hub_dict["hub_class"]`` and runs ``main()`` then ``finalize()``,
the reference's call order.  Spokes (``cylinders.LagrangianOuterBound``,
``cylinders.XhatShuffleInnerBound``) live on the hub's GPU as extra handles with their own
streams; they are created at the hub's first ``sync`` (once the hub's batch exists) and fed
device-to-device from then on (see ``cylinders.py``).  Termination on the inter-cylinder gap
(``rel_gap`` / ``abs_gap`` / ``max_stalled_iters`` in the hub options) follows
``hub.py:130-166``.
"""
import math
import os

from . import _lib, cylinders
from .utils import sputils


class PHHub:
    def __init__(self, spbase_object, options=None, spoke_dicts=None):
        self.opt = spbase_object
        self.opt.spcomm = self
        self.options = options or {}
        self.spoke_dicts = list(spoke_dicts or [])
        self.spokes = []
        self.BestOuterBound = -math.inf if self.opt.is_minimizing else math.inf
        self.BestInnerBound = math.inf if self.opt.is_minimizing else -math.inf
        self.latest_ob_char = self.latest_ib_char = None
        self.use_trivial_bound = True
        self.last_gap = float("inf")
        self.stalled_iter_cnt = 0
        self.trace = []

    # ------------------------------------------------------------------ bounds
    def OuterBoundUpdate(self, b, char="*"):
        better = b > self.BestOuterBound if self.opt.is_minimizing else b < self.BestOuterBound
        if better:
            self.latest_ob_char = char
            return b
        return self.BestOuterBound

    def InnerBoundUpdate(self, b, char="*"):
        better = b < self.BestInnerBound if self.opt.is_minimizing else b > self.BestInnerBound
        if better:
            self.latest_ib_char = char
            return b
        return self.BestInnerBound

    @property
    def has_innerbound_spokes(self):
        return any(s.get("spoke_class").bound_kind == "inner" for s in self.spoke_dicts)

    @property
    def has_outerbound_spokes(self):
        return any(s.get("spoke_class").bound_kind == "outer" for s in self.spoke_dicts)

    def compute_gaps(self):
        return cylinders.gaps(self)

    def _take(self, sp, b):
        if b is None:
            return
        if sp.bound_kind == "outer":
            self.BestOuterBound = self.OuterBoundUpdate(b, sp.converger_spoke_char)
        else:
            self.BestInnerBound = self.InnerBoundUpdate(b, sp.converger_spoke_char)

    # ------------------------------------------------------------------ hub protocol
    def setup_hub(self):
        if self.opt.extobject is not None and hasattr(self.opt.extobject, "setup_hub"):
            self.opt.extobject.setup_hub()

    def sync(self):
        """``hub.py:516-532``: send W / nonants to the spokes, receive their bounds."""
        if self.spoke_dicts and not self.spokes:
            self.spokes = [cylinders.spoke_from_dict(self.opt, d) for d in self.spoke_dicts]
        for sp in self.spokes:
            self._take(sp, sp.update())
        if self.opt.extobject is not None and hasattr(self.opt.extobject, "sync_with_spokes"):
            self.opt.extobject.sync_with_spokes()

    def sync_with_spokes(self):
        self.sync()

    def is_converged(self):
        """``hub.py:534-565``."""
        if self.opt._PHIter == 1 and self.use_trivial_bound:
            self.BestOuterBound = self.OuterBoundUpdate(self.opt.trivial_bound)
        self.trace.append((self.opt._PHIter, self.BestOuterBound, self.BestInnerBound))
        if not self.has_innerbound_spokes:
            return False
        return self.determine_termination()

    def determine_termination(self):
        """``hub.py:130-166``."""
        o = self.options
        if not any(k in o for k in ("rel_gap", "abs_gap", "max_stalled_iters")):
            return False
        abs_gap, rel_gap = self.compute_gaps()
        rel_ok = "rel_gap" in o and rel_gap <= o["rel_gap"]
        abs_ok = "abs_gap" in o and abs_gap <= o["abs_gap"]
        stalled = False
        if "max_stalled_iters" in o:
            if abs_gap < self.last_gap:
                self.last_gap = abs_gap
                self.stalled_iter_cnt = 0
            else:
                self.stalled_iter_cnt += 1
                stalled = self.stalled_iter_cnt >= o["max_stalled_iters"]
        return bool(rel_ok or abs_ok or stalled)

    def current_iteration(self):
        return self.opt._PHIter

    def main(self):
        self.opt.ph_main(finalize=False)

    def hub_finalize(self):
        """``hub.py:168-177``: last bounds from the spokes."""
        for sp in self.spokes:
            self._take(sp, sp.finalize())

    def finalize(self):
        self.hub_finalize()
        return self.opt.post_loops(self.opt.extobject)


class WheelSpinner:
    def __init__(self, hub_dict, list_of_spoke_dict):
        self.hub_dict = hub_dict
        self.list_of_spoke_dict = list(list_of_spoke_dict or [])
        self.spcomm = None

    def spin(self, comm_world=None):
        hd = self.hub_dict
        opt_kwargs = dict(hd["opt_kwargs"])
        if comm_world is not None:
            opt_kwargs["mpicomm"] = comm_world
        opt = hd["opt_class"](**opt_kwargs)
        hub_kwargs = dict(hd.get("hub_kwargs", {}))
        hub = hd.get("hub_class", PHHub)(opt, spoke_dicts=self.list_of_spoke_dict, **hub_kwargs)
        hub.setup_hub()
        self.spcomm = hub
        self.strata_rank = 0
        self.global_rank = opt.cylinder_rank
        hub.main()
        self.Eobj = hub.finalize()
        self.BestInnerBound = hub.BestInnerBound
        self.BestOuterBound = hub.BestOuterBound
        for sp in hub.spokes:
            sp.close()
        return self

    # ------------------------------------------------------------------ solutions (spin_the_wheel.py:166-213)
    def _incumbent_spoke(self):
        """The inner-bound spoke holding the best incumbent (``_determine_innerbound_winner``)."""
        best = None
        for sp in self.spcomm.spokes:
            if sp.bound_kind == "inner" and getattr(sp, "best_X", None) is not None:
                if best is None or sp._better(sp.bound, best.bound) == sp.bound:
                    best = sp
        return best

    def _with_incumbent(self, fn):
        opt = self.spcomm.opt
        sp = self._incumbent_spoke()
        if sp is None:
            if opt.cylinder_rank == 0:
                print("No incumbent solution available to write!")
            return False
        saved = {}
        for k, (sname, s) in enumerate(opt.local_scenarios.items()):
            saved[sname] = s._solution
            s._solution = sp.best_X[k]
        try:
            fn(opt)
        finally:
            for sname, s in opt.local_scenarios.items():
                s._solution = saved[sname]
        return True

    def write_first_stage_solution(self, solution_file_name,
                                   first_stage_solution_writer=sputils.first_stage_nonant_writer):
        """Writes the incumbent's ROOT nonants (``spbase.py:639-655``) on rank 0."""
        def w(opt):
            if opt.cylinder_rank == 0:
                d = os.path.dirname(solution_file_name)
                if d:
                    os.makedirs(d, exist_ok=True)
                s = opt.local_scenarios[opt.local_scenario_names[0]]
                first_stage_solution_writer(solution_file_name, s, False)
        return self._with_incumbent(w)

    def write_tree_solution(self, solution_directory_name,
                            scenario_tree_solution_writer=sputils.scenario_tree_solution_writer):
        """One file per scenario with the incumbent's full solution (``spbase.py:657-675``)."""
        def w(opt):
            if opt.cylinder_rank == 0:
                os.makedirs(solution_directory_name, exist_ok=True)
            opt.mpicomm.Barrier()
            for sname, s in opt.local_scenarios.items():
                scenario_tree_solution_writer(solution_directory_name, sname, s, False)
        return self._with_incumbent(w)

    def local_nonant_cache(self):
        """{node name: nonant values} of the hub's local scenarios (``spin_the_wheel.py:197-209``)."""
        opt = self.spcomm.opt
        xn = opt.engine.get(_lib.F_XN).reshape(opt.engine.S, -1)
        out = {}
        for k, s in enumerate(opt.local_scenarios.values()):
            pos = 0
            for nd in s._mpisppy_node_list:
                ln = len(nd.nonant_vardata_list)
                if nd.name not in out:
                    out[nd.name] = list(xn[k, pos:pos + ln])
                pos += ln
        return out
