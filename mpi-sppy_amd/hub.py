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

from . import cylinders


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
