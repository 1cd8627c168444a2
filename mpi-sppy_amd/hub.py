"""Hub-only cylinder driver (restates the PHHub <-> opt contract of ``mpisppy/cylinders/hub.py:462-616``
and the hub-only path of ``WheelSpinner`` (``mpisppy/spin_the_wheel.py:40-164``)).

``WheelSpinner(hub_dict, []).spin()`` constructs ``hub_dict["opt_class"](**opt_kwargs)``, wraps it
in ``hub_dict["hub_class"]`` and runs ``main()`` then ``finalize()``, exactly the call order the
reference uses when no spokes are given (``test_w_writer.py:72-76``).  Spokes (Lagrangian / xhat
bounders) are a later milestone; ``PHHub.is_converged`` therefore never stops PH (as in the
reference without inner-bound spokes).
"""
import math


class PHHub:
    def __init__(self, spbase_object, options=None):
        self.opt = spbase_object
        self.opt.spcomm = self
        self.options = options or {}
        self.BestOuterBound = -math.inf if self.opt.is_minimizing else math.inf
        self.BestInnerBound = math.inf if self.opt.is_minimizing else -math.inf
        self.use_trivial_bound = True
        self.trace = []

    def OuterBoundUpdate(self, b):
        if self.opt.is_minimizing:
            return max(self.BestOuterBound, b)
        return min(self.BestOuterBound, b)

    def setup_hub(self):
        if self.opt.extobject is not None and hasattr(self.opt.extobject, "setup_hub"):
            self.opt.extobject.setup_hub()

    def sync(self):
        if self.opt.extobject is not None and hasattr(self.opt.extobject, "sync_with_spokes"):
            self.opt.extobject.sync_with_spokes()

    def is_converged(self):
        if self.opt._PHIter == 1 and self.use_trivial_bound:
            self.BestOuterBound = self.OuterBoundUpdate(self.opt.trivial_bound)
        self.trace.append((self.opt._PHIter, self.BestOuterBound, self.BestInnerBound))
        return False

    def current_iteration(self):
        return self.opt._PHIter

    def main(self):
        self.opt.ph_main(finalize=False)

    def finalize(self):
        return self.opt.post_loops(self.opt.extobject)


class WheelSpinner:
    def __init__(self, hub_dict, list_of_spoke_dict):
        if list_of_spoke_dict:
            raise NotImplementedError("spokes are not implemented yet: use WheelSpinner(hub_dict, [])")
        self.hub_dict = hub_dict
        self.spcomm = None

    def spin(self, comm_world=None):
        hd = self.hub_dict
        opt_kwargs = dict(hd["opt_kwargs"])
        if comm_world is not None:
            opt_kwargs["mpicomm"] = comm_world
        opt = hd["opt_class"](**opt_kwargs)
        hub = hd.get("hub_class", PHHub)(opt, **hd.get("hub_kwargs", {}))
        hub.setup_hub()
        self.spcomm = hub
        self.strata_rank = 0
        self.global_rank = opt.cylinder_rank
        hub.main()
        self.Eobj = hub.finalize()
        self.BestInnerBound = hub.BestInnerBound
        self.BestOuterBound = hub.BestOuterBound
        return self
