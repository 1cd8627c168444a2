"""Solver-tolerance schedule by PH iteration (restates ``mpisppy/extensions/mipgapper.py:15-60``).

The reference's ``Gapper`` sets ``ph.current_solver_options["mipgap"]`` from
``options["gapperoptions"]["mipgapdict"]`` (PH iteration -> gap) at ``pre_iter0`` (key 0) and at
``miditer`` (the iteration's key), so every ``solve_loop`` of that iteration runs at that gap.  The
PDHG engine has no MIP gap; its tolerance is the relative KKT error ``pdhg_eps``, so
``gapperoptions["solver_option"]`` names the option the schedule drives (default ``"mipgap"``, the
reference's; ``"pdhg_eps"`` for the GPU plugin: loose early solves, tight ones once PH is close).

The extension only changes solver options, keyed by the iteration number, so the pipelined PH loop
(``PHBase.update_and_solve``, which enqueues solve k before the host has read conv_{k-1}) can run
it: ``pipeline_safe`` tells ``PHBase._can_pipeline`` so, and the loop calls ``miditer`` with
``_PHIter`` = k before it enqueues solve k -- the same option for the same solve as the reference's
statement order.
"""
from .extension import Extension


class Gapper(Extension):
    pipeline_safe = True

    def __init__(self, ph):
        super().__init__(ph)
        self.ph = ph
        self.cylinder_rank = ph.cylinder_rank
        self.gapperoptions = ph.options["gapperoptions"]       # required, as in the reference
        self.mipgapdict = self.gapperoptions["mipgapdict"]
        self.option = self.gapperoptions.get("solver_option", "mipgap")
        self.verbose = ph.options["verbose"] or self.gapperoptions.get("verbose", False)
        self.history = []        # (PH iteration, value) of every change (tests, diagnostics)

    def _vb(self, msg):
        if self.verbose and self.cylinder_rank == 0:
            print("(rank0) mipgapper:" + msg)

    def set_mipgap(self, mipgap):
        """Set the scheduled option in the current solver options (``mipgapper.py:30-40``)."""
        opts = self.ph.current_solver_options
        if opts is None:
            opts = self.ph.current_solver_options = {}
        old = opts.get(self.option)
        self._vb(f"Changing {self.option} from {old} to {mipgap}")
        opts[self.option] = float(mipgap)
        self.history.append((self.ph._PHIter, float(mipgap)))

    def pre_iter0(self):
        if self.mipgapdict is None:
            return
        if 0 in self.mipgapdict:
            self.set_mipgap(self.mipgapdict[0])

    def miditer(self):
        if self.mipgapdict is None:
            return
        if self.ph._PHIter in self.mipgapdict:
            self.set_mipgap(self.mipgapdict[self.ph._PHIter])
