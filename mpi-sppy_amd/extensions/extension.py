"""Extension hook interface (restates ``mpisppy/extensions/extension.py:18-152`` and
``MultiExtension`` :154-233).

PHBase calls these hooks around the batched device solve; the defaults do nothing.  Only
``pre_solve`` / ``post_solve`` have no per-subproblem meaning here (all scenarios are one batched
launch), so PHBase calls ``pre_solve_loop`` / ``post_solve_loop`` around the launch instead.
"""

_HOOKS = ("setup_hub", "initialize_spoke_indices", "sync_with_spokes", "pre_solve_loop",
          "post_solve_loop", "pre_iter0", "iter0_post_solver_creation", "post_iter0",
          "post_iter0_after_sync", "miditer", "enditer", "enditer_after_sync", "post_everything")


class Extension:
    def __init__(self, spopt_object):
        self.opt = spopt_object

    def setup_hub(self):
        pass

    def initialize_spoke_indices(self):
        pass

    def sync_with_spokes(self):
        pass

    def pre_solve(self, subproblem):
        pass

    def post_solve(self, subproblem, results):
        return results

    def pre_solve_loop(self):
        pass

    def post_solve_loop(self):
        pass

    def pre_iter0(self):
        pass

    def iter0_post_solver_creation(self):
        pass

    def post_iter0(self):
        pass

    def post_iter0_after_sync(self):
        pass

    def miditer(self):
        pass

    def enditer(self):
        pass

    def enditer_after_sync(self):
        pass

    def post_everything(self):
        pass


class MultiExtension(Extension):
    """Runs several extensions, in the order given, for every hook."""

    def __init__(self, ph, ext_classes):
        super().__init__(ph)
        self.extdict = {cls.__name__: cls(ph) for cls in ext_classes}
        # the pipelined PH loop may run them only if every member only touches solver options
        self.pipeline_safe = all(getattr(e, "pipeline_safe", False) for e in self.extdict.values())

    def post_solve(self, subproblem, results):
        for e in self.extdict.values():
            results = e.post_solve(subproblem, results)
        return results

    def pre_solve(self, subproblem):
        for e in self.extdict.values():
            e.pre_solve(subproblem)


def _fan_out(name):
    def hook(self):
        for e in self.extdict.values():
            getattr(e, name)()
    hook.__name__ = name
    return hook


for _h in _HOOKS:
    setattr(MultiExtension, _h, _fan_out(_h))
