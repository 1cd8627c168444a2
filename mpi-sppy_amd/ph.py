"""PH on the MI355X engine (restates ``mpisppy/opt/ph.py:23-76``)."""
from .phbase import PHBase


class PH(PHBase):
    """PH. See PHBase for the list of args."""

    def ph_main(self, finalize=True):
        """``opt/ph.py:31-76``: PH_Prep -> Iter0 -> iterk_loop -> [post_loops].

        Returns (conv, Eobj or None, trivial_bound)."""
        smoothed = self.options.get("smoothed", 0)
        self.PH_Prep(attach_smooth=smoothed)
        trivial_bound = self.Iter0()
        if self.options.get("asynchronousPH"):
            raise RuntimeError("asynchronousPH is deprecated; use APH")
        self.iterk_loop()
        Eobj = self.post_loops(self.extobject) if finalize else None
        return self.conv, Eobj, trivial_bound
