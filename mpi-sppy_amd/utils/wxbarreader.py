"""WXBarReader extension (restates ``mpisppy/utils/wxbarreader.py:36-106``).

Options: ``init_W_fname`` (file, or directory when ``init_separate_W_files``), ``init_Xbar_fname``.
The values are loaded in ``miditer`` of PH iteration 1 -- after iteration 0's W / xbar update and
before iteration 1's batched solve -- and W and prox are re-enabled, as the reference does.
"""
import os

from ..extensions.extension import Extension
from . import wxbarutils


class WXBarReader(Extension):
    def __init__(self, ph):
        super().__init__(ph)
        o = ph.options
        self.PHB = ph
        self.cylinder_rank = ph.cylinder_rank
        self.sep_files = bool(o.get("init_separate_W_files", False))
        self.w_fname = o.get("init_W_fname")
        self.x_fname = o.get("init_Xbar_fname")
        # a missing input ends the run (the reference prints and quit()s)
        if self.w_fname is not None and not os.path.exists(self.w_fname):
            kind = "path" if self.sep_files else "file"
            raise SystemExit(f"Cannot find {kind} {self.w_fname}")
        if self.x_fname is not None and not os.path.exists(self.x_fname):
            raise SystemExit(f"Cannot find file {self.x_fname}")
        if self.w_fname is None and self.x_fname is None and self.cylinder_rank == 0:
            print("Warning: no input files provided to WXBarReader. "
                  "W and Xbar will be initialized to their default values.")

    def miditer(self):
        if self.PHB._PHIter != 1:
            return
        if self.w_fname:
            wxbarutils.set_W_from_file(self.w_fname, self.PHB, self.cylinder_rank, sep_files=self.sep_files)
            self.PHB._reenable_W()
        if self.x_fname:
            wxbarutils.set_xbar_from_file(self.x_fname, self.PHB)
            self.PHB._reenable_prox()
