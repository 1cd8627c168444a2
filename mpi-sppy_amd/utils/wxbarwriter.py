"""WXBarWriter extension (restates ``mpisppy/utils/wxbarwriter.py:36-110``).

Options (in the PH options dict): ``W_fname`` (file, or directory when ``separate_W_files``),
``Xbar_fname``, ``separate_W_files``.  W and xbar are written once, in ``post_everything``.
"""
import os

from ..extensions.extension import Extension
from . import wxbarutils


class WXBarWriter(Extension):
    def __init__(self, ph):
        super().__init__(ph)
        o = ph.options
        self.PHB = ph
        self.cylinder_rank = ph.cylinder_rank
        self.w_fname = o.get("W_fname")
        self.x_fname = o.get("Xbar_fname")
        self.sep_files = bool(o.get("separate_W_files", False))
        rank0 = self.cylinder_rank == 0
        if self.w_fname is None and self.x_fname is None and rank0:
            print("Warning: no output files provided to WXBarWriter. No values will be saved.")
        if self.w_fname and not self.sep_files and os.path.exists(self.w_fname) and rank0:
            print(f"Warning: specified W_fname ({self.w_fname}) already exists. "
                  "Results will be appended to this file.")
        elif self.w_fname and self.sep_files and not os.path.exists(self.w_fname):
            if rank0:
                print(f"Warning: path {self.w_fname} does not exist. Creating...")
            os.makedirs(self.w_fname, exist_ok=True)
        if self.x_fname and os.path.exists(self.x_fname) and rank0:
            print(f"Warning: specified Xbar_fname ({self.x_fname}) already exists. "
                  "Results will be appended to this file.")

    def post_everything(self):
        if self.w_fname:
            wxbarutils.write_W_to_file(self.PHB, self.w_fname, sep_files=self.sep_files)
        if self.x_fname:
            wxbarutils.write_xbar_to_file(self.PHB, self.x_fname)
