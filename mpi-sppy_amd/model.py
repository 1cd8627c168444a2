"""Pyomo-free linear scenario models: the object a ``scenario_creator`` returns in this engine.

The reference's ``scenario_creator(name, **kw)`` returns a Pyomo ``ConcreteModel`` carrying
``_mpisppy_node_list`` (``mpisppy/scenario_tree.py:51-103``) and ``_mpisppy_probability``
(``mpisppy/spbase.py:509-526``).  Pyomo is absent on both the build container and the MI355X box, so
the engine's scenario creators return a :class:`LinearModel` -- the same information already in the
standard form the batched solver consumes::

    min/max  c^T x  s.t.  row_lo <= A x <= row_hi,  col_lo <= x <= col_hi

Variables are grouped in :class:`VarBlock` objects indexed like Pyomo ``Var`` components, so
``ScenarioNode(nonant_list=[model.DevotedAcreage])`` expands to the SORTED keys exactly as
``scenario_tree.build_vardatalist`` does (``mpisppy/scenario_tree.py:45-46``).
"""
import numpy as np

INF = float("inf")
minimize = 1
maximize = -1


class VarData:
    __slots__ = ("model", "col", "name")

    def __init__(self, model, col, name):
        self.model = model
        self.col = col
        self.name = name

    @property
    def value(self):
        return self.model.value_of(self.col)

    _value = value

    def __repr__(self):
        return self.name


class VarBlock:
    """An indexed (or scalar, index=None) block of columns, Pyomo ``Var``-like."""

    def __init__(self, model, name, index):
        self.model = model
        self.name = name
        self._data = {}
        if index is None:
            self._scalar = True
            self._data[None] = VarData(model, model._new_col(name), name)
        else:
            self._scalar = False
            for k in index:
                nm = f"{name}[{k}]"
                self._data[k] = VarData(model, model._new_col(nm), nm)

    def is_indexed(self):
        return not self._scalar

    def keys(self):
        return self._data.keys()

    def __getitem__(self, k):
        return self._data[k]

    def __iter__(self):
        return iter(self._data)

    def __len__(self):
        return len(self._data)

    def values(self):
        return self._data.values()

    @property
    def col(self):
        if not self._scalar:
            raise TypeError(f"{self.name} is indexed")
        return self._data[None].col


class LinearModel:
    def __init__(self, name=""):
        self.name = name
        self._colnames = []
        self._lo = []
        self._hi = []
        self._cost = []
        self._rows = []          # (dict col->coef, lo, hi, name)
        self._blocks = []        # VarBlocks in creation order
        self.sense = minimize
        self.obj_offset = 0.0
        self._solution = None    # filled by the engine after a solve (x of this scenario)

    # --------------------------------------------------------------------------- building
    def _new_col(self, name):
        self._colnames.append(name)
        self._lo.append(-INF)
        self._hi.append(INF)
        self._cost.append(0.0)
        return len(self._colnames) - 1

    def add_var(self, name, index=None, bounds=(0.0, INF)):
        blk = VarBlock(self, name, index)
        for vd in blk.values():
            lo, hi = bounds(vd) if callable(bounds) else bounds
            self._lo[vd.col] = -INF if lo is None else float(lo)
            self._hi[vd.col] = INF if hi is None else float(hi)
        setattr(self, name, blk)
        self._blocks.append(blk)
        return blk

    def add_row(self, coefs, lo=-INF, hi=INF, name=""):
        """coefs: iterable of (VarData or column index, coefficient)."""
        d = {}
        for v, a in (coefs.items() if isinstance(coefs, dict) else coefs):
            j = v.col if isinstance(v, VarData) else int(v)
            d[j] = d.get(j, 0.0) + float(a)
        self._rows.append((d, -INF if lo is None else float(lo), INF if hi is None else float(hi), name))

    def set_objective(self, coefs, sense=minimize, offset=0.0):
        self.sense = sense
        self.obj_offset = float(offset)
        for v, a in (coefs.items() if isinstance(coefs, dict) else coefs):
            j = v.col if isinstance(v, VarData) else int(v)
            self._cost[j] += float(a)

    # --------------------------------------------------------------------------- views
    @property
    def n(self):
        return len(self._colnames)

    @property
    def m(self):
        return len(self._rows)

    def column_names(self):
        return list(self._colnames)

    def pattern(self):
        """CSR pattern (rowptr, colidx) with column indices sorted inside each row."""
        rowptr = np.zeros(self.m + 1, np.int32)
        cols = []
        for i, (d, _, _, _) in enumerate(self._rows):
            cols.extend(sorted(d))
            rowptr[i + 1] = len(cols)
        return rowptr, np.array(cols, np.int32)

    def csr_values(self):
        vals = []
        for d, _, _, _ in self._rows:
            vals.extend(d[j] for j in sorted(d))
        return np.array(vals, np.float64)

    def arrays(self):
        rp, ci = self.pattern()
        return dict(
            c=np.array(self._cost, np.float64), rowptr=rp, colidx=ci, vals=self.csr_values(),
            row_lo=np.array([r[1] for r in self._rows], np.float64),
            row_hi=np.array([r[2] for r in self._rows], np.float64),
            col_lo=np.array(self._lo, np.float64), col_hi=np.array(self._hi, np.float64),
        )

    def value_of(self, col):
        if self._solution is None:
            return None
        return float(self._solution[col])

    def objective_value(self, x=None):
        x = self._solution if x is None else x
        return float(np.dot(self._cost, x)) + self.obj_offset
