"""GPU batch engine: one ``libphg`` handle holding all local scenarios of a rank on its GPU.

Builds the ``phg_batch`` C struct (include/phg.h) from the local scenario models -- the shared
CSR pattern, per-scenario values / costs / bounds, and the scenario-tree index maps of
``SPBase`` -- and exposes the hot-path calls the PH driver makes each iteration:

* :meth:`solve`            -- ``solve_loop`` for every local scenario (``spopt.py:250-341``)
* :meth:`node_sums` ... :meth:`conv` -- ``Compute_Xbar`` / ``Update_W`` / ``convergence_diff``
  (``phbase.py:32-112, 301-371``) with the cross-GPU SUMs done by the communicator (RCCL)
"""
import numpy as np

from . import _lib
from ._lib import as_f64, as_i32, ptr


def _node_level(name):
    return name.count("_")


class BatchArrays:
    """Host-side standard-form batch (numpy) for the local scenarios, in local order."""

    def __init__(self, models, all_nodenames, prob, scen_global0, S_global, virt_nproc):
        m0 = models[0]
        rp, ci = m0.pattern()
        self.rowptr, self.colidx = rp, ci
        S = len(models)
        n, m, nnz = m0.n, m0.m, len(ci)
        self.S, self.n, self.m, self.nnz = S, n, m, nnz
        vals = np.empty((S, nnz))
        c = np.empty((S, n))
        cl = np.empty((S, n))
        cu = np.empty((S, n))
        rl = np.empty((S, m))
        ru = np.empty((S, m))
        off = np.empty(S)
        for s, md in enumerate(models):
            if md.n != n or md.m != m:
                raise ValueError(f"scenario {md.name}: shape ({md.n},{md.m}) differs from ({n},{m}); "
                                 "the batch needs one shared sparsity pattern")
            a = md.arrays()
            if s and (not np.array_equal(a["rowptr"], rp) or not np.array_equal(a["colidx"], ci)):
                raise ValueError(f"scenario {md.name}: sparsity pattern differs from the first scenario")
            vals[s] = a["vals"]
            c[s] = a["c"]
            cl[s], cu[s], rl[s], ru[s] = a["col_lo"], a["col_hi"], a["row_lo"], a["row_hi"]
            off[s] = md.obj_offset
        self.vals, self.c, self.cl, self.cu, self.rl, self.ru, self.off = vals, c, cl, cu, rl, ru, off
        self.sense = m0.sense
        # scenario tree
        nodes0 = m0._mpisppy_node_list
        self.L = len(nodes0)
        self.level_len = np.array([len(nd.nonant_vardata_list) for nd in nodes0], np.int32)
        cols0 = [v.col for nd in nodes0 for v in nd.nonant_vardata_list]
        self.nonant_col = np.array(cols0, np.int32)
        self.N = len(cols0)
        self.nonant_level = np.concatenate([np.full(ln, l, np.int32) for l, ln in enumerate(self.level_len)])
        self.nonant_pos = np.concatenate([np.arange(ln, dtype=np.int32) for ln in self.level_len])
        self.all_nodenames = list(all_nodenames)
        node_id = {nm: g for g, nm in enumerate(self.all_nodenames)}
        lvl = [_node_level(nm) for nm in self.all_nodenames]
        self.node_off = np.zeros(len(self.all_nodenames), np.int32)
        tot = 0
        for g, nm in enumerate(self.all_nodenames):
            self.node_off[g] = tot
            if lvl[g] < self.L:
                tot += int(self.level_len[lvl[g]])
        self.N_tot = tot
        self.scen_node = np.zeros((S, self.L), np.int32)
        self.prob_coeff = np.zeros((S, self.L))
        # variable_probability (spbase.py:398-438): per-nonant coefficients, else None
        varprob = any(getattr(md._mpisppy_data, "has_variable_probability", False) for md in models)
        self.prob_coeff_var = np.zeros((S, self.N)) if varprob else None
        for s, md in enumerate(models):
            nl = md._mpisppy_node_list
            if len(nl) != self.L:
                raise ValueError("all scenarios must have the same number of tree levels")
            if [v.col for nd in nl for v in nd.nonant_vardata_list] != cols0:
                raise ValueError(f"scenario {md.name}: nonant columns differ from the first scenario")
            for l, nd in enumerate(nl):
                if nd.name not in node_id:
                    raise RuntimeError(f"Tree node '{nd.name}' not in all_nodenames")
                self.scen_node[s, l] = node_id[nd.name]
                pcn = md._mpisppy_data.prob_coeff[nd.name]
                if isinstance(pcn, np.ndarray):
                    self.prob_coeff[s, l] = np.nan      # per-variable: only prob_coeff_var is meaningful
                    self.prob_coeff_var[s, self.nonant_level == l] = pcn
                else:
                    self.prob_coeff[s, l] = pcn
                    if self.prob_coeff_var is not None:
                        self.prob_coeff_var[s, self.nonant_level == l] = pcn
        self.prob = np.asarray(prob, np.float64)
        self.scen_global0, self.S_global, self.virt_nproc = scen_global0, S_global, virt_nproc

    def c_struct(self):
        keep = []

        def k(a):
            keep.append(a)
            return ptr(a)
        b = _lib.PhgBatch()
        b.S, b.n, b.m, b.nnz = self.S, self.n, self.m, self.nnz
        b.rowptr, b.colidx = k(as_i32(self.rowptr)), k(as_i32(self.colidx))
        b.vals, b.c = k(as_f64(self.vals)), k(as_f64(self.c))
        b.col_lo, b.col_hi = k(as_f64(self.cl)), k(as_f64(self.cu))
        b.row_lo, b.row_hi = k(as_f64(self.rl)), k(as_f64(self.ru))
        b.obj_offset = k(as_f64(self.off))
        b.sense = int(self.sense)
        b.N, b.nonant_col, b.L = self.N, k(as_i32(self.nonant_col)), self.L
        b.nonant_level, b.nonant_pos = k(as_i32(self.nonant_level)), k(as_i32(self.nonant_pos))
        b.level_len, b.scen_node = k(as_i32(self.level_len)), k(as_i32(self.scen_node))
        b.n_nodes, b.node_off, b.N_tot = len(self.all_nodenames), k(as_i32(self.node_off)), self.N_tot
        b.prob, b.prob_coeff = k(as_f64(self.prob)), k(as_f64(self.prob_coeff))
        b.scen_global0, b.S_global, b.virt_nproc = self.scen_global0, self.S_global, self.virt_nproc
        b.prob_coeff_var = k(as_f64(self.prob_coeff_var)) if self.prob_coeff_var is not None else None
        form = getattr(self, "vals_form", _lib.VALS_PER_SCENARIO)
        if form == _lib.VALS_SHARED:
            if not (self.vals == self.vals[0]).all():
                raise ValueError("vals_form SHARED: the scenarios' matrices differ")
            b.vals, b.vals_form = k(as_f64(self.vals[0])), form
        elif form == _lib.VALS_DELTA:
            # the SURVEY 8(b) sparse delta list: the positions whose value differs from scenario 0's
            pos = np.flatnonzero((self.vals != self.vals[0]).any(axis=0)).astype(np.int32)
            b.vals, b.vals_form = k(as_f64(self.vals[0])), form
            b.n_delta, b.delta_pos = len(pos), k(as_i32(pos))
            b.delta_vals = k(as_f64(self.vals[:, pos]))
        return b, keep


def plan_layout(batch):
    """Host-only dry run of the lane-local layout planner (``phg_plan``): dict or None."""
    import ctypes
    lib = _lib.load()
    b, keep = batch.c_struct()
    out = np.zeros(8, np.int32)
    _lib.check(lib.phg_plan(ctypes.byref(b), ptr(out)))
    del keep
    if out[0] < 0:
        return None
    return {"variant": int(out[0]), "lanes_per_scenario": int(out[1]), "cols_per_lane": int(out[2]),
            "rows_per_lane": int(out[3]), "coupling_slots": int(out[4]), "coupling_rows": int(out[5]),
            "lanes_used": int(out[6]), "kernel_variant": int(out[7])}


def implied_bounds(batch):
    """Host-only: the column bounds the safe outer bounds use (``phg_implied_bounds``): (lo, hi) as
    [S, n] arrays and the number of columns left with an infinite side."""
    lib = _lib.load()
    b, keep = batch.c_struct()
    lo = np.empty(batch.S * batch.n)
    hi = np.empty(batch.S * batch.n)
    nf = np.zeros(1, np.int32)
    _lib.check(lib.phg_implied_bounds(__import__("ctypes").byref(b), ptr(lo), ptr(hi), ptr(nf)))
    del keep
    return lo.reshape(batch.S, batch.n), hi.reshape(batch.S, batch.n), int(nf[0])


class Engine:
    """One libphg handle on one GPU (no CPU fallback: raises if the library or device is missing)."""

    LAYOUTS = {"auto": 0, "gather": 1, "local": 2, "block": 3, "mfma": 4, "stream": 5, "border": 6, "wave": 7}

    def __init__(self, batch, device=0, stream=None, exchange=None, layout="auto", presolve=True):
        self.lib = _lib.load()
        self.batch = batch
        import ctypes
        h = ctypes.c_void_p()
        _lib.check(self.lib.phg_create(int(device), ctypes.byref(h)))
        self.h = h
        if stream is not None:
            _lib.check(self.lib.phg_set_stream(self.h, ctypes.c_void_p(int(stream))))
        _lib.check(self.lib.phg_set_layout(self.h, self.LAYOUTS[layout]))
        _lib.check(self.lib.phg_set_presolve(self.h, int(bool(presolve))))
        b, keep = batch.c_struct()
        _lib.check(self.lib.phg_load_batch(self.h, ctypes.byref(b)))
        del keep
        self.S, self.N, self.N_tot, self.P = batch.S, batch.N, batch.N_tot, batch.virt_nproc
        # multi-GPU: ONE packed device tensor [2 N_tot node sums | 2P+2 partials | flag]
        # (include/phg.h, phg_exchange_layout) all-reduced by the communicator; None on one GPU
        self.exchange = exchange
        lay = np.zeros(3, np.int32)
        _lib.check(self.lib.phg_exchange_layout(self.h, ptr(lay)))
        self.exchange_len = int(lay[2])
        if exchange is not None and int(exchange.numel()) != self.exchange_len:
            raise ValueError(f"exchange buffer has {exchange.numel()} doubles, the batch needs {self.exchange_len}")
        info = np.zeros(8, np.int32)
        _lib.check(self.lib.phg_info(self.h, ptr(info)))
        self.variant = int(info[6])
        self.lanes_per_scenario = int(info[7])
        self.layout = ("wave" if self.variant >= 700 else "border" if self.variant >= 500 else "stream" if self.variant >= 400 else
                       "mfma" if self.variant >= 300 else "block" if self.variant >= 200 else
                       "local" if self.variant >= 100 else "gather")
        # multi-workgroup layouts (range-split stream 400 + K, bordered 500 + K): workgroups per scenario
        self.workgroups_per_scenario = self.variant % 100 if 400 <= self.variant < 700 else 1
        # bordered layout: 600 + K the register-resident kernel, 500 + K the memory-resident one
        self.border_reg = 600 <= self.variant < 700
        pi = np.zeros(2, np.int32)
        _lib.check(self.lib.phg_presolve_info(self.h, ptr(pi)))
        self.rows_folded, self.rows_kept = int(pi[0]), int(pi[1])

    def values_info(self):
        """Value form of the loaded batch (phg_values_info): positions varying between scenarios,
        whether the shared-scaling delta form is in use (and its unit form: the matrix held in LDS as
        +-1 entry codes), and the matrix values one A x + A^T y of
        the workgroup kernel reads per scenario / from the one shared copy."""
        out = np.zeros(4, np.int32)
        _lib.check(self.lib.phg_values_info(self.h, ptr(out)))
        return {"varying": int(out[0]), "delta": bool(out[1]), "unit": int(out[1]) == 2,
                "per_scenario_vals": int(out[2]), "shared_vals": int(out[3])}

    def local_info(self):
        """Lane-local layout (phg_local_info): the variant, lanes per scenario, whether the next
        launch takes the lone-wave build (small shards), and the fp64 operations one lane issues per
        PDHG iteration in the variant's hot loop (FMA = 2; pdhg_local.hip local_loop_ops)."""
        out = np.zeros(4, np.int32)
        _lib.check(self.lib.phg_local_info(self.h, ptr(out)))
        return {"variant": int(out[0]), "lanes": int(out[1]), "lone": bool(out[2]),
                "loop_ops_per_lane": int(out[3]) / 100.0}

    def mfma_fragments(self):
        """MFMA instructions per PDHG iteration per 16 scenarios (nonzero 16x4 fragments of A x and
        A^T y) of the shared-matrix layout (phg_mfma_info)."""
        out = np.zeros(4, np.int32)
        _lib.check(self.lib.phg_mfma_info(self.h, ptr(out)))
        return int(out[2] + out[3])

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.phg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ data movement
    _SIZES = None

    def _count(self, field):
        S, n, m, N = self.batch.S, self.batch.n, self.batch.m, self.N
        return {_lib.F_X: S * n, _lib.F_Y: S * m, _lib.F_XN: S * N, _lib.F_W: S * N, _lib.F_RHO: S * N,
                _lib.F_XBAR: self.N_tot, _lib.F_XSQBAR: self.N_tot, _lib.F_OBJ: S, _lib.F_BOUND: S,
                _lib.F_EVAL: S, _lib.F_KKT: S, _lib.F_FIXED: S * N, _lib.F_CONV_PART: 2 * self.P + 2,
                _lib.F_OMEGA: S, _lib.F_Z: S * N, _lib.F_SMOOTH_P: S * N, _lib.F_SMOOTH_BETA: S * N}[field]

    def get(self, field):
        out = np.empty(self._count(field))
        _lib.check(self.lib.phg_get(self.h, field, ptr(out)))
        return out

    def set(self, field, values):
        a = as_f64(np.broadcast_to(np.asarray(values, np.float64), (self._count(field),)).copy())
        _lib.check(self.lib.phg_set(self.h, field, ptr(a)))

    def results(self, x=True):
        """(status, iters, kkt, obj, bound, x or None) of the last solve in one synchronisation
        (``phg_solve_results``); x is [S, n]."""
        S = self.S
        st, it = np.empty(S, np.int32), np.empty(S, np.int32)
        kkt, obj, bnd = np.empty(S), np.empty(S), np.empty(S)
        X = np.empty((S, self.batch.n)) if x else None
        _lib.check(self.lib.phg_solve_results(self.h, ptr(st), ptr(it), ptr(kkt), ptr(obj), ptr(bnd),
                                              ptr(X) if x else None))
        return st, it, kkt, obj, bnd, X

    def get_i32(self, field):
        out = np.empty(self.S, np.int32)
        _lib.check(self.lib.phg_get_i32(self.h, field, ptr(out)))
        return out

    # ------------------------------------------------------------------ hot path
    def solve(self, w_on, prox_on, eps=1e-9, max_iter=100000, check_every=32, warm_start=3,
              fix_nonants=False, schedule=True, beta=(0.0, 0.0, 0.0), theta=0.0, skip_below=0.0, fix_tol=0.0,
              safe_bound=False):
        """safe_bound: every scenario's F_BOUND is a valid outer bound whatever its status (bound.hip;
        2: a weak-duality certificate also for the converged scenarios, whose own dual objective is
        accurate to eps on either side;
        -inf / +inf only where the dual iterate yields no finite certificate)."""
        o = _lib.PhgOpts(float(eps), int(max_iter), int(check_every), int(warm_start),
                         int(bool(fix_nonants)), int(bool(schedule)), *[float(v) for v in beta],
                         float(theta), float(skip_below), float(fix_tol), int(safe_bound))
        self.last_safe_bound = bool(safe_bound) and not fix_nonants
        import ctypes
        _lib.check(self.lib.phg_solve(self.h, int(w_on), int(prox_on), ctypes.byref(o)))

    def sync(self):
        _lib.check(self.lib.phg_sync(self.h))

    # views of the packed exchange buffer (multi-GPU)
    @property
    def nodesum_view(self):
        return None if self.exchange is None else self.exchange[: 2 * self.N_tot]

    @property
    def convpart_view(self):
        return None if self.exchange is None else self.exchange[2 * self.N_tot:]

    def _ns_ptr(self):
        return None if self.exchange is None else self.exchange.data_ptr()

    def _cp_ptr(self):
        return None if self.exchange is None else self.exchange.data_ptr() + 8 * 2 * self.N_tot

    def node_sums(self):
        _lib.check(self.lib.phg_node_sums(self.h, self._ns_ptr()))

    def apply_xbar(self):
        _lib.check(self.lib.phg_apply_xbar(self.h, self._ns_ptr(), self._cp_ptr()))

    def ph_head(self, convthresh, first):
        """Gated W update of the pipelined iteration (phg_ph_head): conv of the previous update from
        the exchanged partials; unless it is below ``convthresh``, xbar / W / this update's partials."""
        _lib.check(self.lib.phg_ph_head(self.h, self._ns_ptr(), float(convthresh), int(bool(first))))

    def ph_step(self, convthresh, first):
        """One GPU (no exchange): node sums + the gated W update of the pipelined iteration, fused into
        one launch where the batch allows it (phg_ph_step).  Returns True if the fused kernel ran."""
        if self.exchange is not None:
            raise RuntimeError("ph_step is the single-GPU form: exchange the node sums with ph_head")
        fused = np.zeros(1, np.int32)
        _lib.check(self.lib.phg_ph_step(self.h, float(convthresh), int(bool(first)), ptr(fused)))
        return bool(fused[0])

    def set_col_bounds(self, lo, hi):
        """New column bounds ([S, n], the models' units) without reloading (phg_set_col_bounds)."""
        lo = as_f64(np.asarray(lo, np.float64).reshape(-1))
        hi = as_f64(np.asarray(hi, np.float64).reshape(-1))
        if lo.size != self.S * self.batch.n or hi.size != lo.size:
            raise ValueError("set_col_bounds: need S * n lower and upper bounds")
        _lib.check(self.lib.phg_set_col_bounds(self.h, ptr(lo), ptr(hi)))

    def set_tail(self, convthresh):
        """Run the next iteration's PH update at the end of the next solve (phg_set_tail): one GPU,
        node sums + gate + next x-bar, which the following ph_step takes over; with an exchange
        buffer, node sums + partials into it, which the following node_sums takes over."""
        mode = 2 if self.exchange is not None else 1
        _lib.check(self.lib.phg_set_tail(self.h, mode, float(convthresh), self._ns_ptr()))

    def tail_info(self):
        """The solve tail's state (phg_tail_info, synchronises): units, final slots, counters not
        re-armed (0 between launches), and the last solve's tail mode."""
        out = np.zeros(4, np.int32)
        _lib.check(self.lib.phg_tail_info(self.h, ptr(out)))
        return {"units": int(out[0]), "final_slots": int(out[1]), "armed_counters": int(out[2]),
                "last_mode": int(out[3])}

    def set_fold(self, on):
        """Folded PH update on / off (phg_set_fold); returns whether this batch's solves take it."""
        out = np.zeros(1, np.int32)
        _lib.check(self.lib.phg_set_fold(self.h, int(bool(on)), ptr(out)))
        return bool(out[0])

    def fold_partials(self):
        """Reduce the per-scenario partials of a folded W update (the last solve's prologue) into the
        exchange buffer's partials region (phg_fold_partials; no-op when none is pending) -- before
        that region is all-reduced."""
        _lib.check(self.lib.phg_fold_partials(self.h, self._cp_ptr()))

    def solve_undo(self):
        """Restore the solve state from before the last solve (phg_solve_undo)."""
        _lib.check(self.lib.phg_solve_undo(self.h))

    def conv_start(self):
        _lib.check(self.lib.phg_conv_start(self.h, self._cp_ptr()))

    def conv_wait(self):
        import ctypes
        v = ctypes.c_double()
        _lib.check(self.lib.phg_conv_wait(self.h, ctypes.byref(v)))
        return v.value

    def conv_finish(self):
        import ctypes
        v = ctypes.c_double()
        _lib.check(self.lib.phg_conv_finish(self.h, self._cp_ptr(), ctypes.byref(v)))
        return v.value

    def copy_from(self, src, field):
        """Device-to-device copy of ``field`` from another handle on the same GPU (stream-ordered)."""
        _lib.check(self.lib.phg_copy_from(self.h, src.h, int(field)))

    def fix_from(self, src, scen):
        """Fix every scenario's nonants to ``src``'s scenario ``scen`` nonants (two-stage xhat)."""
        _lib.check(self.lib.phg_fix_from(self.h, src.h, int(scen)))

    def idle(self):
        out = np.zeros(1, np.int32)
        _lib.check(self.lib.phg_query(self.h, ptr(out)))
        return bool(out[0])

    def set_smoothing(self, on):
        _lib.check(self.lib.phg_set_smoothing(self.h, int(bool(on))))

    def solve_summary(self):
        """(scenarios not at the KKT tolerance, numerical failures) of the solve preceding the last
        PH update, as read back by :meth:`conv_finish` (summed over GPUs)."""
        out = np.zeros(2, np.int32)
        _lib.check(self.lib.phg_solve_summary(self.h, ptr(out)))
        return int(out[0]), int(out[1])

    def eval_objective(self, w_on, prox_on):
        _lib.check(self.lib.phg_eval_objective(self.h, int(w_on), int(prox_on)))
        return self.get(_lib.F_EVAL)

    def timing_reset(self, solves=True, updates=False):
        _lib.check(self.lib.phg_timing_reset(self.h, int(bool(solves)) | (2 if updates else 0)))

    def timing(self, which):
        """(total ms, launches, PDHG iterations summed over scenarios) since timing_reset."""
        import ctypes
        ms, n, it = ctypes.c_double(), ctypes.c_int32(), ctypes.c_int64()
        _lib.check(self.lib.phg_timing(self.h, int(which), ctypes.byref(ms), ctypes.byref(n), ctypes.byref(it)))
        return ms.value, n.value, it.value
