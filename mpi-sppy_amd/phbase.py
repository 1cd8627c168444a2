"""PHBase on the MI355X engine (restates ``mpisppy/phbase.py`` + the solve plumbing of
``mpisppy/spopt.py``).

The public surface matches the reference -- ``PHBase(options, all_scenario_names,
scenario_creator, scenario_denouement=None, all_nodenames=None, mpicomm=None,
scenario_creator_kwargs=None, extensions=None, extension_kwargs=None, ph_converger=None,
rho_setter=None, variable_probability=None)``, ``Iter0``, ``iterk_loop``, ``post_loops``,
``Compute_Xbar``, ``Update_W``, ``convergence_diff``, ``Ebound``, ``Eobjective``, ``_update_E1``,
``feas_prob``, ``_populate_W_cache``, ``W_from_flat_list``, ``disable_W_and_prox`` ... -- and the
order of operations in ``Iter0`` / ``iterk_loop`` (``phbase.py:829-1061``) is kept line for line.
What changes is underneath: every local scenario lives in one GPU batch (``engine.Engine``), the
solve loop is one batched PDHG launch, and xbar / W / conv are device kernels whose cross-rank SUMs
go through the communicator (RCCL).  Nothing of size S x n crosses PCIe inside the PH loop; each
iteration reads back one convergence scalar (2 x virtual-rank doubles).

Documented deviations: per-subproblem extension hooks ``pre_solve``/``post_solve`` cannot run
inside a batched launch (``pre_solve_loop``/``post_solve_loop`` do); ``linearize_proximal_terms``
raises (the kernels solve the exact prox QP).  ``variable_probability`` (``prob_coeff`` per nonant,
``prob0_mask``) and smoothed PH are supported.
"""
import math
import os
import time

import numpy as np

from . import _lib
from .engine import BatchArrays, Engine
from .spbase import SPBase

# PDHG controls read from iter0_solver_options / iterk_solver_options (other solver options,
# e.g. "mipgap" or "threads", belong to CPU solvers and are ignored)
def _omega_bits(keep):
    """pdhg_keep_omega: False re-initialises the primal weight every solve, True carries it over
    (phg_opts.warm_start bit 1), "blend" starts from the geometric mean of the carried and the fresh
    estimate (bit 2)."""
    if keep == "blend":
        return 4
    return 2 if keep else 0


# pdhg_check_every None: by layout (check_every_default)
_SOLVER_DEFAULTS = {"pdhg_eps": 1e-9, "pdhg_max_iter": 200000, "pdhg_check_every": None, "pdhg_keep_omega": None,
                    "pdhg_schedule": True, "pdhg_beta_sufficient": 0.0, "pdhg_beta_necessary": 0.0,
                    "pdhg_beta_artificial": 0.0, "pdhg_primal_weight_theta": 0.0}


def check_every_default(layout, threads=0):
    """PDHG restart / termination check interval by kernel layout (measured on MI355X): 64 for the
    one-wave-per-scenario gather kernel (tiny subproblems: hydro 2 000, 6.2 vs 5.3 M solves/s, the
    slowest scenario 704 vs 1 024 PDHG iterations, time to PH conv 0.029 vs 0.34 s over the same
    ~104 PH iterations) and the workgroup-block kernel (netdes 1 024: 19.9 vs 22.0 ms per PH
    iteration, sslp 4 096: 5.50 vs 5.65 ms) and the shared-matrix MFMA kernel (hydro 20 000, round
    5: 0.565 vs 0.688 ms per PH iteration; 96 / 128: 0.80 / 0.77 ms; its round-2 parity miss at 64
    predates the gap test on the whole objective), 32 elsewhere (farmer: 40 / 48 / 64 cost time to
    conv)."""
    # (Round 5 gave the 256-thread block kernel 96 with an artificial-restart fraction of 0.15, from
    # the per-iteration time of sslp_15_45_10 early in PH.  Held out, round 6 (profiles/r06/heldout_ab.json):
    # on sslp_5_25_50 the pair reached conv 1.3e-3 in 120 s against 4.1e-4 at 64 / 0.25 (23.7 vs
    # 13.2 ms per PH iteration over the run; 96 alone: 1.3e-2 in 60 s), and on sslp_15_45_10 itself
    # the time to conv was 27.7 vs 26.2 s -- so it is gone.)
    return 64 if layout in ("gather", "block", "mfma") else 32


def keep_omega_default(layout):
    """pdhg_keep_omega by layout: the primal weight re-estimated at every solve on the shared-matrix
    MFMA kernel (hydro 20 000 at check interval 64: 0.537 vs 0.565 ms per PH iteration with the
    blend, 1.60 ms carried -- round 5), the blend elsewhere (farmer: DESIGN.md (d) round 2)."""
    return False if layout == "mfma" else "blend"


def beta_artificial_default(layout, threads=0):
    """PDHG artificial-restart fraction by kernel layout (0: the library's 0.25), from round 5's
    sweeps on MI355X (`profiles/r05/betaart/`, `profiles/r05/uc/sweep/`):
    * bordered / range-split (UC 64, eps 1e-7): PDLP's 0.36 -- 477 vs 581 ms per PH iteration
      (0.5: 478, 0.6: 507, 0.8: 536);
    * workgroup block: the library's 0.25.  (Round 5's 0.15 for 256-thread workgroups -- 5.24-5.26
      vs 5.46-5.47 ms per PH iteration on sslp 4 096 -- lost the time to PH conv on the held-out
      sslp_5_25_50 and on sslp_15_45_10 itself in round 6: see check_every_default);
    * wave gather (hydro 2 000): per iteration 0.15 -- 0.318 vs 0.325 ms (0.1: 0.315, 0.36: 0.353),
      but see below;
    * lane-local (farmer 10k): the library's 0.25 (0.15: 0.2924, 0.2: 0.2897, 0.36: 0.3009 vs
      0.2885 ms).
    (The one-wave-per-scenario shared-matrix kernel, on request for block-kernel problems, follows
    the block kernel.)
    Time to PH conv decides where the per-iteration gain does not carry over: the gather kernel's
    0.15 made hydro 2 000's conv leg 0.141 vs 0.030 s over the same 105 PH iterations, and netdes'
    1 024-thread block kernel converged in 37.3 vs 32.8 s -- both keep the library's 0.25."""
    return {"border": 0.36, "stream": 0.36, "wave": 0.15}.get(layout, 0.0)


class PHBase(SPBase):
    def __init__(self, options, all_scenario_names, scenario_creator, scenario_denouement=None,
                 all_nodenames=None, mpicomm=None, scenario_creator_kwargs=None, extensions=None,
                 extension_kwargs=None, ph_converger=None, rho_setter=None,
                 variable_probability=None):
        self._PHIter = 0
        super().__init__(options, all_scenario_names, scenario_creator,
                         scenario_denouement=scenario_denouement, all_nodenames=all_nodenames,
                         mpicomm=mpicomm, scenario_creator_kwargs=scenario_creator_kwargs,
                         variable_probability=variable_probability)
        self.options = options
        self.options_check()
        self.ph_converger = ph_converger
        self.rho_setter = rho_setter
        self.iter0_solver_options = options.get("iter0_solver_options") or {}
        self.iterk_solver_options = options.get("iterk_solver_options") or {}
        self.current_solver_options = self.iter0_solver_options
        self.convobject = None
        self.extensions = extensions
        self.extension_kwargs = extension_kwargs
        self.extobject = None
        if extensions is not None:
            self.extobject = extensions(self) if extension_kwargs is None else extensions(self, **extension_kwargs)
        self.engine = None
        self.W_on = 0
        self.prox_on = 0
        self.start_time = time.perf_counter()
        self.conv = None
        self.solve_count = 0

    # ------------------------------------------------------------------------------- options
    def options_check(self):
        """``phbase.py:791-826``."""
        required = ["solver_name", "PHIterLimit", "defaultPHrho", "convthresh", "verbose", "display_progress"]
        missing = [k for k in required if k not in self.options]
        if missing:
            raise ValueError(f"Missing option(s): {missing}")
        self.options.setdefault("display_timing", False)
        self.options.setdefault("display_convergence_detail", False)
        self.options.setdefault("smoothed", 0)
        self.options.setdefault("time_limit", None)
        if self.options["smoothed"]:
            for k in ("defaultPHp", "defaultPHbeta"):
                if k not in self.options:
                    raise ValueError(f"smoothed PH needs option {k}")
        if self.options.get("linearize_proximal_terms"):
            raise NotImplementedError("linearize_proximal_terms: the engine solves the exact prox QP")

    # ------------------------------------------------------------------------------- engine
    def _virt_nproc(self):
        return int(self.options.get("virtual_nproc", self.n_proc))

    def _create_solvers(self):
        """Build the GPU batch (replaces SolverFactory per subproblem, ``spopt.py:876-913``)."""
        if self.engine is not None:
            return
        models = [self.local_scenarios[n] for n in self.local_scenario_names]
        prob = [m._mpisppy_probability for m in models]
        batch = BatchArrays(models, self.all_nodenames, prob, self.scen_global0,
                            len(self.all_scenario_names), self._virt_nproc())
        # how the values cross the C ABI (phg_batch.vals_form: 0 per scenario, 1 shared, 2 delta list)
        batch.vals_form = int(self.options.get("pdhg_vals_form", _lib.VALS_PER_SCENARIO))
        device, stream, exchange = self._device_setup(batch)
        self.engine = Engine(batch, device=device, stream=stream, exchange=exchange,
                             layout=self.options.get("pdhg_layout", "auto"),
                             presolve=self.options.get("pdhg_presolve", True))
        if hasattr(self.mpicomm, "attach"):   # comm.PhgGroupComm: the library's own RCCL group
            self.mpicomm.attach(self.engine)
        self.engine.set(_lib.F_RHO, float(self.options["defaultPHrho"]))

    def _device_setup(self, batch):
        device = int(self.options.get("device", 0))
        stream = None
        exchange = None
        try:
            import torch
            if torch.cuda.is_available():
                device = torch.cuda.current_device() if "device" not in self.options else device
                stream = torch.cuda.current_stream(device).cuda_stream
                # one packed buffer, one all-reduce per pipelined iteration (pdhg_exchange: also on
                # one rank, to run the exchange path through a 1-rank communicator in tests)
                if self.n_proc > 1 or self.options.get("pdhg_exchange", False):
                    exchange = torch.zeros(2 * batch.N_tot + 2 * batch.virt_nproc + 3, dtype=torch.float64,
                                           device=f"cuda:{device}")
        except ImportError:
            pass
        return device, stream, exchange

    def _solver_opts(self):
        o = dict(_SOLVER_DEFAULTS)
        for k in _SOLVER_DEFAULTS:
            if k in self.options:
                o[k] = self.options[k]
            if self.current_solver_options and k in self.current_solver_options:
                o[k] = self.current_solver_options[k]
        if o["pdhg_check_every"] is None:
            o["pdhg_check_every"] = check_every_default(getattr(self.engine, "layout", "auto"),
                                                        getattr(self.engine, "lanes_per_scenario", 0))
        if o["pdhg_keep_omega"] is None:
            o["pdhg_keep_omega"] = keep_omega_default(getattr(self.engine, "layout", "auto"))
        if not o["pdhg_beta_artificial"]:
            o["pdhg_beta_artificial"] = beta_artificial_default(getattr(self.engine, "layout", "auto"),
                                                                getattr(self.engine, "lanes_per_scenario", 0))
        return o

    # ------------------------------------------------------------------------------- W / prox
    def attach_Ws_and_prox(self):
        self.W_on = 0
        self.prox_on = 0

    def PH_Prep(self, attach_duals=True, attach_prox=True, attach_smooth=0):
        """``phbase.py:763-788``: W, rho, xbar (and the smoothing z, p, beta of
        ``attach_smoothing``, ``phbase.py:641-655``) live on the device; W_on = prox_on = 0."""
        self.attach_Ws_and_prox()
        self._attach_duals = attach_duals
        self._attach_prox = attach_prox
        self._attach_smooth = attach_smooth
        self._create_solvers()
        if attach_smooth:
            self.engine.set(_lib.F_Z, 0.0)
            self.engine.set(_lib.F_SMOOTH_P, float(self.options["defaultPHp"]))
            self.engine.set(_lib.F_SMOOTH_BETA, float(self.options["defaultPHbeta"]))
            self.engine.set_smoothing(True)

    def _disable_prox(self):
        self.prox_on = 0

    def _disable_W(self):
        self.W_on = 0

    def disable_W_and_prox(self):
        self._disable_W()
        self._disable_prox()

    def _reenable_prox(self):
        self.prox_on = 1

    def _reenable_W(self):
        self.W_on = 1

    def reenable_W_and_prox(self):
        self._reenable_W()
        self._reenable_prox()

    @property
    def W_disabled(self):
        return not bool(self.W_on)

    @property
    def prox_disabled(self):
        return not bool(self.prox_on)

    # ------------------------------------------------------------------------------- solves
    def solve_loop(self, solver_options=None, use_scenarios_not_subproblems=False, dtiming=False,
                   dis_W=False, dis_prox=False, gripe=False, disable_pyomo_signal_handling=False,
                   tee=False, verbose=False, need_solution=True, warm_start=True, skip_below=0.0,
                   safe_bound=None):
        """``phbase.py:522-603`` + ``spopt.py:250-341``: one batched launch for all local scenarios.
        skip_below > 0 makes the launch a device-side no-op when the conv of the last
        ``engine.conv_start`` is below it (see :meth:`update_and_solve`).  safe_bound (default: the
        ``pdhg_safe_bound`` option, on) makes every scenario's outer bound valid whatever its status
        (``phg_opts.safe_bound``); the pipelined hub solves leave it off (nothing reads their bounds)."""
        if safe_bound is None:
            safe_bound = bool(self.options.get("pdhg_safe_bound", True))
        saved = (self.W_on, self.prox_on)
        if dis_W:
            self._disable_W()
        if dis_prox:
            self._disable_prox()
        if self.extobject is not None:
            self.extobject.pre_solve_loop()
        if solver_options is not None:
            self.current_solver_options = solver_options
        o = self._solver_opts()
        w_on = int(self.W_on and getattr(self, "_attach_duals", True))
        prox_on = int(self.prox_on and getattr(self, "_attach_prox", True))
        t0 = time.perf_counter()
        self.engine.solve(w_on, prox_on, eps=o["pdhg_eps"], max_iter=o["pdhg_max_iter"],
                          check_every=o["pdhg_check_every"],
                          warm_start=(1 | _omega_bits(o["pdhg_keep_omega"])) if warm_start else 0,
                          schedule=o["pdhg_schedule"],
                          beta=(o["pdhg_beta_sufficient"], o["pdhg_beta_necessary"], o["pdhg_beta_artificial"]),
                          theta=o["pdhg_primal_weight_theta"], skip_below=skip_below, safe_bound=safe_bound)
        self.solve_count += self.engine.S
        # The launch is asynchronous: the statuses reach the host with the next convergence
        # readback (phg_solve_summary, checked in convergence_diff), so a PH iteration costs one
        # host synchronisation; feas_prob / infeas_prob (Iter0) and dtiming fetch them at once.
        self._status_pending = (gripe, need_solution)
        if dtiming:
            self._check_status_now(gripe, need_solution)
        if dtiming and self.cylinder_rank == 0:
            print(f"batched solve of {self.engine.S} subproblems: {time.perf_counter() - t0:.4f} s")
        if self.extobject is not None:
            self.extobject.post_solve_loop()
        self.W_on, self.prox_on = saved if (dis_W or dis_prox) else (self.W_on, self.prox_on)

    def _check_status_now(self, gripe, need_solution):
        """Per-scenario statuses of the last solve (synchronous; spopt.py:194-231 semantics)."""
        status = self.engine.get_i32(_lib.I_STATUS)
        self._status = status
        self._feasible = status != 2
        self._status_pending = None
        if gripe and (status != 0).any():
            bad = [self.local_scenario_names[i] for i in np.nonzero(status != 0)[0][:5]]
            print(f"[{self.__class__.__name__}] {int((status != 0).sum())} subproblem(s) did not reach "
                  f"the KKT tolerance (first: {bad})")
        if need_solution and (status == 2).any():
            raise RuntimeError("PDHG numerical failure (NaN) in scenario(s) "
                               f"{[self.local_scenario_names[i] for i in np.nonzero(status == 2)[0][:5]]}")

    def _check_status_summary(self):
        """Deferred status check of the solve before this PH update (counts summed over ranks)."""
        pend = getattr(self, "_status_pending", None)
        if pend is None:
            return
        gripe, need_solution = pend
        self._status_pending = None
        n_bad, n_nan = self.engine.solve_summary()
        if gripe and n_bad and self.cylinder_rank == 0:
            print(f"[{self.__class__.__name__}] {n_bad} subproblem(s) did not reach the KKT tolerance")
        if need_solution and n_nan:
            raise RuntimeError(f"PDHG numerical failure (NaN) in {n_nan} subproblem(s)")

    # ------------------------------------------------------------------------------- PH update
    def Compute_Xbar(self, verbose=False):
        """``phbase.py:32-112``: node sums on the device, SUM across ranks (RCCL)."""
        self.engine.node_sums()
        if self.engine.exchange is not None:
            self.mpicomm.allreduce_sum_(self.engine.nodesum_view)
        self._xbar_pending = True

    def Update_W(self, verbose=False):
        """``phbase.py:301-326``: W += rho (x - xbar) (fused with the conv partials)."""
        self.engine.apply_xbar()
        self._xbar_pending = False

    def Update_z(self, verbose=False):
        """``phbase.py:329-346`` z += beta (x - z): fused into the Update_W kernel (same x, same
        iteration) whenever smoothing is attached, so there is nothing left to launch here."""
        return None

    def convergence_diff(self):
        """``phbase.py:349-371``: mean over (virtual) ranks of the per-rank mean |x - xbar|."""
        if self.engine.exchange is not None:
            self.mpicomm.allreduce_sum_(self.engine.convpart_view)
        conv = self.engine.conv_finish()
        self._check_status_summary()
        return conv

    def _can_pipeline(self):
        """The pipelined iteration (:meth:`update_and_solve`) enqueues the solve before the host
        has seen conv, so nothing may act between convergence_diff and solve_loop: no extension
        (miditer), no converger object, no per-solve timing.  (A time limit is checked before the
        solve is enqueued, see :meth:`iterk_loop`.)"""
        o = self.options
        ext_ok = self.extobject is None or bool(getattr(self.extobject, "pipeline_safe", False))
        return (ext_ok and self.ph_converger is None
                and not o.get("display_timing", False) and o.get("pdhg_pipeline", True))

    def _apply_eps_schedule(self):
        """Built-in PDHG tolerance schedule (``options["pdhg_eps_schedule"]``): pairs (conv_above,
        eps) in order; the next solve runs at the eps of the first pair whose conv_above the last
        known convergence metric reaches (+inf before the first metric), and the schedule never
        loosens again once it has tightened.  The reference's mechanism for a per-iteration solver
        tolerance is ``current_solver_options`` (set by extensions such as the Gapper,
        ``extensions/mipgapper.py:15-60``); this sets ``current_solver_options["pdhg_eps"]`` from the
        metric instead of the iteration number.  In the pipelined loop the last known metric is
        conv_{k-2} when solve k is enqueued (one iteration of lag)."""
        sched = self.options.get("pdhg_eps_schedule")
        if not sched:
            return
        conv = math.inf if self.conv is None else float(self.conv)
        idx = len(sched) - 1
        for i, (above, _eps) in enumerate(sched):
            if conv >= above:
                idx = i
                break
        idx = max(idx, getattr(self, "_eps_sched_idx", 0))
        self._eps_sched_idx = idx
        if self.current_solver_options is None:
            self.current_solver_options = {}
        self.current_solver_options["pdhg_eps"] = float(sched[idx][1])

    def update_and_solve(self, verbose=False, first=False):
        """One pipelined PH iteration k with ONE all-reduce (include/phg.h, phg_ph_head).

        The device runs: node sums of x_{k-1} into the packed exchange buffer; one SUM across GPUs
        of [node sums | partials of update k-1]; conv_{k-1} from those partials; and, unless
        conv_{k-1} < convthresh, Compute_Xbar / Update_W of iteration k and its partials; then
        solve_loop k, gated on conv_{k-1} too.  The host waits for conv_{k-1} only, while update k
        and solve k run.  So the solve is speculative by one iteration: conv_{k-1} < convthresh
        means the reference broke at iteration k-1 BEFORE solve k-1 (``phbase.py:1008-1010``);
        the device has skipped update k and solve k, and with the double-buffered solve state
        (a gated solve writes nothing) the state is the one before solve k-1.

        Returns conv_{k-1} (+inf when ``first``: no update precedes iteration 1)."""
        eng = self.engine
        thr = float(self.options["convthresh"])
        if eng.exchange is not None:
            eng.node_sums()
            self.mpicomm.allreduce_sum_(eng.exchange)
            eng.ph_head(thr, first)
        else:   # one GPU: node sums and the gated W update in one launch (phg_ph_step)
            eng.ph_step(thr, first)
        # the next iteration's node sums (+ head on one GPU) at the end of this solve's launch
        # (include/phg.h phg_set_tail; taken over by the next ph_step / node_sums when the solve ran)
        tail = self.options.get("pdhg_tail")
        if tail is None:   # (off by default until it measures faster: DESIGN.md (d) round 5; PHG_TAIL=1 on)
            tail = os.environ.get("PHG_TAIL", "0") == "1"
        if thr > 0 and tail and hasattr(eng, "set_tail"):
            eng.set_tail(thr)
        self.solve_loop(solver_options=self.current_solver_options, gripe=verbose, verbose=verbose,
                        skip_below=thr if thr > 0 else 0.0, safe_bound=False)
        self._spec_pending = True
        conv = eng.conv_wait()
        if not first:
            # statuses of the solve that preceded update k-1 (they ride with its partials)
            n_bad, n_nan = eng.solve_summary()
            if verbose and n_bad and self.cylinder_rank == 0:
                print(f"[{self.__class__.__name__}] {n_bad} subproblem(s) did not reach the KKT tolerance")
            if n_nan:
                raise RuntimeError(f"PDHG numerical failure (NaN) in {n_nan} subproblem(s)")
        if conv < thr:
            # solve k did nothing and solve k-1 is undone (its state swap is reverted by solve k's)
            self.solve_count -= 2 * eng.S
            self._spec_pending = False
        return conv

    def _drain_speculation(self):
        """Finish the pipeline: conv of the last pipelined update (the partials not yet exchanged)
        and, if PH had converged before the solve that followed it, undo that solve.  Returns
        (conv, undone)."""
        eng = self.engine
        eng.fold_partials()        # a folded W update's partials (include/phg.h), before the SUM
        if eng.exchange is not None:
            self.mpicomm.allreduce_sum_(eng.convpart_view)
        conv = eng.conv_finish()
        self._spec_pending = False
        if eng.solve_summary()[1]:
            raise RuntimeError(f"PDHG numerical failure (NaN) in {eng.solve_summary()[1]} subproblem(s)")
        if conv < float(self.options["convthresh"]):
            eng.solve_undo()
            self.solve_count -= eng.S
            self._status_pending = (False, True)    # the front solve state changed: refetch statuses
            return conv, True
        return conv, False

    def _time_over(self):
        if self.options["time_limit"] is None:
            return False
        over = (time.perf_counter() - self.start_time) >= self.options["time_limit"]
        if self.n_proc > 1:
            over = self.mpicomm.allreduce_scalar(float(over)) > 0
        return over

    # ------------------------------------------------------------------------------- expectations
    def _rank_fsum(self, vals):
        local = math.fsum(vals)
        return self.mpicomm.allreduce_scalar(local) if self.n_proc > 1 else local

    def _valid_bounds(self):
        """Per-scenario outer bounds of the last solve, model sense.  With safe bounds (the default
        for every solve whose bounds are read, ``phg_opts.safe_bound``) each is a weak-duality
        certificate whatever the scenario's status -- -inf / +inf where none exists, as a solver that
        reports no Lower_bound would leave it (spopt.py:225-230).  Without, the PDHG dual objective
        counts only at a KKT-optimal point (status 0): an iteration-limited or failed scenario's dual
        iterate may be infeasible on infinite-bound columns, so its bound is the trivial one."""
        b = self.engine.get(_lib.F_BOUND)
        self._statuses()
        if getattr(self.engine, "last_safe_bound", False):
            bad = (self._status == 2) | ~np.isfinite(b)
        else:
            bad = self._status != 0
        if bad.any():
            b = b.copy()
            b[bad] = -math.inf if self.is_minimizing else math.inf
        return b

    def Ebound(self, verbose=False, extra_sum_terms=None):
        """``spopt.py:377-422`` (outer bound = the solver's dual bound, see :meth:`_valid_bounds`)."""
        b = self._valid_bounds()
        p = self.engine.batch.prob
        vals = [p[k] * b[k] for k in range(len(b))]
        if extra_sum_terms is None:
            return self._rank_fsum(vals)
        arr = np.array([math.fsum(vals)] + list(extra_sum_terms))
        if self.n_proc > 1:
            arr = self.mpicomm.allreduce_array(arr)
        return arr[0], arr[1:]

    def Eobjective(self, verbose=False):
        """``spopt.py:344-374``: sum p_s * pyo.value(objfct) with the current W/prox toggles."""
        w_on = int(self.W_on and getattr(self, "_attach_duals", True))
        prox_on = int(self.prox_on and getattr(self, "_attach_prox", True))
        ev = self.engine.eval_objective(w_on, prox_on)
        p = self.engine.batch.prob
        return self._rank_fsum([p[k] * ev[k] for k in range(len(ev))])

    def _update_E1(self):
        self.E1 = self._rank_fsum(list(self.engine.batch.prob))

    def _statuses(self):
        if getattr(self, "_status_pending", None) is not None or not hasattr(self, "_status"):
            self._check_status_now(*(getattr(self, "_status_pending", None) or (False, True)))
        return self._feasible

    def feas_prob(self):
        self._statuses()
        p = self.engine.batch.prob
        return self._rank_fsum([p[k] for k in range(len(p)) if self._feasible[k]])

    def infeas_prob(self):
        self._statuses()
        p = self.engine.batch.prob
        return self._rank_fsum([p[k] for k in range(len(p)) if not self._feasible[k]])

    # ------------------------------------------------------------------------------- caches
    def _populate_W_cache(self, cache, padding):
        """``phbase.py:374-394``: local W in local-scenario x nonant order."""
        W = self.engine.get(_lib.F_W)
        if len(W) + padding != len(cache):
            raise RuntimeError(f"W cache length mismatch: total W len {len(W)} but cache len {len(cache)}")
        cache[:len(W)] = W

    def W_from_flat_list(self, flat_list):
        """``phbase.py:397-413``."""
        self.engine.set(_lib.F_W, np.asarray(flat_list[: self.engine.S * self.engine.N], np.float64))

    def _save_nonants(self):
        self._load_solutions()

    def _save_original_nonants(self):
        pass

    def _load_solutions(self):
        """Copy x back into the scenario models (only at finalisation / on request)."""
        X = self.engine.get(_lib.F_X).reshape(self.engine.S, -1)
        for k, sname in enumerate(self.local_scenario_names):
            self.local_scenarios[sname]._solution = X[k]

    # convenient views
    def nonants(self):
        return self.engine.get(_lib.F_XN).reshape(self.engine.S, self.engine.N)

    def Ws(self):
        return self.engine.get(_lib.F_W).reshape(self.engine.S, self.engine.N)

    def xbars(self):
        return self.engine.get(_lib.F_XBAR)

    # ------------------------------------------------------------------------------- loops
    def Iter0(self):
        """``phbase.py:829-946``."""
        if self.extobject is not None:
            self.extobject.pre_iter0()
        verbose = self.options["verbose"]
        dprogress = self.options["display_progress"]
        self._PHIter = 0
        self._create_solvers()
        if self.extobject is not None:
            self.extobject.iter0_post_solver_creation()
        self.solve_loop(solver_options=self.current_solver_options, dtiming=self.options["display_timing"],
                        gripe=True, verbose=verbose, warm_start=False)
        self._update_E1()
        if abs(1 - self.E1) > self.E1_tolerance:
            raise RuntimeError(f"Total probability of scenarios was {self.E1};  E1_tolerance = ", self.E1_tolerance)
        feasP = self.feas_prob()
        if feasP != self.E1:
            raise RuntimeError(f"Infeasibility detected; E_feas={feasP}, E1={self.E1}")
        if self.extobject is not None:
            self.extobject.post_iter0()
        if self.spcomm is not None:
            self.spcomm.sync()
        if self.extobject is not None:
            self.extobject.post_iter0_after_sync()
        if self.rho_setter is not None:
            self._use_rho_setter(verbose and self.cylinder_rank == 0)
        if self.options["smoothed"] == 2 and getattr(self, "_attach_smooth", 0):
            # "ratio" smoothing: p *= rho (phbase.py:918-922)
            self.engine.set(_lib.F_SMOOTH_P, self.engine.get(_lib.F_SMOOTH_P) * self.engine.get(_lib.F_RHO))
        if self.ph_converger is not None:
            self.convobject = self.ph_converger(self)
        self.conv = None
        self.trivial_bound = self.Ebound(verbose)
        if dprogress and self.cylinder_rank == 0:
            print("")
            print("After PH Iteration", self._PHIter)
            print("Trivial bound =", self.trivial_bound)
            print("PHBase Convergence Metric =", self.conv)
            print("Elapsed time: %6.2f" % (time.perf_counter() - self.start_time))
        self.reenable_W_and_prox()
        self.current_solver_options = self.iterk_solver_options
        return self.trivial_bound

    def _use_rho_setter(self, verbose):
        """``phbase.py:415-434``: rho_setter(scenario) -> [(vardata, rho)] (vardata or its id)."""
        rho = self.engine.get(_lib.F_RHO).reshape(self.engine.S, self.engine.N)
        for k, sname in enumerate(self.local_scenario_names):
            s = self.local_scenarios[sname]
            pos = {}
            i = 0
            for nd in s._mpisppy_node_list:
                for v in nd.nonant_vardata_list:
                    pos[id(v)] = i
                    i += 1
            for v, r in self.rho_setter(s, **self.options.get("rho_setter_kwargs", {})):
                rho[k, pos[v if isinstance(v, int) else id(v)]] = r
        self.engine.set(_lib.F_RHO, rho.ravel())

    def iterk_loop(self):
        """``phbase.py:949-1061``.  With :meth:`_can_pipeline`, iteration k runs as
        :meth:`update_and_solve` (one host synchronisation, one all-reduce, the solve speculative
        by one iteration; every break leaves exactly the reference's state: see
        :meth:`_drain_speculation`), otherwise statement by statement."""
        verbose = self.options["verbose"]
        dprogress = self.options["display_progress"]
        thr = self.options["convthresh"]
        self.conv = None
        max_iterations = int(self.options["PHIterLimit"])
        self.conv_history = []
        self.iter_walltimes = []    # perf_counter at the end of every PH iteration (diagnostics)
        pipelined = self._can_pipeline()
        self._spec_pending = False
        for self._PHIter in range(1, max_iterations + 1):
            iteration_start_time = time.time()
            if pipelined and self.options["time_limit"] is not None and self._time_over():
                # leave the pipeline before enqueueing: settle the previous iteration first, then
                # run this one statement by statement (its own time check breaks below)
                if self._spec_pending:
                    c, undone = self._drain_speculation()
                    # either way conv of the previous iteration's update is part of the history
                    # (the sequential loop appended it there)
                    self.conv = c
                    self.conv_history.append(c)
                    if undone:
                        self._PHIter -= 1
                        break
                pipelined = False
            if pipelined:
                # solver-option hooks keyed by the iteration (pipeline-safe extensions: the Gapper)
                # and the conv-keyed eps schedule, before solve k is enqueued
                self._apply_eps_schedule()
                if self.extobject is not None:
                    self.extobject.miditer()
                c = self.update_and_solve(verbose, first=self._PHIter == 1)
                if self._PHIter > 1:
                    self.conv = c
                    self.conv_history.append(c)
                    if c < thr:
                        self._PHIter -= 1       # the reference broke at the previous iteration
                        break
            else:
                self.Compute_Xbar(verbose)
                self.Update_W(verbose)
                self.conv = self.convergence_diff()
                self.conv_history.append(self.conv)
                if self.extobject is not None:
                    self.extobject.miditer()
                if self.ph_converger is not None and self.convobject.is_converged():
                    break
                if self.conv is not None and self.conv < thr:
                    break
                if self._time_over():
                    break
                # nothing reads the bounds of the prox-QP solves inside the loop: no
                # safe-bound pass, as in the pipelined form
                self._apply_eps_schedule()
                self.solve_loop(solver_options=self.current_solver_options, dtiming=self.options["display_timing"],
                                gripe=verbose, verbose=verbose, safe_bound=False)
            if self.extobject is not None:
                self.extobject.enditer()
            if self.spcomm is not None:
                self.spcomm.sync()
                if self.spcomm.is_converged():
                    break
            if self.extobject is not None:
                self.extobject.enditer_after_sync()
            self.iter_walltimes.append(time.perf_counter())
            if dprogress and self.cylinder_rank == 0:
                print("")
                print("After PH Iteration", self._PHIter)
                print("Scaled PHBase Convergence Metric=", self.conv)
                print("Iteration time: %6.2f" % (time.time() - iteration_start_time))
                print("Elapsed time:   %6.2f" % (time.perf_counter() - self.start_time))
        else:
            self.mpicomm.Barrier()
        if self._spec_pending:      # PHIterLimit or the hub ended a pipelined loop
            # conv_K of the last update K; below convthresh the reference broke at THIS iteration K
            # before solve K, so the undo restores its state and _PHIter stays K (the in-loop paths
            # decrement because they learn conv one iteration late).  Documented deviation: when a
            # hub sync ran at iteration K it already handed the spokes that speculative solve's
            # nonants (the reference would not have synced at K); the spokes' bounds stay valid.
            c, _undone = self._drain_speculation()
            self.conv = c
            self.conv_history.append(c)

    def post_loops(self, extensions=None):
        """``phbase.py:1064-1119``."""
        self._statuses()          # the last solve's statuses (deferred inside iterk_loop)
        self.mpicomm.Barrier()
        if self.scenario_denouement is not None:
            self._load_solutions()
            for sname, s in self.local_scenarios.items():
                self.scenario_denouement(self.cylinder_rank, sname, s)
        self.mpicomm.Barrier()
        if self.extobject is not None:
            self.extobject.post_everything()
        if self.ph_converger is not None and hasattr(self.convobject, "post_everything"):
            self.convobject.post_everything()
        Eobj = self.Eobjective(self.options["verbose"])
        self.mpicomm.Barrier()
        if self.options["display_progress"] and self.cylinder_rank == 0:
            print("")
            print("Current ***weighted*** E[objective] =", Eobj)
            print("")
        return Eobj
