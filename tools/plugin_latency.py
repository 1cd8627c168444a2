"""Per-solve latency of the ``phg`` solver plugin under the reference's own PH loop.

The reference's ``solve_loop`` calls ``SPOpt.solve_one`` once per local scenario
(``mpisppy/spopt.py:99-247``), each on its own persistent plugin (``_create_solvers``,
``spopt.py:876-893``); the xhat evaluation fixes a candidate's nonants in place before a solve and
frees them after (``_fix_nonants`` / ``_restore_nonants``, ``spopt.py:588-640``).  This tool runs
exactly that through ``SolverFactory("phg")`` on farmer (cm=1) with S plugins -- one engine each --
and times every ``solve_one`` call on the host clock (the plugin synchronises on each solve):

* Iter0 + ``--iters`` PH iterations (the solve's objective re-read, the solve, the result reads);
* ``--xhat`` candidate evaluations: fix all nonants at x-bar (``update_var``), solve, free them,
  solve again (the bound change goes to the loaded engine, ``phg_set_col_bounds``).

One JSON line per S.  Run on the GPU box:  python tools/plugin_latency.py --scen 3 1000
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests"))
import _pkg  # noqa: E402  (the package directory "mpi-sppy_amd" imported as mpisppy_amd)

_pkg.load()


PROFILE = False


def _stats(ts):
    a = np.asarray(ts) * 1e3
    return {"n": int(a.size), "median_ms": round(float(np.median(a)), 4), "mean_ms": round(float(a.mean()), 4),
            "p90_ms": round(float(np.percentile(a, 90)), 4), "max_ms": round(float(a.max()), 4)}


def run(S, iters, xhat):
    from test_gpu_f4 import _SolveOnePH, spopt_solve_one   # the reference's solve_one, restated
    from oracle import models as om

    t0 = time.perf_counter()
    o = _SolveOnePH(dict(defaultPHrho=1.0, PHIterLimit=iters, convthresh=-1.0), om.farmer_names(S), om.farmer,
                    dict(crops_multiplier=1, num_scens=S), persistent=True)
    t_setup = time.perf_counter() - t0
    times = []
    solve_one = o.solve_one

    def timed(k):
        t = time.perf_counter()
        solve_one(k)
        times.append(time.perf_counter() - t)
    o.solve_one = timed
    t0 = time.perf_counter()
    o.Iter0()
    t_iter0 = time.perf_counter() - t0
    first = list(times)
    times.clear()
    t0 = time.perf_counter()
    if PROFILE:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
    o.iterk_loop()
    t_loop = time.perf_counter() - t0
    if PROFILE:
        pr.disable()
        pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(30)
    ph_times = list(times)
    # xhat candidates: fix every nonant at x-bar, solve, free, solve (spopt.py:588-640)
    fix_t, free_t = [], []
    for k in range(min(xhat, S)):
        s = o.models[k]
        for i, j in enumerate(s.cols):
            s.vars[j].fixed, s.vars[j].value = True, float(o.xbar[k, i])
            s._solver_plugin.update_var(s.vars[j])
        t = time.perf_counter()
        spopt_solve_one(s, o.is_minimizing, True)
        fix_t.append(time.perf_counter() - t)
        for j in s.cols:
            s.vars[j].fixed = False
            s._solver_plugin.update_var(s.vars[j])
        t = time.perf_counter()
        spopt_solve_one(s, o.is_minimizing, True)
        free_t.append(time.perf_counter() - t)
    pdhg_it = sum(m._solver_plugin.pdhg_iterations for m in o.models)
    n_solves = sum(m._solver_plugin.solves for m in o.models)
    rebuilds = sorted({m._solver_plugin.rebuilds for m in o.models})
    bu = sum(m._solver_plugin.bound_updates for m in o.models)
    for m in o.models:
        m._solver_plugin.close()
    # the batched PH on the same instance for comparison: one engine, one launch per PH iteration
    import torch
    from mpisppy_amd.examples import farmer
    from mpisppy_amd.ph import PH
    ph = PH({"solver_name": "phg", "PHIterLimit": iters, "defaultPHrho": 1.0, "convthresh": -1.0,
             "verbose": False, "display_progress": False},
            farmer.scenario_names_creator(S), farmer.scenario_creator,
            scenario_creator_kwargs=dict(crops_multiplier=1, num_scens=S))
    ph.PH_Prep()
    ph.Iter0()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ph.iterk_loop()
    torch.cuda.synchronize()
    t_batched = (time.perf_counter() - t0) / iters
    from mpisppy_amd import _lib
    b_it = float(ph.engine.get_i32(_lib.I_ITERS).mean())
    ph.engine.close()
    return {"scenarios": S, "plugins": S, "setup_s": round(t_setup, 3),
            "iter0_first_solve": _stats(first), "iter0_s": round(t_iter0, 3),
            "ph_iterations": iters, "ph_solve": _stats(ph_times), "ph_loop_s": round(t_loop, 3),
            "ph_iteration_ms": round(t_loop / iters * 1e3, 3),
            "xhat_fixed_solve": _stats(fix_t) if fix_t else None,
            "xhat_freed_solve": _stats(free_t) if free_t else None,
            "rebuilds_per_plugin": rebuilds, "bound_updates": bu,
            "pdhg_iterations_per_solve": round(pdhg_it / max(1, n_solves), 1),
            "warm_bits": os.environ.get("PHG_PLUGIN_WARM", "3"),
            "batched_ph_iteration_ms": round(t_batched * 1e3, 4),
            "batched_per_scenario_us": round(t_batched / S * 1e6, 3),
            "batched_pdhg_iterations_last": round(b_it, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scen", type=int, nargs="+", default=[3, 1000])
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--xhat", type=int, default=20)
    ap.add_argument("--out", default=None)
    ap.add_argument("--profile", action="store_true", help="cProfile of the PH loop to stderr")
    a = ap.parse_args()
    global PROFILE
    PROFILE = a.profile
    rows = []
    for S in a.scen:
        r = run(S, a.iters, a.xhat)
        print(json.dumps(r), flush=True)
        rows.append(r)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
