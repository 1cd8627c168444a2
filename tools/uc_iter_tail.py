"""Per-scenario PDHG iteration counts of the UC case over PH iterations: where the launch time of
the bordered kernel goes (the slowest scenario sets it).  Prints, per PH iteration, percentiles of
the iterations per scenario, the slowest scenarios, their status / final omega.

Usage: python tools/uc_iter_tail.py [S] [ph_iters] [eps]
"""
import os
import sys
import json
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkg  # noqa: E402

_pkg.load()
from mpisppy_amd import _lib  # noqa: E402
from mpisppy_amd.examples import uc  # noqa: E402
from mpisppy_amd.ph import PH  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    eps = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-6
    so = {"pdhg_eps": eps, **json.loads(os.environ.get("UC_OPTS", "{}"))}   # e.g. '{"pdhg_primal_weight_theta": 0.5}'
    o = {"solver_name": "phg", "PHIterLimit": K, "defaultPHrho": 1.0, "convthresh": 0.0, "verbose": False,
         "display_progress": False, "iter0_solver_options": so, "iterk_solver_options": so}
    ph = PH(o, uc.scenario_names_creator(S), uc.scenario_creator, scenario_creator_kwargs={"num_scens": S})
    ph.PH_Prep()
    t0 = time.perf_counter()
    ph.Iter0()
    eng = ph.engine

    tot = []

    def report(tag, t0):
        it = eng.get_i32(_lib.I_ITERS).copy()   # (synchronises with the solve)
        dt = time.perf_counter() - t0
        st = eng.get_i32(_lib.I_STATUS).copy()
        om = eng.get(_lib.F_OMEGA).copy()
        order = np.argsort(-it)
        tot.append((dt, int(it.max()), float(it.mean())))
        print(f"{tag}: {dt * 1e3:.0f} ms  iters p50 {np.percentile(it, 50):.0f} p90 {np.percentile(it, 90):.0f} "
              f"max {it.max()} mean {it.mean():.0f}  status {np.bincount(st, minlength=3).tolist()}  slowest "
              + ", ".join(f"s{k}:{it[k]}/om {om[k]:.3g}" for k in order[:4]), flush=True)

    report("Iter0", t0)
    for k in range(1, K + 1):
        ph.Compute_Xbar()
        ph.Update_W()
        t0 = time.perf_counter()
        ph.solve_loop(solver_options=ph.current_solver_options)
        report(f"PH {k}", t0)
    ph_ = tot[1:]
    print(f"SUMMARY {os.environ.get('UC_OPTS', '{}')}: PH 1..{K} {sum(t for t, _, _ in ph_) * 1e3:.0f} ms, "
          f"mean max iters {np.mean([m for _, m, _ in ph_]):.0f}, mean iters {np.mean([a for _, _, a in ph_]):.0f}", flush=True)


if __name__ == "__main__":
    main()
