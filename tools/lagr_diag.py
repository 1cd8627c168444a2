"""Diagnostics of the Lagrangian bound at the north-star's converged W (farmer cm=10): PH to conv
< 1e-4 on the GPU, then the Lagrangian solve (W on, prox off) at a given PDHG cap with safe bounds;
dumps W, statuses, iterations, KKT, objectives, bounds and the unscaled x / y of every scenario to an
npz for CPU analysis (tools/lagr_analyze.py).  Usage: python tools/lagr_diag.py S CAP OUT.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkg  # noqa: E402

_pkg.load()
import torch  # noqa: E402
from mpisppy_amd import _lib  # noqa: E402
from mpisppy_amd.engine import Engine  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402
from mpisppy_amd.ph import PH  # noqa: E402


def main():
    S, cap, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    torch.cuda.set_device(0)
    opts = {"solver_name": "phg", "PHIterLimit": 20000, "defaultPHrho": 1.0, "convthresh": 1e-4,
            "verbose": False, "display_progress": False,
            "iter0_solver_options": {"pdhg_eps": 1e-9}, "iterk_solver_options": {"pdhg_eps": 1e-9}}
    ph = PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator,
            scenario_creator_kwargs={"crops_multiplier": 10, "num_scens": S})
    conv, eobj, tb = ph.ph_main()
    print(f"PH iters {ph._PHIter} conv {conv:.3e} Eobj {eobj:.6f}", flush=True)
    W = ph.Ws().copy()
    xbar = ph.xbars().copy()
    res = {"W": W, "xbar": xbar, "Eobj": eobj}
    for tag, warm in (("cold", 0), ("hub1", 1), ("hub3", 3), ("hub5", 5)):
        eng = Engine(ph.engine.batch, device=0, presolve=True)
        eng.copy_from(ph.engine, _lib.F_W)
        if warm:
            eng.copy_from(ph.engine, _lib.F_WARM)
        eng.solve(1, 0, eps=1e-9, max_iter=cap, check_every=32, warm_start=warm, schedule=False, safe_bound=True)
        eng.sync()
        st = eng.get_i32(_lib.I_STATUS)
        res[tag + "_status"] = st
        res[tag + "_iters"] = eng.get_i32(_lib.I_ITERS)
        res[tag + "_kkt"] = eng.get(_lib.F_KKT)
        res[tag + "_obj"] = eng.get(_lib.F_OBJ)
        res[tag + "_bound"] = eng.get(_lib.F_BOUND)
        res[tag + "_x"] = eng.get(_lib.F_X).reshape(S, -1)
        res[tag + "_y"] = eng.get(_lib.F_Y).reshape(S, -1)
        p = ph.engine.batch.prob
        print(f"{tag}: statuses {np.bincount(st, minlength=3).tolist()}, bound {float(p @ res[tag + '_bound']):.6f}",
              flush=True)
        eng.close()
    np.savez(out, **res)


if __name__ == "__main__":
    main()
