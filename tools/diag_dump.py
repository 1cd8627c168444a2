"""Run PH to a given iteration on the GPU and dump the state of scenarios whose PDHG solve
did not reach the tolerance (for CPU-side investigation)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import _pkg
_pkg.load()
from mpisppy_amd import _lib
from mpisppy_amd.examples import farmer
from mpisppy_amd.ph import PH

S, upto = int(sys.argv[1]), int(sys.argv[2])
opts = {"solver_name": "phg", "PHIterLimit": upto, "defaultPHrho": 1.0, "convthresh": 1e-4,
        "verbose": False, "display_progress": False, "pdhg_max_iter": 20000}
ph = PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator,
        scenario_creator_kwargs={"crops_multiplier": 10, "num_scens": S})
ph.PH_Prep(); ph.Iter0()
e = ph.engine
for k in range(1, upto + 1):
    ph.Compute_Xbar(); ph.Update_W(); conv = ph.convergence_diff()
    W = e.get(_lib.F_W); xbar = e.get(_lib.F_XBAR)
    ph.solve_loop()
    st = e.get_i32(_lib.I_STATUS)
    if (st != 0).sum() >= 5:
        break
bad = np.nonzero(st != 0)[0]
np.savez(os.path.join(ROOT, "gpurun_out", "diag_dump.npz"), W=W, xbar=xbar, bad=bad, k=k,
         kkt=e.get(_lib.F_KKT), iters=e.get_i32(_lib.I_ITERS), xN=e.get(_lib.F_XN), conv=conv)
print("iteration", k, "bad", len(bad), "kkt of bad", e.get(_lib.F_KKT)[bad][:10])
