"""Re-solve dumped stuck scenarios on the GPU: cold, then warm repeats."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import _pkg
_pkg.load()
from mpisppy_amd import _lib
from mpisppy_amd.examples import farmer
from mpisppy_amd.ph import PH
d = np.load(os.path.join(ROOT, "tools", "_diag", "diag_dump.npz"))
S, N = 10000, 30
bad = d["bad"]
W = d["W"].reshape(S, N)[bad]
names = [f"scen{k}" for k in bad]
opts = {"solver_name": "phg", "PHIterLimit": 1, "defaultPHrho": 1.0, "convthresh": 1e-4,
        "verbose": False, "display_progress": False, "pdhg_max_iter": 20000}
ph = PH(opts, names, farmer.scenario_creator, scenario_creator_kwargs={"crops_multiplier": 10, "num_scens": S})
ph.PH_Prep()
e = ph.engine
e.set(_lib.F_W, W.ravel()); e.set(_lib.F_XBAR, d["xbar"])
for rep, warm in enumerate([False, True, True, False]):
    e.solve(1, 1, eps=1e-9, max_iter=20000, check_every=64, warm_start=warm)
    e.sync()
    print(rep, "warm" if warm else "cold", e.get_i32(_lib.I_ITERS), e.get(_lib.F_KKT))
for eps in [1e-8, 1e-10]:
    e.solve(1, 1, eps=eps, max_iter=20000, check_every=64, warm_start=False); e.sync()
    print("eps", eps, e.get_i32(_lib.I_ITERS), e.get(_lib.F_KKT))
