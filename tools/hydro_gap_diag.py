"""Diagnostic: obj-vs-bound gaps of the hydro prox-QP solves at 20 000 scenarios, per layout."""
import sys
import numpy as np
sys.path.insert(0, ".")
import _pkg  # noqa: E402
_pkg.load()
from mpisppy_amd import _lib  # noqa: E402
from mpisppy_amd.examples import hydro  # noqa: E402
from mpisppy_amd.ph import PH  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
for layout in sys.argv[2:] or ["mfma", "gather"]:
    fan = hydro.synthetic_fanouts(S)
    o = {"solver_name": "phg", "PHIterLimit": 3, "defaultPHrho": 1.0, "convthresh": 1e-10, "verbose": False,
         "display_progress": False, "pdhg_layout": layout,
         "iterk_solver_options": {"pdhg_eps": 1e-9}, "iter0_solver_options": {"pdhg_eps": 1e-9}}
    ph = PH(o, hydro.scenario_names_creator(S), hydro.synthetic_scenario_creator,
            all_nodenames=hydro.synthetic_nodenames(fan), scenario_creator_kwargs={"fanouts": fan})
    ph.PH_Prep()
    ph.Iter0()
    for tag in ("iter0", "prox"):
        if tag == "prox":
            ph.Compute_Xbar()
            ph.Update_W()
            ph.solve_loop()
        e = ph.engine
        obj, bnd, kkt = e.get(_lib.F_OBJ), e.get(_lib.F_BOUND), e.get(_lib.F_KKT)
        st, it = e.get_i32(_lib.I_STATUS), e.get_i32(_lib.I_ITERS)
        gap = np.abs(obj - bnd) / (1.0 + np.abs(obj))
        k = int(np.argmax(gap))
        print(layout, tag, "status", np.bincount(st + 1).tolist(), "gap max", gap.max(), "n>1e-6", int((gap > 1e-6).sum()),
              "worst", k, obj[k], bnd[k], "kkt", kkt[k], "iters", it[k], "median it", float(np.median(it)), flush=True)
