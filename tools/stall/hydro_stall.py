"""The hydro 20 000 MFMA prox-QP stall: Iter0, one PH update, the prox solve
(test_hydro_mfma_full_size_properties_and_sampled_parity's sequence) at STALL_THETA / STALL_CHECK;
prints the scenarios that end at status 1 (run again with PHG_WATCH_SCEN=s for the check history)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _pkg  # noqa: E402

_pkg.load()
from mpisppy_amd import _lib  # noqa: E402
from mpisppy_amd.examples import hydro  # noqa: E402
from mpisppy_amd.ph import PH  # noqa: E402

torch.cuda.set_device(0)
S = 20000
fan = hydro.synthetic_fanouts(S)
o = {"solver_name": "phg", "PHIterLimit": 3, "defaultPHrho": 1.0, "convthresh": 1e-10, "verbose": False,
     "display_progress": False, "iterk_solver_options": {"pdhg_eps": 1e-9}, "iter0_solver_options": {"pdhg_eps": 1e-9}}
if os.environ.get("STALL_THETA"):
    o["pdhg_primal_weight_theta"] = float(os.environ["STALL_THETA"])
if os.environ.get("STALL_CHECK"):
    o["pdhg_check_every"] = int(os.environ["STALL_CHECK"])
ph = PH(o, hydro.scenario_names_creator(S), hydro.synthetic_scenario_creator, all_nodenames=hydro.synthetic_nodenames(fan),
        scenario_creator_kwargs={"fanouts": fan})
ph.PH_Prep()
ph.Iter0()
ph.Compute_Xbar()
ph.Update_W()
ph.solve_loop()
st = ph.engine.get_i32(_lib.I_STATUS)
it = ph.engine.get_i32(_lib.I_ITERS)
bad = np.nonzero(st != 0)[0]
print("status counts", np.bincount(st + 1), "max iters", it.max(), flush=True)
for s in bad[:8]:
    print(f"STALL {s} iters {it[s]} status {st[s]}", flush=True)
