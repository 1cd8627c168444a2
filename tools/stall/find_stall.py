"""Find PDHG solves that run far past the typical iteration count in the bench's farmer 10k PH
trajectory (bench.py's options, pipelined loop): prints step, scenario, iterations, status, KKT."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _pkg  # noqa: E402

_pkg.load()
from mpisppy_amd import _lib  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402
from mpisppy_amd.ph import PH  # noqa: E402

S = int(os.environ.get("STALL_S", "10000"))
K = int(os.environ.get("STALL_K", "40"))
torch.cuda.set_device(0)
opts = {"solver_name": "phg", "PHIterLimit": K, "defaultPHrho": 1.0, "convthresh": 1e-4, "verbose": False,
        "display_progress": False, "pdhg_layout": "auto", "pdhg_schedule": True, "pdhg_check_every": None,
        "pdhg_beta_artificial": 0.0, "pdhg_beta_sufficient": 0.0, "pdhg_beta_necessary": 0.0,
        "pdhg_primal_weight_theta": 0.0, "pdhg_presolve": True, "pdhg_keep_omega": None,
        "iterk_solver_options": {"pdhg_eps": 1e-9}, "iter0_solver_options": {"pdhg_eps": 1e-9}, "pdhg_exchange": False}
ph = PH(dict(opts), farmer.scenario_names_creator(S), farmer.scenario_creator,
        scenario_creator_kwargs={"crops_multiplier": 10, "num_scens": S})
ph.PH_Prep()
ph.Iter0()
ph.current_solver_options = ph.iterk_solver_options
eng = ph.engine
for k in range(1, K + 1):
    ph.update_and_solve(first=k == 1)
    it = eng.get_i32(_lib.I_ITERS)
    st = eng.get_i32(_lib.I_STATUS)
    s = int(np.argmax(it))
    flag = " <-- STALL" if it[s] >= int(os.environ.get("STALL_MIN", "20000")) else ""
    print(f"step {k:3d} max_iters {int(it[s]):7d} scen {s:6d} status {int(st[s])} median {int(np.median(it))} "
          f"n_status1 {int((st == 1).sum())}{flag}", flush=True)
    if flag and os.environ.get("STALL_STOP"):
        print(f"STALL {k} {s}", flush=True)
        break
