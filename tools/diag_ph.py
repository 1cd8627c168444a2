"""Diagnostics: per-PH-iteration PDHG launch time / iteration statistics on the GPU."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
import _pkg
_pkg.load()
from mpisppy_amd import _lib
from mpisppy_amd.examples import farmer
from mpisppy_amd.ph import PH

S = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 300
eps = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-9
cm = int(sys.argv[4]) if len(sys.argv) > 4 else 10
opts = {"solver_name": "phg", "PHIterLimit": iters, "defaultPHrho": 1.0, "convthresh": 1e-4,
        "verbose": False, "display_progress": False, "pdhg_eps": eps,
        "pdhg_keep_omega": (sys.argv[5] != "0") if len(sys.argv) > 5 else True,
        "pdhg_max_iter": int(sys.argv[6]) if len(sys.argv) > 6 else 200000}
ph = PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator,
        scenario_creator_kwargs={"crops_multiplier": cm, "num_scens": S})
ph.PH_Prep()
ph.Iter0()
e = ph.engine
its = e.get_i32(_lib.I_ITERS)
rows = [dict(k=0, ms=e.last_ms(0), mean=float(its.mean()), max=int(its.max()),
             p99=float(np.percentile(its, 99)), bad=int((e.get_i32(_lib.I_STATUS) != 0).sum()))]
t0 = time.perf_counter()
for k in range(1, iters + 1):
    ph.Compute_Xbar(); ph.Update_W(); conv = ph.convergence_diff()
    if conv < 1e-4:
        break
    ph.solve_loop()
    its = e.get_i32(_lib.I_ITERS)
    st = e.get_i32(_lib.I_STATUS)
    om = e.get(_lib.F_OMEGA)
    rows.append(dict(k=k, conv=conv, ms=e.last_ms(0), mean=float(its.mean()), max=int(its.max()),
                     om_min=float(om.min()), om_med=float(np.median(om)), om_max=float(om.max()),
                     p99=float(np.percentile(its, 99)), bad=int((st != 0).sum())))
    if k % 25 == 0:
        print(json.dumps(rows[-1]), flush=True)
print("total", time.perf_counter() - t0, flush=True)
json.dump(rows, open(os.path.join(ROOT, "gpurun_out", f"diag_{S}_{eps}_{sys.argv[5] if len(sys.argv) > 5 else 1}.json"), "w"))
