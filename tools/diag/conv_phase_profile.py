"""Where the 10k conv leg's time goes, by PH phase (diagnostic, GPU): farmer cm=10 x 10 000, the
pipelined loop to conv < 1e-4 as bench.py's conv leg; every 250 PH iterations a read-only,
pipeline-safe extension records the wall time and the last solve's PDHG iteration counts
(mean / max; I_ITERS, one sync).  Prints one JSON line."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import _pkg  # noqa: E402

_pkg.load()
from mpisppy_amd import _lib  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402
from mpisppy_amd.extensions.extension import Extension  # noqa: E402
from mpisppy_amd.ph import PH  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
EVERY = 250
rec = []


class Probe(Extension):
    pipeline_safe = True

    def miditer(self):
        k = self.opt._PHIter
        if k % EVERY == 0 or k in (2, 5, 10, 20, 50, 100):
            it = self.opt.engine.get_i32(_lib.I_ITERS)
            rec.append({"ph_iter": k, "t": time.perf_counter(), "pdhg_mean": float(it.mean()),
                        "pdhg_max": int(it.max()), "conv": self.opt.conv})


opts = {"solver_name": "phg", "PHIterLimit": 20000, "defaultPHrho": 1.0, "convthresh": 1e-4,
        "verbose": False, "display_progress": False}
ph = PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator,
        scenario_creator_kwargs={"crops_multiplier": 10, "num_scens": S}, extensions=Probe)
ph.PH_Prep()
t0 = time.perf_counter()
conv, eobj, tb = ph.ph_main(finalize=False)
t1 = time.perf_counter()
for r in rec:
    r["t"] = round(r["t"] - t0, 4)
seg = []
for a, b in zip(rec, rec[1:]):
    n = b["ph_iter"] - a["ph_iter"]
    seg.append({"from": a["ph_iter"], "to": b["ph_iter"], "ms_per_ph_iter": round((b["t"] - a["t"]) / n * 1e3, 4),
                "pdhg_mean_at_start": round(a["pdhg_mean"], 1), "pdhg_max_at_start": a["pdhg_max"]})
print(json.dumps({"scenarios": S, "seconds": round(t1 - t0, 3), "ph_iters": ph._PHIter, "conv": conv,
                  "probes_note": "each probe adds one device sync (I_ITERS read)", "segments": seg}))
