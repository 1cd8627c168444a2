"""HBM roofline sweep of the fused PH update ("report a sweep S*N in {1e6, 1e7, 1e8}
for the >= 60 % claim").

A synthetic two-stage batch -- S scenarios with N nonants each, one dense row (sum x <= N) -- is
loaded through the C ABI (no solves), the nonants are set to seeded random values, and
node_sums + W update + conv (phg_node_sums / phg_apply_xbar / phg_conv_start+wait) are timed with
the library's HIP events over R repetitions (the update from the node sums' begin to the W update's
end, and each kernel alone).  Algorithmic bytes per update:
8 S N (x read, W read, W write, [rho per scenario ? 1 : 0] rho read) + 8 S + 16 N_tot -- rho is the
same in every scenario here (defaultPHrho), so the W update reads its [N] copy: 3 streams.  The
result is checked on the host (xbar = mean of the nonants, W = rho (x - xbar)) before timing.

Usage: python tools/ph_update_sweep.py [OUT_JSON]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkg  # noqa: E402

_pkg.load()
from mpisppy_amd import _lib  # noqa: E402
from mpisppy_amd.engine import BatchArrays, Engine  # noqa: E402

HBM_PEAK_GBS = 8000.0


def synthetic_batch(S, N):
    b = BatchArrays.__new__(BatchArrays)
    n, m = N, 1
    b.S, b.n, b.m, b.nnz = S, n, m, N
    b.rowptr = np.array([0, N], np.int32)
    b.colidx = np.arange(N, dtype=np.int32)
    b.vals = np.ones((S, N))
    b.c = np.ones((S, n))
    b.cl, b.cu = np.zeros((S, n)), np.full((S, n), 10.0)
    b.rl, b.ru = np.full((S, m), -np.inf), np.full((S, m), float(N))
    b.off = np.zeros(S)
    b.sense = 1
    b.L = 1
    b.level_len = np.array([N], np.int32)
    b.nonant_col = np.arange(N, dtype=np.int32)
    b.N = N
    b.nonant_level = np.zeros(N, np.int32)
    b.nonant_pos = np.arange(N, dtype=np.int32)
    b.all_nodenames = ["ROOT"]
    b.node_off = np.zeros(1, np.int32)
    b.N_tot = N
    b.scen_node = np.zeros((S, 1), np.int32)
    b.prob = np.full(S, 1.0 / S)
    b.prob_coeff = np.full((S, 1), 1.0 / S)
    b.prob_coeff_var = None
    b.scen_global0, b.S_global, b.virt_nproc = 0, S, 1
    return b


def run(S, N, reps=20):
    import torch
    t0 = time.perf_counter()
    eng = Engine(synthetic_batch(S, N), device=torch.cuda.current_device(), presolve=False)
    rng = np.random.default_rng(1134)
    x = rng.uniform(0.0, 10.0, size=S * N)
    eng.set(_lib.F_XN, x)
    eng.set(_lib.F_RHO, 1.0)
    setup = time.perf_counter() - t0
    # correctness on the first update
    eng.node_sums()
    eng.apply_xbar()
    eng.conv_start()
    conv = eng.conv_wait()
    xb = eng.get(_lib.F_XBAR)
    X = x.reshape(S, N)
    xb_host = (X / S).sum(0)
    err_xbar = float(np.abs(xb - xb_host).max() / max(1.0, np.abs(xb_host).max()))
    W = eng.get(_lib.F_W).reshape(S, N)
    err_w = float(np.abs(W - (X - xb[None, :])).max())
    conv_host = float(np.abs(X - xb[None, :]).mean())
    ok = err_xbar < 1e-12 and err_w < 1e-9 and abs(conv - conv_host) <= 1e-9 * max(1.0, conv_host)
    # timed updates (HIP events on the library's stream, PH updates only)
    eng.timing_reset(solves=False, updates=True)
    for _ in range(reps):
        eng.node_sums()
        eng.apply_xbar()
        eng.conv_start()
        eng.conv_wait()
    ms, n_upd, _ = eng.timing(1)
    ns_ms, n_ns, _ = eng.timing(2)
    wu_ms, n_wu, _ = eng.timing(3)
    eng.timing_reset(solves=False, updates=False)
    eng.close()
    avg_s = ms / n_upd / 1e3
    alg = 8 * S * N * 3 + 8 * S + 16 * N
    gbs = alg / avg_s / 1e9
    ns_s, wu_s = ns_ms / max(1, n_ns) / 1e3, wu_ms / max(1, n_wu) / 1e3
    return {"S": S, "N": N, "SN": S * N, "avg_us": round(avg_s * 1e6, 2), "bytes_per_update": alg,
            "achieved_GBs": round(gbs, 1), "frac_hbm": round(gbs / HBM_PEAK_GBS, 4), "updates": n_upd,
            "node_sums_us": round(ns_s * 1e6, 2), "w_update_us": round(wu_s * 1e6, 2),
            # each kernel on its own algorithmic bytes: node sums read x (8 S N), the W update reads x
            # and W and writes W (24 S N)
            "node_sums_GBs": round(8 * S * N / ns_s / 1e9, 1) if n_ns else None,
            "w_update_GBs": round(24 * S * N / wu_s / 1e9, 1) if n_wu else None,
            "check_ok": bool(ok), "err_xbar": err_xbar, "err_w": err_w, "setup_s": round(setup, 2)}


def run_fold(S, N, reps=10):
    """The folded PH iteration (include/phg.h phg_fold_partials): the W update moves into the next
    solve's prologue.  Its cost there is measured as the difference of the same short solve (one
    check trip, max_iter 2) with and without the fold, each preceded by its own update launches
    (fold: node sums + xbar head; no fold: node sums + W update head).  Folded PH update time =
    node sums + head + prologue difference; rate = the SURVEY 3-stream bytes over that time."""
    import torch
    eng = Engine(synthetic_batch(S, N), device=torch.cuda.current_device(), presolve=False)
    eng.set(_lib.F_RHO, 1.0)
    if eng.layout != "local":
        eng.close()
        return {"S": S, "N": N, "skipped": f"layout {eng.layout}: the fold is lane-local only"}
    kw = dict(eps=1e-9, max_iter=2, check_every=2, warm_start=1, schedule=False)
    eng.solve(0, 0, **kw)                       # a consistent x (scaled state and nonants)
    out = {}
    for tag, on in (("fold", True), ("nofold", False)):
        active = eng.set_fold(on)
        eng.ph_step(0.0, True)
        eng.solve(1, 1, **kw)
        eng.sync()
        eng.timing_reset(solves=True, updates=True)
        for _ in range(reps):
            eng.ph_step(0.0, False)
            eng.solve(1, 1, **kw)
        sv_ms, n_sv, _ = eng.timing(0)
        up_ms, n_up, _ = eng.timing(1)
        ns_ms, n_ns, _ = eng.timing(2)
        hd_ms, n_hd, _ = eng.timing(3)
        eng.timing_reset(solves=False, updates=False)
        out[tag] = {"active": active, "solve_us": sv_ms / n_sv * 1e3, "update_us": up_ms / n_up * 1e3,
                    "node_sums_us": ns_ms / max(1, n_ns) * 1e3, "head_us": hd_ms / max(1, n_hd) * 1e3}
    eng.set_fold(True)
    eng.close()
    d_solve = out["fold"]["solve_us"] - out["nofold"]["solve_us"]
    t_fold = out["fold"]["update_us"] + d_solve
    alg = 8 * S * N * 3 + 8 * S + 16 * N
    r = {"S": S, "N": N, "SN": S * N, "bytes_per_update": alg,
         "fold": {k: round(v, 2) if isinstance(v, float) else v for k, v in out["fold"].items()},
         "nofold": {k: round(v, 2) if isinstance(v, float) else v for k, v in out["nofold"].items()},
         "prologue_w_update_us": round(d_solve, 2), "folded_update_us": round(t_fold, 2),
         "unfolded_update_us": round(out["nofold"]["update_us"], 2),
         "folded_GBs": round(alg / (t_fold / 1e6) / 1e9, 1),
         "folded_frac_hbm": round(alg / (t_fold / 1e6) / 1e9 / HBM_PEAK_GBS, 4)}
    return r


def main():
    import torch
    torch.cuda.set_device(0)
    out = []
    cases = ((10000, 100), (100000, 100), (100000, 1000))
    if os.environ.get("SWEEP_CASES"):   # e.g. "100000x1000,10000x100"
        cases = tuple(tuple(int(v) for v in c.split("x")) for c in os.environ["SWEEP_CASES"].split(","))
    only_fold = os.environ.get("SWEEP_ONLY_FOLD") == "1"
    for S, N in (() if only_fold else cases):
        r = run(S, N)
        print(json.dumps(r), flush=True)
        out.append(r)
    fold_cases = ((10000, 100), (100000, 100), (1000000, 100))
    if os.environ.get("SWEEP_FOLD_CASES"):
        fold_cases = tuple(tuple(int(v) for v in c.split("x")) for c in os.environ["SWEEP_FOLD_CASES"].split(","))
    fold = []
    for S, N in fold_cases:
        r = run_fold(S, N)
        print(json.dumps(r), flush=True)
        fold.append(r)
    if len(sys.argv) > 1:
        json.dump({"kernel": "node_sums_kernel + w_update_kernel (+ fused conv gate)",
                   "bytes_formula": "8*S*N*3 + 8*S + 16*N_tot (SURVEY 8(d)3, rho shared: no rho stream)",
                   "timing": "HIP events on the library stream around each update (phg_timing(1))",
                   "results": out,
                   "folded": {"what": "W update in the next solve's prologue; its cost = the solve's time "
                                      "with the fold minus without (one check trip, max_iter 2)",
                              "results": fold}}, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
