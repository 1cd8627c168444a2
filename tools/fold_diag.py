"""Where does the folded W update (phg_set_fold) part from the two-launch update?  Runs the pipelined
PH iteration on farmer (S scenarios) with and without the fold on two handles side by side and
reports, per iteration, the largest |W| / xN / xbar difference and the first differing element.

Usage: python tools/fold_diag.py [S] [cm] [iters]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import _pkg  # noqa: E402

_pkg.load()
from mpisppy_amd import _lib  # noqa: E402
from mpisppy_amd.examples import farmer  # noqa: E402
from mpisppy_amd.ph import PH  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    cm = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    phs = []
    for fold in (True, False):
        o = {"solver_name": "phg", "PHIterLimit": iters, "defaultPHrho": 1.0, "convthresh": 0.0,
             "verbose": False, "display_progress": False}
        ph = PH(o, farmer.scenario_names_creator(S), farmer.scenario_creator,
                scenario_creator_kwargs={"crops_multiplier": cm, "num_scens": S})
        ph.PH_Prep()
        ph.Iter0()
        print("fold active" if ph.engine.set_fold(fold) else "fold off", flush=True)
        # the folded update takes x = xs dc (the scaled state times the column scaling); the two-launch
        # update takes the epilogue's xN -- are they the same bits?
        xN = ph.engine.get(_lib.F_XN).reshape(S, ph.engine.N)
        xu = ph.engine.get(_lib.F_X).reshape(S, -1)[:, ph.engine.batch.nonant_col]
        print("  xN vs xs*dc after Iter0: max |diff|", float(np.abs(xN - xu).max()),
              "differing", int((xN != xu).sum()), "of", xN.size, flush=True)
        phs.append(ph)
    xN0 = phs[1].engine.get(_lib.F_XN).copy()
    for k in range(1, iters + 1):
        for ph in phs:
            ph.engine.ph_step(0.0, k == 1)
            ph.solve_loop(solver_options=ph.current_solver_options, skip_below=0.0, safe_bound=False)
            ph.engine.conv_wait()
        a, b = phs
        # xN before anything flushes the pending update: the solve's nonants
        xa, xb = a.engine.get(_lib.F_XN), b.engine.get(_lib.F_XN)
        xba, xbb = a.engine.get(_lib.F_XBAR), b.engine.get(_lib.F_XBAR)
        Wa, Wb = a.engine.get(_lib.F_W), b.engine.get(_lib.F_W)   # (fold: flushes nothing -- applied by the solve)
        dW, dx, dxb = np.abs(Wa - Wb), np.abs(xa - xb), np.abs(xba - xbb)
        line = f"it {k}: max|dW| {dW.max():.3e} max|dxN| {dx.max():.3e} max|dxbar| {dxb.max():.3e}"
        if k == 1:   # W_1 = rho (x_0 - xbar_1) with rho = 1, W_0 = 0: exact on the host
            Wh = xN0 - np.tile(xba, S)
            line += (f"\n  host W_1: fold differs in {int((Wa != Wh).sum())}, two-launch in {int((Wb != Wh).sum())} of {Wh.size}"
                     f"; xbar_1 fold == two-launch: {bool((xba == xbb).all())}")
        if dW.max() > 0:
            e = int(np.argmax(dW > 0))
            line += f"  first W diff at {e} (s {e // a.engine.N}, k {e % a.engine.N}): {Wa[e]!r} vs {Wb[e]!r}"
        print(line, flush=True)
        if dW.max() > 0 or dx.max() > 0:
            break


if __name__ == "__main__":
    main()
