"""Host-side cost of the pipelined PH iteration (PHBase.update_and_solve + iterk_loop's own
bookkeeping) on the farmer 10k instance: the wall time per PH iteration next to the GPU time per
iteration (solve launch + node sums, from the library's HIP events), and a cProfile of the loop's
Python work.  If the host's time per iteration exceeds the GPU's, the GPU idles between launches.

    python tools/conv_host_profile.py [ITERS] > out.txt
"""
import cProfile
import os
import pstats
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import _pkg  # noqa: E402

_pkg.load()


def main(iters=400, warm=3000):
    import torch
    from mpisppy_amd.examples import farmer
    from mpisppy_amd.ph import PH
    S = 10000
    ph = PH({"solver_name": "phg", "PHIterLimit": iters + warm, "defaultPHrho": 1.0, "convthresh": 1e-12,
             "verbose": False, "display_progress": False},
            farmer.scenario_names_creator(S), farmer.scenario_creator,
            scenario_creator_kwargs={"crops_multiplier": 10, "num_scens": S})
    ph.PH_Prep()
    ph.Iter0()
    torch.cuda.synchronize()
    eng = ph.engine
    # late PH iterations (the solves get cheaper as PH converges: the conv leg's regime)
    for k in range(warm):
        ph.update_and_solve(first=k == 0)
    torch.cuda.synchronize()
    # wall time per pipelined iteration, no events
    t0 = time.perf_counter()
    for k in range(iters // 2):
        ph.update_and_solve(first=False)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / (iters // 2)
    # the same with the solve / update launches timed on the device
    eng.timing_reset(solves=True, updates=True)
    for k in range(iters // 4):
        ph.update_and_solve(first=False)
    torch.cuda.synchronize()
    sv_ms, n_sv, _ = eng.timing(0)
    up_ms, n_up, _ = eng.timing(1)
    eng.timing_reset(solves=False, updates=False)
    print(f"wall per PH iteration {wall * 1e3:.4f} ms; solve launch {sv_ms / max(1, n_sv):.4f} ms, "
          f"update launch {up_ms / max(1, n_up):.4f} ms (device events)")
    # host-only cost: the Python / API work of an iteration whose device work is already done
    pr = cProfile.Profile()
    pr.enable()
    t0 = time.perf_counter()
    for k in range(iters // 4):
        ph.update_and_solve(first=False)
    torch.cuda.synchronize()
    pr.disable()
    print(f"profiled wall per PH iteration {(time.perf_counter() - t0) / (iters // 4) * 1e3:.4f} ms")
    pstats.Stats(pr, stream=sys.stdout).sort_stats("tottime").print_stats(25)
    eng.close()


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]))
