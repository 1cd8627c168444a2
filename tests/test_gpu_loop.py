"""GPU: the pipelined PH iteration (PHBase.update_and_solve) against the sequential one at the loop's
exits -- a time limit tripping mid-run (the drained conv must stay in conv_history) and
the PHIterLimit exit -- on farmer cm=10, 30 scenarios.  The time limit is made deterministic by
patching PHBase._time_over to trip at a given iteration."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from mpisppy_amd.examples import farmer  # noqa: E402
from mpisppy_amd.ph import PH  # noqa: E402


def _run(pipeline, trip_at=None, limit=12, tail=False):
    # (tail=False: the separate-launch pipeline; the solve's fused tail gives the same bits:
    # test_gpu_parity.test_solve_tail_matches_separate_launches)
    opts = {"solver_name": "phg", "PHIterLimit": limit, "defaultPHrho": 1.0, "convthresh": 1e-10,
            "verbose": False, "display_progress": False, "pdhg_pipeline": pipeline,
            "time_limit": 1e9 if trip_at else None, "pdhg_tail": tail}
    ph = PH(opts, farmer.scenario_names_creator(30), farmer.scenario_creator,
            scenario_creator_kwargs={"crops_multiplier": 10, "num_scens": 30})
    if trip_at:
        ph._time_over = lambda: ph._PHIter >= trip_at
    ph.ph_main(finalize=False)
    return ph


@pytest.mark.parametrize("trip_at", [None, 1, 2, 5])
def test_pipelined_exits_match_sequential(trip_at):
    a, b = _run(True, trip_at), _run(False, trip_at)
    assert a._PHIter == b._PHIter
    assert len(a.conv_history) == len(b.conv_history) == a._PHIter
    np.testing.assert_allclose(a.conv_history, b.conv_history, rtol=1e-12)
    np.testing.assert_array_equal(a.Ws(), b.Ws())
    np.testing.assert_array_equal(a.nonants(), b.nonants())
    np.testing.assert_array_equal(a.xbars(), b.xbars())


@pytest.mark.parametrize("trip_at", [None, 2, 5])
def test_tail_pipeline_exits_match_sequential(trip_at):
    """The same exits with the PH update fused into the solve's tail (ph_tail.h): the drain after the
    time limit / PHIterLimit must discard the last tail's staged x-bar and recompute conv from the
    partials -- the state equals the sequential loop's bit for bit (W, x, x-bar; conv summed in the
    folded update's order, 1e-12)."""
    a, b = _run(True, trip_at, tail=True), _run(False, trip_at)
    assert a._PHIter == b._PHIter
    assert len(a.conv_history) == len(b.conv_history) == a._PHIter
    np.testing.assert_allclose(a.conv_history, b.conv_history, rtol=1e-12)
    np.testing.assert_array_equal(a.Ws(), b.Ws())
    np.testing.assert_array_equal(a.nonants(), b.nonants())
    np.testing.assert_array_equal(a.xbars(), b.xbars())


def test_ungated_solve_after_converged_head_is_fresh():
    """a head that found conv below its convthresh leaves the folded W update pending; a
    later solve the caller does NOT gate (a final or extension solve after PH converged) must run --
    W untouched (the reference breaks before Update_W, phbase.py:1008-1010) and every output fresh --
    instead of inheriting the head's gate and silently keeping the previous launch's values."""
    from mpisppy_amd import _lib
    opts = {"solver_name": "phg", "PHIterLimit": 4, "defaultPHrho": 1.0, "convthresh": 1e-10,
            "verbose": False, "display_progress": False}
    ph = PH(opts, farmer.scenario_names_creator(30), farmer.scenario_creator,
            scenario_creator_kwargs={"crops_multiplier": 10, "num_scens": 30})
    ph.PH_Prep()
    ph.Iter0()
    ph.current_solver_options = ph.iterk_solver_options
    for k in range(3):
        ph.update_and_solve(first=k == 0)
    eng = ph.engine
    if not eng.set_fold(True):
        pytest.skip("this batch's layout does not take the folded update")
    W0 = eng.get(_lib.F_W)           # (nothing pending: the last gated solve applied its update)
    eng.ph_step(1e30, False)        # conv < 1e30: the head keeps x-bar and leaves W alone
    assert eng.conv_wait() < 1e30
    eng.solve(1, 1, eps=1e-9, max_iter=32, check_every=32, warm_start=1, skip_below=0.0)
    it = eng.get_i32(_lib.I_ITERS)
    np.testing.assert_array_equal(eng.get(_lib.F_W), W0)     # the flushed update was gated: W unchanged
    # this launch's counts (<= its cap of 32), not the last PH solve's (hundreds at eps 1e-9)
    assert ((it > 0) & (it <= 32)).all(), it


def test_launch_schedule_in_the_node_sum_launch():
    """The next solve's launch order (schedule.h: heaviest first by the last solve's PDHG iterations in
    check-interval units) computed by the extra workgroup of the pipelined node-sum launch
    (node_sums_kernel HEADX) or on its own launch (PHG_SCHED_FUSE=0): after every pipelined
    iteration the order is a permutation of the scenarios whose buckets never increase along it for
    one of the recent solves' counts, and the two paths give bit-identical PH states."""
    import os
    from mpisppy_amd import _lib

    def run(fuse):
        if fuse:
            os.environ.pop("PHG_SCHED_FUSE", None)
        else:
            os.environ["PHG_SCHED_FUSE"] = "0"
        try:
            S = 3000
            opts = {"solver_name": "phg", "PHIterLimit": 20, "defaultPHrho": 1.0, "convthresh": 1e-10,
                    "verbose": False, "display_progress": False}
            ph = PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator,
                    scenario_creator_kwargs={"crops_multiplier": 10, "num_scens": S})
            ph.PH_Prep()
            ph.Iter0()
            ph.current_solver_options = ph.iterk_solver_options
            unit = ph._solver_opts()["pdhg_check_every"]
            eng = ph.engine
            recent = [eng.get_i32(_lib.I_ITERS)]
            for k in range(9):
                ph.update_and_solve(first=k == 0)
                recent.append(eng.get_i32(_lib.I_ITERS))   # (a due schedule reads this solve's counts)
                order = eng.get_i32(_lib.I_ORDER)
                assert np.array_equal(np.sort(order), np.arange(S)), k
                bad = [int((np.diff(np.minimum(it // unit, 4095)[order]) > 0).sum()) for it in recent[-5:]]
                assert min(bad) == 0, (k, fuse, bad)
            return ph.Ws().copy(), ph.nonants().copy(), ph.xbars().copy()
        finally:
            os.environ.pop("PHG_SCHED_FUSE", None)

    a, b = run(True), run(False)
    for u, v in zip(a, b):
        np.testing.assert_array_equal(u, v)


def test_one_hop_node_sum_head_matches_two_hops():
    """node_sums_kernel HEADX: every rank forming conv itself and writing its own x-bar (one hand-off,
    the default) gives the state of the two-hand-off form (PHG_HEADX_ONEHOP=0) bit for bit, conv
    history included."""
    import os
    runs = []
    for v in ("0", None):
        if v is None:
            os.environ.pop("PHG_HEADX_ONEHOP", None)
        else:
            os.environ["PHG_HEADX_ONEHOP"] = v
        try:
            runs.append(_run(True, None, limit=12))
        finally:
            os.environ.pop("PHG_HEADX_ONEHOP", None)
    a, b = runs
    assert a._PHIter == b._PHIter
    np.testing.assert_array_equal(a.conv_history, b.conv_history)
    np.testing.assert_array_equal(a.Ws(), b.Ws())
    np.testing.assert_array_equal(a.nonants(), b.nonants())
    np.testing.assert_array_equal(a.xbars(), b.xbars())
