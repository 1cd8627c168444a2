"""GPU parity for subproblems larger than a wavefront (workgroup-per-scenario kernel,
pdhg_block.hip): sslp_15_45_10 and netdes network-50-30-H-01 LP relaxations against the CPU oracle
(HiGHS).  LP optima can be non-unique, so iteration 0 is compared on objectives / bounds (1e-6
relative); the prox-QPs of later PH iterations are strictly convex in the nonants, which are then
compared directly (same W / xbar fed to both solvers)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("needs a HIP device", allow_module_level=True)

from mpisppy_amd import _lib  # noqa: E402
from mpisppy_amd.examples import netdes, sslp, uc  # noqa: E402
from mpisppy_amd.ph import PH  # noqa: E402
from oracle import models as om  # noqa: E402
from oracle import ph as oph  # noqa: E402


def _opts(**kw):
    o = {"solver_name": "phg", "PHIterLimit": 3, "defaultPHrho": 1.0, "convthresh": 1e-10,
         "verbose": False, "display_progress": False}
    o.update(kw)
    return o


CASES = {
    "sslp": (lambda S: sslp.scenario_names_creator(S), sslp.scenario_creator, {},
             lambda S: om.sslp_names(S), om.sslp, {}),
    "netdes": (lambda S: netdes.scenario_names_creator(S), netdes.scenario_creator, {"num_scens": 3},
               lambda S: om.netdes_names(S), om.netdes, {"num_scens": 3}),
    # UC-shaped, a small instance of the same generator (6 units x 8 periods)
    "uc_small": (lambda S: uc.scenario_names_creator(S), uc.scenario_creator,
                 {"num_gens": 6, "num_periods": 8, "num_scens": 4},
                 lambda S: om.uc_names(S), om.uc, {"num_gens": 6, "num_periods": 8, "num_scens": 4}),
    # 24 units x 12 periods: the demand / reserve rows (24 nonzeros) link the per-unit blocks
    "uc_mid": (lambda S: uc.scenario_names_creator(S), uc.scenario_creator,
               {"num_gens": 24, "num_periods": 12, "num_scens": 3},
               lambda S: om.uc_names(S), om.uc, {"num_gens": 24, "num_periods": 12, "num_scens": 3}),
}


# held-out instances: the round-5 per-layout defaults were swept on the two
# instances above only
HELDOUT = {
    "sslp_5_25_50": (lambda S: sslp.scenario_names_creator(S), sslp.scenario_creator, {"instance": "sslp_5_25_50"},
                     lambda S: om.sslp_names(S), om.sslp, {"instance": "sslp_5_25_50"}),
    "network-10-20-H-01": (lambda S: netdes.scenario_names_creator(S), netdes.scenario_creator,
                           {"num_scens": 4, "instance": "network-10-20-H-01"},
                           lambda S: om.netdes_names(S), om.netdes, {"num_scens": 4, "instance": "network-10-20-H-01"}),
}


@pytest.mark.parametrize("case", sorted(HELDOUT))
def test_heldout_iter0_and_prox_qp_vs_oracle(case):
    """The held-out sslp_5_25_50 / network-10-20-H-01 LP relaxations on whatever layout AUTO picks:
    Iter0 objectives and bounds at 1e-6 against HiGHS, then two prox-QP rounds with the oracle's W /
    x-bar fed to the device: nonants at 1e-5, objectives at 1e-6."""
    S = 4
    pn, pc, pkw, on, oc, okw = HELDOUT[case]
    ph = PH(_opts(), pn(S), pc, scenario_creator_kwargs=pkw)
    ph.PH_Prep()
    tb = ph.Iter0()
    o = oph.OraclePH(_opts(), on(S), oc, okw)
    otb = o.Iter0()
    assert abs(tb - otb) <= 1e-6 * max(1.0, abs(otb)), (ph.engine.layout, tb, otb)
    np.testing.assert_allclose(ph.engine.get(_lib.F_OBJ), o.obj, rtol=1e-6, atol=1e-6)
    assert (ph.engine.get_i32(_lib.I_STATUS) == 0).all()
    for it in range(2):
        o.Compute_Xbar()
        o.Update_W()
        ph.engine.set(_lib.F_W, o.W.ravel())
        ph.engine.set(_lib.F_XBAR, o.xbar[0])
        ph.solve_loop()
        o.solve_loop()
        xg = ph.nonants()
        xo = np.array([o.nonants(k) for k in range(S)])
        np.testing.assert_allclose(xg, xo, rtol=1e-5, atol=1e-5 * max(1.0, float(np.abs(xo).max())))
        np.testing.assert_allclose(ph.engine.get(_lib.F_OBJ), o.obj, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("case,S", [("sslp", 4), ("netdes", 3)])
def test_iter0_lp_block_kernel(case, S):
    pn, pc, pkw, on, oc, okw = CASES[case]
    ph = PH(_opts(), pn(S), pc, scenario_creator_kwargs=pkw)
    ph.PH_Prep()
    assert ph.engine.layout == "block"
    tb = ph.Iter0()
    o = oph.OraclePH(_opts(), on(S), oc, okw)
    otb = o.Iter0()
    assert abs(tb - otb) <= 1e-6 * abs(otb), (tb, otb)
    np.testing.assert_allclose(ph.engine.get(_lib.F_OBJ), o.obj, rtol=1e-6)
    np.testing.assert_allclose(ph.engine.get(_lib.F_BOUND), o.outer, rtol=1e-6)
    assert (ph.engine.get_i32(_lib.I_STATUS) == 0).all()


@pytest.mark.parametrize("case,S,layout", [("sslp", 4, "auto"), ("sslp", 4, "wave"), ("netdes", 3, "auto"),
                                           ("sslp", 4, "stream"), ("uc_small", 4, "stream")])
def test_prox_qp_block_kernel(case, S, layout):
    """layout "stream": the range-split multi-workgroup kernel (pdhg_stream.hip) with K > 1
    workgroups per scenario (few scenarios: K = 16), its cross-workgroup barriers and sums;
    (the bordered kernel: test_border_matches_block_kernel)."""
    pn, pc, pkw, on, oc, okw = CASES[case]
    ph = PH(_opts(pdhg_layout=layout), pn(S), pc, scenario_creator_kwargs=pkw)
    ph.PH_Prep()
    ph.Iter0()
    o = oph.OraclePH(_opts(), on(S), oc, okw)
    o.Iter0()
    for it in range(2):
        o.Compute_Xbar()
        o.Update_W()
        ph.engine.set(_lib.F_W, o.W.ravel())
        ph.engine.set(_lib.F_XBAR, o.xbar[0])
        ph.solve_loop()
        o.solve_loop()
        xg = ph.nonants()
        xo = np.array([o.nonants(k) for k in range(S)])
        np.testing.assert_allclose(xg, xo, rtol=1e-5, atol=1e-5 * max(1.0, np.abs(xo).max()))
        np.testing.assert_allclose(ph.engine.get(_lib.F_OBJ), o.obj, rtol=1e-6)
        assert (ph.engine.get_i32(_lib.I_STATUS) == 0).all()
    if layout == "stream":
        assert ph.engine.layout == layout and ph.engine.workgroups_per_scenario > 1


def test_netdes_delta_values(monkeypatch):
    """SURVEY 8(b) value forms on netdes (only the vubs' u_e vary, examples/netdes/netdes.py:39-80):
    the per-scenario [S*nnz] form and the sparse delta list load the same device data (same bits),
    with ONE scaling for all scenarios so the kernel streams per scenario only the piece-entry rows
    holding a u_e; PHG_DELTA=0 (per-scenario scaling and copies) reaches the same prox-QP solutions
    (1e-6) with a different preconditioner; the unit form (constant entries +-1 held in LDS as entry
    codes) returns the delta form's bits.  Both against the oracle's certified QPs (1e-5 / 1e-6)."""
    S = 40
    kw = {"num_scens": S}
    o = oph.OraclePH(_opts(), om.netdes_names(S)[:4], om.netdes, {"num_scens": 4})
    o.Iter0()
    o.Compute_Xbar()
    o.Update_W()
    res = {}
    for tag, form, env, unit in (("dense", 0, "1", "1"), ("delta", 2, "1", "1"), ("vs", 2, "1", "0"),
                                 ("off", 0, "0", "1")):
        monkeypatch.setenv("PHG_DELTA", env)
        monkeypatch.setenv("PHG_UNIT", unit)
        ph = PH(_opts(pdhg_vals_form=form), netdes.scenario_names_creator(S), netdes.scenario_creator,
                scenario_creator_kwargs=kw)
        ph.PH_Prep()
        assert ph.engine.layout == "block"
        vi = ph.engine.values_info()
        assert vi["varying"] == 1470, vi
        if env == "1":
            # two entry rows of 1024 per product: the x_e column pieces and the vub row pieces
            assert vi["delta"] and 0 < vi["per_scenario_vals"] <= 4 * 1024 and vi["shared_vals"] > 0, vi
            # netdes's constant entries are all +-1: the unit form (matrix in LDS) unless PHG_UNIT=0
            assert vi["unit"] == (unit == "1"), vi
        else:
            assert not vi["delta"] and vi["per_scenario_vals"] >= 2 * 5880, vi
        ph.Iter0()
        ob0 = ph.engine.get(_lib.F_OBJ).copy()
        W = np.zeros((S, ph.engine.N))
        W[:4] = o.W
        ph.engine.set(_lib.F_W, W.ravel())
        ph.engine.set(_lib.F_XBAR, o.xbar[0])
        ph.solve_loop()
        assert (ph.engine.get_i32(_lib.I_STATUS) == 0).all()
        res[tag] = (ob0, ph.engine.get(_lib.F_OBJ).copy(), ph.engine.get_i32(_lib.I_ITERS).copy(), ph.nonants())
    for a, b in zip(res["dense"], res["delta"]):
        np.testing.assert_array_equal(a, b)
    # the unit form adds / subtracts where the delta form fma's +-1: the same bits
    for a, b in zip(res["delta"], res["vs"]):
        np.testing.assert_array_equal(a, b)
    a, b = res["dense"], res["off"]
    np.testing.assert_allclose(a[0], b[0], rtol=1e-6)
    np.testing.assert_allclose(a[1], b[1], rtol=1e-6)
    np.testing.assert_allclose(a[3], b[3], atol=1e-5)
    # the first 4 scenarios' prox-QPs against the oracle
    o.solve_loop()
    xo = np.array([o.nonants(k) for k in range(4)])
    np.testing.assert_allclose(res["delta"][3][:4], xo, rtol=1e-5, atol=1e-5 * max(1.0, np.abs(xo).max()))
    np.testing.assert_allclose(res["delta"][1][:4], o.obj, rtol=1e-6)


def test_border_split_solves_match_uninterrupted(monkeypatch, capfd):
    """Split solves (pdhg_border.hip, BorderLayout::slice): with more scenarios than slots, a solve
    still running after slice x check_every PDHG iterations while the queue's first pass lasts is
    suspended at that check and re-queued; resuming restores its iterate, running sums, restart point
    and restart / step state and recomputes A x / A^T y with the same gathers, so Iter0 and three PH
    iterations give bit-identical objectives, bounds, iteration counts and nonants to
    uninterrupted solves.
    24 scenarios of a 24-unit x 12-period UC LP on 16 slots (PHG_STREAM_K=16); slice 1 suspends at
    the first check past 32 iterations, and the launch reports how many solves it split."""
    monkeypatch.setenv("PHG_STREAM_K", "16")
    monkeypatch.setenv("PHG_BORDER_STATS", "1")
    S = 24
    kw = {"num_gens": 24, "num_periods": 12, "num_scens": S}
    res = {}
    for sl in ("0", "1"):
        monkeypatch.setenv("PHG_BORDER_SLICE", sl)
        ph = PH(_opts(pdhg_layout="border", pdhg_check_every=32, pdhg_max_iter=20000), uc.scenario_names_creator(S),
                uc.scenario_creator, scenario_creator_kwargs=kw)
        ph.PH_Prep()
        assert ph.engine.layout == "border" and ph.engine.variant >= 600   # the register-resident kernel
        capfd.readouterr()
        ph.Iter0()
        r = [ph.engine.get(_lib.F_OBJ).copy(), ph.engine.get(_lib.F_BOUND).copy(),
             ph.engine.get_i32(_lib.I_ITERS).copy(), ph.nonants().copy()]
        for _ in range(3):   # (warm-started PH solves end near the first checks: a termination at the
            ph.Compute_Xbar()   # check that would suspend must not suspend)
            ph.Update_W()
            ph.solve_loop()
            r += [ph.engine.get(_lib.F_OBJ).copy(), ph.engine.get(_lib.F_BOUND).copy(),
                  ph.engine.get_i32(_lib.I_ITERS).copy(), ph.nonants().copy(), ph.engine.get_i32(_lib.I_STATUS).copy()]
        err = capfd.readouterr().err
        split = [int(ln.split()[4]) for ln in err.splitlines() if ln.startswith("PHG_BORDER_SPLIT")]
        res[sl] = (r, split)
    (ra, sa), (rb, sb) = res["0"], res["1"]
    assert sa == [] and len(sb) >= 2 and sb[0] > 0, (sa, sb)
    for a, b in zip(ra, rb):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("reg", ["1", "0"])
def test_border_matches_block_kernel(monkeypatch, reg):
    """reg "0" (PHG_BORDER_REG=0): the memory-resident bordered variant the planner falls back to
    when the register variant's LDS or per-thread budget is exceeded (its average
    iterate's linking-row A^T y read a running-sum array nothing wrote).
    The bordered block-diagonal kernel (pdhg_border.hip: 16 workgroups per scenario, one block
    per unit, the 24-nonzero demand / reserve rows as linking rows) runs the same arithmetic as the
    workgroup-per-scenario block kernel in a different order: on a 24-unit x 12-period UC LP and
    one prox-QP at the oracle's W / x-bar, both reach the same iteration counts and objectives (to
    rounding), and the objectives match HiGHS at 1e-6.  (This LP is hard for PDHG: one scenario
    stops at the 2e5-iteration cap with a 1e-9-level KKT error, in both kernels.)  Both with the
    per-scenario scaling the bordered kernel uses (PHG_DELTA=0: the derates vary a few entries, which
    would otherwise put the block kernel on the shared-scaling delta form)."""
    monkeypatch.setenv("PHG_DELTA", "0")
    monkeypatch.setenv("PHG_BLOCK_SEG", "0")   # (row segments sum the pieces in another order)
    monkeypatch.setenv("PHG_BORDER_REG", reg)
    kw = {"num_gens": 24, "num_periods": 12, "num_scens": 3}
    o = oph.OraclePH(_opts(), om.uc_names(3), om.uc, kw)
    o.Iter0()
    o.Compute_Xbar()
    o.Update_W()
    res = {}
    for layout in ("block", "border"):
        # the same check interval and artificial-restart fraction on both (the defaults are by
        # layout: phbase.check_every_default, beta_artificial_default)
        ph = PH(_opts(pdhg_layout=layout, pdhg_check_every=32, pdhg_beta_artificial=0.25), uc.scenario_names_creator(3),
                uc.scenario_creator, scenario_creator_kwargs=kw)
        ph.PH_Prep()
        assert ph.engine.layout == layout
        ph.Iter0()
        ob0 = ph.engine.get(_lib.F_OBJ).copy()
        ph.engine.set(_lib.F_W, o.W.ravel())
        ph.engine.set(_lib.F_XBAR, o.xbar[0])
        ph.solve_loop()
        res[layout] = (ob0, ph.engine.get(_lib.F_OBJ).copy(), ph.engine.get_i32(_lib.I_ITERS).copy(), ph.nonants())
        if layout == "border":
            assert ph.engine.workgroups_per_scenario > 1
            assert bool(ph.engine.border_reg) == (reg == "1")
    (a0, a1, ai, ax), (b0, b1, bi, bx) = res["block"], res["border"]
    np.testing.assert_array_equal(ai, bi)
    np.testing.assert_allclose(b0, a0, rtol=1e-11)
    np.testing.assert_allclose(b1, a1, rtol=1e-11)
    np.testing.assert_allclose(bx, ax, atol=1e-8)
    o.solve_loop()
    np.testing.assert_allclose(b1, o.obj, rtol=1e-6)


@pytest.mark.parametrize("S,layout", [(2, "auto"), (2, "stream"), (40, "auto")])
def test_uc_fullsize_stream_vs_oracle(S, layout):
    """The UC-shaped LP at full size (n = 20 400, m = 20 326, N = 4 080) through the AUTO layout
    (too large for a workgroup's LDS: a multi-workgroup kernel, K > 1 workgroups per scenario):
    the bordered block-diagonal kernel (pdhg_border.hip: one block per unit, the 96 demand /
    reserve rows linking them; what AUTO picks) and the range-split kernel (pdhg_stream.hip,
    layout "stream"); S = 40 puts several scenarios through each slot's queue.  At this size PDHG
    needs > 2e5 iterations for a 1e-9 relative KKT error, so the solve runs at pdhg_eps = 1e-6 (the
    accuracy PDLP-class solvers default to): Iter0 LP objectives and dual bounds against HiGHS at
    1e-5 relative (LP optima may be non-unique: objectives only; the oracle solves a sample of
    scenarios when S is large)."""
    so = {"pdhg_eps": 1e-6}
    ph = PH(_opts(iter0_solver_options=so, iterk_solver_options=so, pdhg_layout=layout), uc.scenario_names_creator(S),
            uc.scenario_creator, scenario_creator_kwargs={"num_scens": S})
    ph.PH_Prep()
    assert ph.engine.layout == ("border" if layout == "auto" else "stream") and ph.engine.workgroups_per_scenario > 1
    tb = ph.Iter0()
    if S > 4:
        pick = [0, 1, S // 2, S - 1]
        # (the generator's data depend on the scenario's name only; num_scens sets the probability)
        o = oph.OraclePH(_opts(), [om.uc_names(S)[k] for k in pick], om.uc, {"num_scens": len(pick)})
        o.Iter0()
        assert (ph.engine.get_i32(_lib.I_STATUS) == 0).all()
        np.testing.assert_allclose(ph.engine.get(_lib.F_OBJ)[pick], o.obj, rtol=1e-5)
        np.testing.assert_allclose(ph.engine.get(_lib.F_BOUND)[pick], o.outer, rtol=1e-5)
        return
    o = oph.OraclePH(_opts(), om.uc_names(S), om.uc, {"num_scens": S})
    otb = o.Iter0()
    assert (ph.engine.get_i32(_lib.I_STATUS) == 0).all()
    assert (ph.engine.get(_lib.F_KKT) <= 1e-6).all()
    assert abs(tb - otb) <= 1e-5 * abs(otb), (tb, otb)
    np.testing.assert_allclose(ph.engine.get(_lib.F_OBJ), o.obj, rtol=1e-5)
    np.testing.assert_allclose(ph.engine.get(_lib.F_BOUND), o.outer, rtol=1e-5)


def test_uc_fullsize_at_north_star_accuracy():
    """The north star asks for bounds within 1e-6 relative: the full-size UC LP (8 scenarios,
    bordered kernel) at pdhg_eps 1e-7 -- every Iter0 solve terminates inside a 1e6-iteration cap
    (two of the eight need more than 2e5), and its objective and its dual bound are within 1e-6 of
    HiGHS' optimum.  (Measured on 2 scenarios: 1.4e-7 and 6e-8; HiGHS' own feasibility tolerances
    are 1e-7, so the oracle is not exact below that.)"""
    so = {"pdhg_eps": 1e-7, "pdhg_max_iter": 1000000}
    S = 8
    ph = PH(_opts(iter0_solver_options=so, iterk_solver_options=so), uc.scenario_names_creator(S),
            uc.scenario_creator, scenario_creator_kwargs={"num_scens": S})
    ph.PH_Prep()
    assert ph.engine.layout == "border"
    ph.Iter0()
    o = oph.OraclePH(_opts(), om.uc_names(S), om.uc, {"num_scens": S})
    o.Iter0()
    assert (ph.engine.get_i32(_lib.I_STATUS) == 0).all(), ph.engine.get_i32(_lib.I_ITERS)
    np.testing.assert_allclose(ph.engine.get(_lib.F_OBJ), o.obj, rtol=1e-6)
    np.testing.assert_allclose(ph.engine.get(_lib.F_BOUND), o.outer, rtol=1e-6)


def test_block_register_pieces_same_bits(monkeypatch):
    """sslp's pieces fit the registers (row pieces <= 8, columns in <= 2 rows), so the block layout
    runs the block kernel with the matrix held in registers for the whole solve; PHG_BLOCK_STREAM=1 forces
    the form that re-reads values / indices every iteration.  Same products in the same order:
    Iter0 and one prox-QP solve give bit-identical objectives, iteration counts and nonants.  (Row
    segments off: the segment form sums a row's pieces pairwise, the streaming variants in order.)"""
    monkeypatch.setenv("PHG_BLOCK_SEG", "0")
    S = 8
    o = oph.OraclePH(_opts(), om.sslp_names(S), om.sslp, {})
    o.Iter0()
    o.Compute_Xbar()
    o.Update_W()
    res = []
    for stream in ("0", "1"):
        monkeypatch.setenv("PHG_BLOCK_STREAM", stream)
        ph = PH(_opts(pdhg_layout="block"), sslp.scenario_names_creator(S), sslp.scenario_creator)
        ph.PH_Prep()
        assert ph.engine.layout == "block"
        ph.Iter0()
        ob0 = ph.engine.get(_lib.F_OBJ).copy()
        ph.engine.set(_lib.F_W, o.W.ravel())
        ph.engine.set(_lib.F_XBAR, o.xbar[0])
        ph.solve_loop()
        res.append((ob0, ph.engine.get(_lib.F_OBJ).copy(), ph.engine.get_i32(_lib.I_ITERS).copy(), ph.nonants()))
    for a, b in zip(*res):
        np.testing.assert_array_equal(a, b)


def test_uc_fullsize_lagrangian_lp_vs_oracle():
    """The Lagrangian spoke's subproblem at full UC size (W on, prox off: lagrangian_bounder.py:21-44
    with the W of the first PH update, phbase.py:301-326) through the bordered kernel, against HiGHS'
    LP with the same W on two sampled scenarios: objectives at 1e-5 relative (pdhg_eps 1e-6, as the
    UC runs); each converged scenario's own dual objective within the solve's tolerance of the LP
    optimum on either side (measured r03: 1.5e-6 ABOVE it on one scenario -- eps (1 + |p| + |d|) at
    1e-6, as a CPU solver's bound at its tolerances); and with phg_opts.safe_bound = 2 (what the
    Lagrangian spoke uses at this eps: cylinders.safe_bound_mode) a weak-duality certificate of the
    dual iterate at or below the LP optimum and within 3e-5 of it."""
    S = 4
    so = {"pdhg_eps": 1e-6}
    ph = PH(_opts(iter0_solver_options=so, iterk_solver_options=so), uc.scenario_names_creator(S),
            uc.scenario_creator, scenario_creator_kwargs={"num_scens": S})
    ph.PH_Prep()
    assert ph.engine.layout == "border" and ph.engine.workgroups_per_scenario > 1
    ph.Iter0()
    ph.Compute_Xbar()
    ph.Update_W()
    W = ph.engine.get(_lib.F_W).reshape(S, ph.engine.N)
    assert np.abs(W).max() > 0
    ph.engine.solve(1, 0, eps=1e-6, max_iter=200000, warm_start=3, safe_bound=2)
    ph.engine.sync()
    obj, bnd = ph.engine.get(_lib.F_OBJ), ph.engine.get(_lib.F_BOUND)
    st = ph.engine.get_i32(_lib.I_STATUS)
    # the same solve's own dual objectives (status 0 keeps them with safe_bound = 1)
    ph.engine.solve(1, 0, eps=1e-6, max_iter=200000, warm_start=3, safe_bound=1)
    ph.engine.sync()
    dob, st1 = ph.engine.get(_lib.F_BOUND), ph.engine.get_i32(_lib.I_STATUS)
    pick = [0, S - 1]
    o = oph.OraclePH(_opts(), [om.uc_names(S)[k] for k in pick], om.uc, {"num_scens": len(pick)})
    o.W = W[pick].copy()
    o.W_on, o.prox_on = 1, 0
    o.solve_loop()
    for i, k in enumerate(pick):
        ref = o.obj[i]
        assert st[k] == 0, (k, st[k])
        assert abs(obj[k] - ref) <= 1e-5 * abs(ref), (k, obj[k], ref)
        # (measured r03: 1.2e-5 below -- the eps 1e-6 iterate's reduced costs charged against the box)
        assert bnd[k] <= ref + 1e-9 * abs(ref) and ref - bnd[k] <= 3e-5 * abs(ref), (k, bnd[k], ref)
        if st1[k] == 0:
            assert abs(dob[k] - ref) <= 4e-6 * abs(ref), (k, dob[k], ref)


def test_uc_fullsize_lagrangian_lp_at_north_star_accuracy():
    """The Lagrangian spoke's full-size UC subproblem (W on, prox off) at pdhg_eps 1e-7 on two
    scenarios: objectives within 1e-6 of HiGHS' LP with the same W, and the safe_bound = 2
    weak-duality certificate at or below the LP optimum (to HiGHS' own 1e-7 tolerances) and within
    3e-6 of it -- the north star's 1e-6 on the outer bound's ingredients."""
    S = 2
    so = {"pdhg_eps": 1e-7}
    ph = PH(_opts(iter0_solver_options=so, iterk_solver_options=so), uc.scenario_names_creator(S),
            uc.scenario_creator, scenario_creator_kwargs={"num_scens": S})
    ph.PH_Prep()
    assert ph.engine.layout == "border"
    ph.Iter0()
    ph.Compute_Xbar()
    ph.Update_W()
    W = ph.engine.get(_lib.F_W).reshape(S, ph.engine.N)
    ph.engine.solve(1, 0, eps=1e-7, max_iter=200000, warm_start=3, safe_bound=2)
    ph.engine.sync()
    obj, bnd, st = ph.engine.get(_lib.F_OBJ), ph.engine.get(_lib.F_BOUND), ph.engine.get_i32(_lib.I_STATUS)
    o = oph.OraclePH(_opts(), om.uc_names(S), om.uc, {"num_scens": S})
    o.W = W.copy()
    o.W_on, o.prox_on = 1, 0
    o.solve_loop()
    for k in range(S):
        ref = o.obj[k]
        assert st[k] == 0, (k, st[k])
        assert abs(obj[k] - ref) <= 1e-6 * abs(ref), (k, obj[k], ref)
        assert bnd[k] <= ref + 2e-7 * abs(ref) and ref - bnd[k] <= 3e-6 * abs(ref), (k, bnd[k], ref)


def test_wave_kernel_matches_block_kernel():
    """sslp (one matrix for every scenario, columns in <= 2 rows) on the wave layout (pdhg_wave.hip, on
    request only: slower than the block kernel on MI355X) -- one wavefront per scenario, the matrix
    once per workgroup in LDS, no workgroup barrier in the loop --
    which adds the same pieces in the same order as the workgroup kernel but reduces its KKT norms
    over a wave instead of a workgroup.  Iter0 and two prox-QP solves at the oracle's W / x-bar, both
    layouts: objectives and bounds agree to 1e-9 relative, nonants to 1e-7, every solve at status 0;
    and the prox-QP nonants against the oracle at 1e-5 (test_prox_qp_block_kernel[sslp-4-auto])."""
    S = 16
    o = oph.OraclePH(_opts(), om.sslp_names(S), om.sslp, {})
    o.Iter0()
    o.Compute_Xbar()
    o.Update_W()
    res = {}
    for layout in ("wave", "block"):
        # the same check interval and artificial-restart fraction on both (the defaults are by
        # layout: phbase.check_every_default, beta_artificial_default)
        ph = PH(_opts(pdhg_layout=layout, pdhg_check_every=32, pdhg_beta_artificial=0.15), sslp.scenario_names_creator(S),
                sslp.scenario_creator)
        ph.PH_Prep()
        assert ph.engine.layout == layout
        ph.Iter0()
        r = [ph.engine.get(_lib.F_OBJ).copy(), ph.engine.get(_lib.F_BOUND).copy()]
        assert (ph.engine.get_i32(_lib.I_STATUS) == 0).all()
        for it in range(2):
            ph.engine.set(_lib.F_W, o.W.ravel() * (it + 1))
            ph.engine.set(_lib.F_XBAR, o.xbar[0])
            ph.solve_loop()
            assert (ph.engine.get_i32(_lib.I_STATUS) == 0).all()
            r += [ph.engine.get(_lib.F_OBJ).copy(), ph.engine.get(_lib.F_BOUND).copy(), ph.nonants().copy(),
                  ph.engine.get_i32(_lib.I_ITERS).copy()]
        res[layout] = r
    a, b = res["wave"], res["block"]
    for u in (0, 1, 2, 3, 6, 7):
        np.testing.assert_allclose(a[u], b[u], rtol=1e-9, atol=1e-9)
    for u in (4, 8):
        np.testing.assert_allclose(a[u], b[u], atol=1e-7)
    print("PDHG iterations wave / block:", a[5].sum() + a[9].sum(), b[5].sum() + b[9].sum())
