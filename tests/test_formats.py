"""CPU tests of the on-disk / wire formats: W / xbar CSV (``wxbarutils.py``),
first-stage and tree solution writers (``sputils.py:53-84``), hub <-> spoke flat buffers, and the
extension hook fan-out.  The device arrays are replaced by a host stand-in with the engine's
field layout; the GPU round trip through the real engine is in ``test_gpu_wxbar.py``.

Pinned by the reference's own fixtures: ``tests/golden/ref_w_file.csv`` / ``ref_xbar_file.csv``
(``mpisppy/tests/examples/w_test_data``) must parse, pass the dual-feasibility check with farmer's
probabilities, and be re-emitted byte for byte by the writers.
"""
import csv
import os

import numpy as np
import pytest

from mpisppy_amd import _lib
from mpisppy_amd.engine import BatchArrays
from mpisppy_amd.examples import farmer
from mpisppy_amd.extensions.extension import Extension, MultiExtension
from mpisppy_amd.spbase import SPBase
from mpisppy_amd.utils import sputils, wxbarutils

GOLD = os.path.join(os.path.dirname(__file__), "golden")


class _HostEngine:
    """Host arrays laid out like the engine's fields (W: S x N, xbar / xsqbar: per tree node)."""

    def __init__(self, batch):
        self.batch, self.S, self.N = batch, batch.S, batch.N
        self.f = {_lib.F_W: np.zeros(batch.S * batch.N), _lib.F_XBAR: np.zeros(batch.N_tot),
                  _lib.F_XSQBAR: np.zeros(batch.N_tot), _lib.F_XN: np.zeros(batch.S * batch.N)}

    def get(self, field):
        return self.f[field].copy()

    def set(self, field, v):
        self.f[field][:] = v


class _HostPH(SPBase):
    def __init__(self, S=3):
        super().__init__({"verbose": False}, farmer.scenario_names_creator(S), farmer.scenario_creator,
                         scenario_creator_kwargs={"num_scens": S})
        models = list(self.local_scenarios.values())
        batch = BatchArrays(models, self.all_nodenames, [m._mpisppy_probability for m in models], 0, S, 1)
        self.engine = _HostEngine(batch)
        self._PHIter = 0
        self.reenabled = []

    def Ws(self):
        return self.engine.get(_lib.F_W).reshape(self.engine.S, self.engine.N)

    def xbars(self):
        return self.engine.get(_lib.F_XBAR)

    def _reenable_W(self):
        self.reenabled.append("W")

    def _reenable_prox(self):
        self.reenabled.append("prox")


def test_parse_golden_w_and_check_dual_feasibility():
    ph = _HostPH()
    wd = wxbarutils._parse_W_csv(os.path.join(GOLD, "ref_w_file.csv"), ph.local_scenario_names,
                                 ph.all_scenario_names, 0)
    assert sorted(wd) == ["scen0", "scen1", "scen2"]
    assert wd["scen0"]["DevotedAcreage[SUGAR_BEETS0]"] == 70.84705093609978
    assert wd["scen1"]["DevotedAcreage[CORN0]"] == -41.104251445950844
    wxbarutils._check_W(wd, ph, 0)          # sum_s p_s w_s = 0 within 1e-7


def test_set_W_from_golden_file_fills_engine_layout():
    ph = _HostPH()
    wxbarutils.set_W_from_file(os.path.join(GOLD, "ref_w_file.csv"), ph, 0)
    W = ph.Ws()
    names = wxbarutils._nonant_names(ph.local_scenarios["scen0"])
    assert W[0, names.index("DevotedAcreage[SUGAR_BEETS0]")] == 70.84705093609978
    assert W[1, names.index("DevotedAcreage[CORN0]")] == -41.104251445950844
    np.testing.assert_allclose((W / 3).sum(0), 0.0, atol=1e-7)


def test_write_W_reproduces_golden_rows(tmp_path):
    ph = _HostPH()
    wxbarutils.set_W_from_file(os.path.join(GOLD, "ref_w_file.csv"), ph, 0)
    out = tmp_path / "w.csv"
    wxbarutils.write_W_to_file(ph, str(out))
    # the first 9 rows of the fixture are one write of the 3 scenarios; values round-trip exactly
    gold = {tuple(r[:2]): r[2] for r in csv.reader(open(os.path.join(GOLD, "ref_w_file.csv")))}
    rows = list(csv.reader(open(out)))
    assert len(rows) == 9
    for s, v, w in rows:
        assert float(w) == float(gold[(s, v)])
    # append semantics
    wxbarutils.write_W_to_file(ph, str(out))
    assert len(open(out).read().splitlines()) == 18


def test_separate_W_files_round_trip(tmp_path):
    ph = _HostPH()
    rng = np.random.default_rng(3)
    W = rng.normal(size=(3, ph.engine.N))
    W -= W.mean(0)
    ph.engine.set(_lib.F_W, W.ravel())
    wxbarutils.write_W_to_file(ph, str(tmp_path), sep_files=True)
    assert sorted(os.listdir(tmp_path)) == [f"scen{k}_weights.csv" for k in range(3)]
    ph2 = _HostPH()
    wxbarutils.set_W_from_file(str(tmp_path), ph2, 0, sep_files=True)
    assert np.array_equal(ph2.Ws(), W)


def test_check_W_errors(tmp_path):
    ph = _HostPH()
    bad = tmp_path / "bad.csv"
    bad.write_text("# comment\n" + "".join(f"scen{k},DevotedAcreage[{c}0],1.0\n"
                                            for k in range(3) for c in ("CORN", "SUGAR_BEETS", "WHEAT")))
    with pytest.raises(RuntimeError, match="dual feasibility"):
        wxbarutils.set_W_from_file(str(bad), ph, 0)
    miss = tmp_path / "miss.csv"
    miss.write_text("".join(f"scen{k},DevotedAcreage[CORN0],0.0\n" for k in range(3)))
    with pytest.raises(RuntimeError, match="missing"):
        wxbarutils.set_W_from_file(str(miss), ph, 0)
    part = tmp_path / "part.csv"
    part.write_text("scen0,DevotedAcreage[CORN0],0.0\nscen9,X,1\n")
    with pytest.raises(RuntimeError, match="could not find"):
        wxbarutils.set_W_from_file(str(part), ph, 0)
    # disable_check skips the test and leaves unspecified entries alone
    wxbarutils.set_W_from_file(str(bad), ph, 0, disable_check=True)
    assert np.all(ph.Ws() == 1.0)


def test_xbar_write_matches_golden_and_sets_xsqbar(tmp_path):
    ph = _HostPH()
    wxbarutils.set_xbar_from_file(os.path.join(GOLD, "ref_xbar_file.csv"), ph)
    xb = ph.xbars()
    names = wxbarutils._nonant_names(ph.local_scenarios["scen0"])
    assert xb[names.index("DevotedAcreage[SUGAR_BEETS0]")] == 274.2239371483933
    assert np.array_equal(ph.engine.get(_lib.F_XSQBAR), xb * xb)
    out = tmp_path / "x.csv"
    wxbarutils.write_xbar_to_file(ph, str(out))
    gold = {r[0]: r[1] for r in csv.reader(open(os.path.join(GOLD, "ref_xbar_file.csv")))}
    rows = list(csv.reader(open(out)))
    assert len(rows) == 3 and all(v == gold[k] for k, v in rows)
    npy = tmp_path / "root.txt"
    wxbarutils.ROOT_xbar_npy_serializer(ph, str(npy))
    assert np.array_equal(np.loadtxt(npy), xb[:3])
    with pytest.raises(RuntimeError, match="required variable"):
        bad = tmp_path / "bad.csv"
        bad.write_text("DevotedAcreage[CORN0],1.0\n")
        wxbarutils.set_xbar_from_file(str(bad), ph)


def test_wxbar_extensions_hook_points(tmp_path):
    from mpisppy_amd.utils.wxbarreader import WXBarReader
    from mpisppy_amd.utils.wxbarwriter import WXBarWriter
    ph = _HostPH()
    ph.options = {"init_W_fname": os.path.join(GOLD, "ref_w_file.csv"),
                  "init_Xbar_fname": os.path.join(GOLD, "ref_xbar_file.csv")}
    r = WXBarReader(ph)
    ph._PHIter = 2
    r.miditer()                                 # only iteration 1 loads
    assert np.all(ph.Ws() == 0)
    ph._PHIter = 1
    r.miditer()
    assert ph.reenabled == ["W", "prox"] and ph.Ws()[0, 1] == 70.84705093609978
    ph.options = {"W_fname": str(tmp_path / "wd"), "separate_W_files": True,
                  "Xbar_fname": str(tmp_path / "x.csv")}
    w = WXBarWriter(ph)                         # creates the directory
    assert os.path.isdir(tmp_path / "wd")
    w.post_everything()
    assert len(os.listdir(tmp_path / "wd")) == 3 and (tmp_path / "x.csv").exists()
    ph.options = {"init_W_fname": str(tmp_path / "nope.csv")}
    with pytest.raises(SystemExit):
        WXBarReader(ph)


def test_solution_writers(tmp_path):
    m = farmer.scenario_creator("scen0", num_scens=3)
    m._solution = np.arange(m.n, dtype=float) + 0.5
    f = tmp_path / "fs.csv"
    sputils.first_stage_nonant_writer(str(f), m, False)
    root = m._mpisppy_node_list[0].nonant_vardata_list
    assert f.read_text().splitlines() == [f"{v.name},{m._solution[v.col]}" for v in root]
    sputils.first_stage_nonant_npy_serializer(str(tmp_path / "fs.npy"), m, False)
    assert np.array_equal(np.load(tmp_path / "fs.npy"), [m._solution[v.col] for v in root])
    sputils.scenario_tree_solution_writer(str(tmp_path), "scen0", m, False)
    rows = (tmp_path / "scen0.csv").read_text().splitlines()
    assert len(rows) == m.n
    blocks = [r.split(",")[0].split("[")[0] for r in rows]
    assert blocks == sorted(blocks)                 # components in name order


def test_flat_buffers():
    class Hub:
        BestOuterBound, BestInnerBound = -110.0, -100.0

        class opt:
            class engine:
                @staticmethod
                def get(field):
                    return np.arange(6.0)
    buf = sputils.hub_send_buffer(Hub, "W", write_id=4)
    assert list(buf) == [0, 1, 2, 3, 4, 5, -110.0, -100.0, 4]
    b = sputils.spoke_send_buffer(-105.5, 7)
    assert sputils.read_spoke_buffer(b, 6) == (-105.5, 7, True)
    assert sputils.read_spoke_buffer(b, 7)[2] is False


def test_multi_extension_fans_out_every_hook():
    calls = []

    def mk(tag):
        class E(Extension):
            def miditer(self):
                calls.append((tag, "miditer"))

            def post_everything(self):
                calls.append((tag, "post_everything"))

            def post_solve(self, sp, res):
                return res + [tag]
        E.__name__ = f"E{tag}"
        return E
    me = MultiExtension(object(), [mk(1), mk(2)])
    me.miditer()
    me.post_everything()
    me.enditer()
    assert calls == [(1, "miditer"), (2, "miditer"), (1, "post_everything"), (2, "post_everything")]
    assert me.post_solve(None, []) == [1, 2]
