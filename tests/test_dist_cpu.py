"""N>1 host path on CPU: two gloo ranks run the product's PHBase orchestration (rank slicing,
BatchArrays index maps, packed node-sum / convergence all-reduces, rank-summed Ebound) with the
device kernels replaced by a numpy stand-in (test infrastructure), and must reproduce the
single-process oracle run with the same virtual rank slicing (n_proc = 2)."""
import math
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class NumpyEngine:
    """Mirror of engine.Engine's interface computing on the host (tests only)."""

    def __init__(self, batch, exchange):
        from oracle import highs
        self.highs = highs
        self.batch = batch
        self.S, self.N, self.N_tot, self.P = batch.S, batch.N, batch.N_tot, batch.virt_nproc
        self.exchange = exchange
        self.W = np.zeros((self.S, self.N))
        self.rho = np.zeros((self.S, self.N))
        self.xbar = np.zeros(self.N_tot)
        self.xN = np.zeros((self.S, self.N))
        self.bound = np.zeros(self.S)
        self.obj = np.zeros(self.S)
        self.X = None
        b = batch
        self.xidx = np.zeros((self.S, self.N), dtype=np.int64)
        for s in range(self.S):
            for k in range(self.N):
                self.xidx[s, k] = b.node_off[b.scen_node[s, b.nonant_level[k]]] + b.nonant_pos[k]

    def set(self, field, v):
        from mpisppy_amd import _lib
        if field == _lib.F_RHO:
            self.rho[:] = v
        elif field == _lib.F_W:
            self.W[:] = np.asarray(v).reshape(self.W.shape)

    def get(self, field):
        from mpisppy_amd import _lib
        return {_lib.F_W: self.W.ravel(), _lib.F_XBAR: self.xbar, _lib.F_XN: self.xN.ravel(),
                _lib.F_BOUND: self.bound, _lib.F_OBJ: self.obj}[field].copy()

    def get_i32(self, field):
        return np.zeros(self.S, np.int32)

    def sync(self):
        pass

    def solve(self, w_on, prox_on, skip_below=0.0, **kw):
        if skip_below > 0 and getattr(self, "_gate", None) is not None and self._gate < skip_below:
            return                    # predicated solve (phg_opts.skip_if_conv_below)
        b = self.batch
        X = []
        for s in range(self.S):
            c = b.c[s].copy()
            cols = b.nonant_col
            q = None
            off = b.off[s]
            if w_on:
                c[cols] += self.W[s]
            if prox_on:
                xb = self.xbar[self.xidx[s]]
                c[cols] -= self.rho[s] * xb
                q = np.zeros_like(c)
                q[cols] = self.rho[s]
                off += float(np.sum(self.rho[s] / 2 * xb * xb))
            r = self.highs.solve(c, b.rowptr, b.colidx, b.vals[s], b.rl[s], b.ru[s], b.cl[s], b.cu[s],
                                 qdiag=q, offset=off)
            assert r.ok
            X.append(r.x)
            self.xN[s] = r.x[cols]
            self.obj[s] = self.bound[s] = r.obj
        self.X = np.array(X)

    def node_sums(self):
        b = self.batch
        ns = np.zeros(2 * self.N_tot)
        for s in range(self.S):
            for k in range(self.N):
                p = b.prob_coeff[s, b.nonant_level[k]]
                j = self.xidx[s, k]
                ns[j] += p * self.xN[s, k]
                ns[self.N_tot + j] += p * self.xN[s, k] ** 2
        self.exchange[0].copy_(torch.from_numpy(ns))

    def apply_xbar(self):
        b = self.batch
        ns = self.exchange[0].numpy()
        self.xbar = ns[:self.N_tot].copy()
        cp = np.zeros(2 * self.P + 2)
        avg = b.S_global / self.P
        for s in range(self.S):
            gs = b.scen_global0 + s
            v = 0 if self.P == 1 else max(i for i in range(self.P) if gs >= int(i * avg))
            d = self.xN[s] - self.xbar[self.xidx[s]]
            self.W[s] += self.rho[s] * d
            cp[2 * v] += np.abs(d).sum()
            cp[2 * v + 1] += self.N
        self.exchange[1].copy_(torch.from_numpy(cp))

    def conv_finish(self):
        cp = self.exchange[1].numpy()
        return sum(cp[2 * v] / cp[2 * v + 1] for v in range(self.P) if cp[2 * v + 1] > 0) / self.P

    def conv_start(self):             # phg_conv_start: conv into the device gate
        self._gate = self.conv_finish()

    def conv_wait(self):
        return self._gate

    def eval_objective(self, w_on, prox_on):
        return self.obj.copy()

    def solve_summary(self):
        cp = self.exchange[1].numpy()
        return int(cp[2 * self.P]), int(cp[2 * self.P + 1])


def _worker(rank, world, port, case, q):
    import sys
    sys.path.insert(0, ROOT)
    import _pkg
    _pkg.load()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from mpisppy_amd.comm import TorchComm
        from mpisppy_amd.engine import BatchArrays
        from mpisppy_amd.ph import PH
        from mpisppy_amd.examples import farmer, hydro
        from mpisppy_amd.spbase import create_nodenames_from_branching_factors

        class CpuPH(PH):
            def _create_solvers(self):
                if self.engine is not None:
                    return
                models = [self.local_scenarios[n] for n in self.local_scenario_names]
                batch = BatchArrays(models, self.all_nodenames, [m._mpisppy_probability for m in models],
                                    self.scen_global0, len(self.all_scenario_names), self._virt_nproc())
                ex = (torch.zeros(2 * batch.N_tot, dtype=torch.float64),
                      torch.zeros(2 * batch.virt_nproc + 2, dtype=torch.float64))
                self.engine = NumpyEngine(batch, ex)
                self.engine.set(0 + 4, float(self.options["defaultPHrho"]))

        opts = {"solver_name": "phg", "PHIterLimit": 4, "defaultPHrho": 1.0, "convthresh": 1e-10,
                "verbose": False, "display_progress": False}
        if case == "farmer":
            ph = CpuPH(opts, farmer.scenario_names_creator(5), farmer.scenario_creator, mpicomm=TorchComm(),
                       scenario_creator_kwargs={"crops_multiplier": 1, "num_scens": 5})
        else:
            bf = [3, 3]
            ph = CpuPH(opts, hydro.scenario_names_creator(9), hydro.scenario_creator, mpicomm=TorchComm(),
                       all_nodenames=create_nodenames_from_branching_factors(bf),
                       scenario_creator_kwargs={"branching_factors": bf})
        conv, eobj, tb = ph.ph_main()
        q.put((rank, ph.conv_history, tb, eobj, ph.engine.xbar.tolist(), ph.engine.W.tolist(),
               ph.local_scenario_names))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("case", ["farmer", "hydro"])
def test_two_rank_gloo_matches_oracle(case):
    from oracle import models as om
    from oracle import ph as oph
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r = q.get(timeout=240)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    opts = {"defaultPHrho": 1.0, "PHIterLimit": 4, "convthresh": 1e-10}
    if case == "farmer":
        o = oph.OraclePH(opts, om.farmer_names(5), om.farmer, dict(crops_multiplier=1, num_scens=5), n_proc=2)
    else:
        o = oph.OraclePH(opts, om.hydro_names(9), om.hydro, {}, n_proc=2)
    conv, eobj, tb = o.ph_main()
    # rank slicing (sputils.py:819-826)
    assert res[0][6] + res[1][6] == o.names
    assert len(res[0][6]) == len(o.slices[0])
    for r in (0, 1):
        np.testing.assert_allclose(res[r][1], o.history, rtol=1e-9, atol=1e-12)
        assert math.isclose(res[r][2], tb, rel_tol=1e-12)
        assert math.isclose(res[r][3], eobj, rel_tol=1e-9)
    Wg = np.array(res[0][5] + res[1][5])
    np.testing.assert_allclose(Wg, o.W, atol=1e-9)
