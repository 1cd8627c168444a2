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
    """Mirror of engine.Engine's interface computing on the host (tests only): the packed exchange
    buffer [2 N_tot node sums | 2P+2 partials | flag] and the double-buffered solve state of
    include/phg.h (phg_ph_head / phg_solve_undo) included."""

    def __init__(self, batch, exchange):
        from oracle import highs
        self.highs = highs
        self.batch = batch
        self.S, self.N, self.N_tot, self.P = batch.S, batch.N, batch.N_tot, batch.virt_nproc
        self.exchange = exchange
        self.exchange_len = 2 * self.N_tot + 2 * self.P + 3
        assert exchange.numel() == self.exchange_len
        self.W = np.zeros((self.S, self.N))
        self.rho = np.zeros((self.S, self.N))
        self.xbar = np.zeros(self.N_tot)
        zero = (np.zeros((self.S, self.N)), np.zeros(self.S), np.zeros(self.S), None)
        self.front, self.back = zero, tuple(v.copy() if v is not None else None for v in zero)
        self._gate = None
        b = batch
        self.xidx = np.zeros((self.S, self.N), dtype=np.int64)
        for s in range(self.S):
            for k in range(self.N):
                self.xidx[s, k] = b.node_off[b.scen_node[s, b.nonant_level[k]]] + b.nonant_pos[k]

    @property
    def xN(self):
        return self.front[0]

    @property
    def nodesum_view(self):
        return self.exchange[: 2 * self.N_tot]

    @property
    def convpart_view(self):
        return self.exchange[2 * self.N_tot:]

    def fold_partials(self):
        pass                       # the stand-in's updates are never folded

    def set(self, field, v):
        from mpisppy_amd import _lib
        if field == _lib.F_RHO:
            self.rho[:] = v
        elif field == _lib.F_W:
            self.W[:] = np.asarray(v).reshape(self.W.shape)

    def get(self, field):
        from mpisppy_amd import _lib
        return {_lib.F_W: self.W.ravel(), _lib.F_XBAR: self.xbar, _lib.F_XN: self.front[0].ravel(),
                _lib.F_BOUND: self.front[2], _lib.F_OBJ: self.front[1]}[field].copy()

    def get_i32(self, field):
        return np.zeros(self.S, np.int32)

    def sync(self):
        pass

    def solve(self, w_on, prox_on, skip_below=0.0, **kw):
        gated = skip_below > 0 and self._gate is not None and self._gate < skip_below
        if not gated:                 # a gated solve (phg_opts.skip_if_conv_below) writes nothing
            b = self.batch
            X, xN, obj = [], np.zeros((self.S, self.N)), np.zeros(self.S)
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
                xN[s] = r.x[cols]
                obj[s] = r.obj
            self.back = (xN, obj, obj.copy(), np.array(X))
        self.front, self.back = self.back, self.front

    def solve_undo(self):
        self.front, self.back = self.back, self.front

    def node_sums(self):
        b = self.batch
        ns = np.zeros(2 * self.N_tot)
        for s in range(self.S):
            for k in range(self.N):
                p = b.prob_coeff[s, b.nonant_level[k]]
                j = self.xidx[s, k]
                ns[j] += p * self.xN[s, k]
                ns[self.N_tot + j] += p * self.xN[s, k] ** 2
        self.nodesum_view.copy_(torch.from_numpy(ns))

    def apply_xbar(self):
        b = self.batch
        ns = self.nodesum_view.numpy()
        self.xbar = ns[:self.N_tot].copy()
        cp = np.zeros(2 * self.P + 3)
        avg = b.S_global / self.P
        for s in range(self.S):
            gs = b.scen_global0 + s
            v = 0 if self.P == 1 else max(i for i in range(self.P) if gs >= int(i * avg))
            d = self.xN[s] - self.xbar[self.xidx[s]]
            self.W[s] += self.rho[s] * d
            cp[2 * v] += np.abs(d).sum()
            cp[2 * v + 1] += self.N
        cp[2 * self.P + 2] = 1.0
        self.convpart_view.copy_(torch.from_numpy(cp))

    def _conv(self):
        cp = self.convpart_view.numpy()
        if cp[2 * self.P + 2] <= 0:
            return math.inf
        return sum(cp[2 * v] / cp[2 * v + 1] for v in range(self.P) if cp[2 * v + 1] > 0) / self.P

    def ph_head(self, convthresh, first):     # phg_ph_head
        self._gate = math.inf if first else self._conv()
        if self._gate < convthresh:
            return
        self.apply_xbar()

    def conv_finish(self):
        self._gate = self._conv()
        return self._gate

    def conv_start(self):             # phg_conv_start: conv into the device gate
        self.conv_finish()

    def conv_wait(self):
        return self._gate

    def eval_objective(self, w_on, prox_on):
        """pyo.value(objfct) with the CURRENT W / xbar (phg_eval_objective)."""
        b = self.batch
        X, xN = self.front[3], self.front[0]
        out = np.zeros(self.S)
        for s in range(self.S):
            f = float(b.c[s] @ X[s]) + b.off[s]
            if w_on:
                f += float(self.W[s] @ xN[s])
            if prox_on:
                xb = self.xbar[self.xidx[s]]
                f += float(np.sum(self.rho[s] / 2 * (xN[s] ** 2 - 2 * xb * xN[s] + xb ** 2)))
            out[s] = b.sense * f if b.sense != 1 else f
        return out

    def solve_summary(self):
        cp = self.convpart_view.numpy()
        return int(cp[2 * self.P]), int(cp[2 * self.P + 1])


def _worker(rank, world, port, case, pipeline, thr, iters, q):
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
                ex = torch.zeros(2 * batch.N_tot + 2 * batch.virt_nproc + 3, dtype=torch.float64)
                self.engine = NumpyEngine(batch, ex)
                self.engine.set(0 + 4, float(self.options["defaultPHrho"]))

        opts = {"solver_name": "phg", "PHIterLimit": iters, "defaultPHrho": 1.0, "convthresh": thr,
                "verbose": False, "display_progress": False, "pdhg_pipeline": pipeline}
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
               ph.local_scenario_names, ph._PHIter, ph.engine.xN.tolist()))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("case,pipeline,stop", [("farmer", True, None), ("hydro", True, None),
                                                ("farmer", False, None), ("farmer", True, 3),
                                                ("farmer", False, 3)])
def test_two_rank_gloo_matches_oracle(case, pipeline, stop):
    """pipeline=True: the pipelined iteration (one packed all-reduce per PH iteration, solve
    speculative by one); False: the statement-by-statement loop (two all-reduces).  stop=k: the
    convergence threshold is set so that the reference breaks at iteration k (before its solve):
    the pipelined run must end in the same state (iteration count, W, xbar, nonants = the solve of
    iteration k-1), i.e. its speculative solve is undone."""
    from oracle import models as om
    from oracle import ph as oph
    iters = 4 if stop is None else 8
    opts = {"defaultPHrho": 1.0, "PHIterLimit": iters, "convthresh": 1e-10}
    if case == "farmer":
        mk = lambda o: oph.OraclePH(o, om.farmer_names(5), om.farmer, dict(crops_multiplier=1, num_scens=5), n_proc=2)
    else:
        mk = lambda o: oph.OraclePH(o, om.hydro_names(9), om.hydro, {}, n_proc=2)
    thr = 1e-10
    if stop is not None:
        probe = mk(dict(opts))
        probe.ph_main()
        h = probe.history
        assert h[stop - 1] < min(h[:stop - 1])        # a threshold between them stops at `stop`
        thr = 0.5 * (h[stop - 1] + min(h[:stop - 1]))
        opts["convthresh"] = thr
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, case, pipeline, thr, iters, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        r = q.get(timeout=120)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    o = mk(opts)
    conv, eobj, tb = o.ph_main()
    # rank slicing (sputils.py:819-826)
    assert res[0][6] + res[1][6] == o.names
    assert len(res[0][6]) == len(o.slices[0])
    for r in (0, 1):
        np.testing.assert_allclose(res[r][1], o.history, rtol=1e-9, atol=1e-12)
        assert math.isclose(res[r][2], tb, rel_tol=1e-12)
        assert math.isclose(res[r][3], eobj, rel_tol=1e-9)
        assert res[r][7] == o._PHIter == (stop if stop is not None else iters)
    Wg = np.array(res[0][5] + res[1][5])
    np.testing.assert_allclose(Wg, o.W, atol=1e-9)
    Xg = np.array(res[0][8] + res[1][8])
    np.testing.assert_allclose(Xg, np.array([o.nonants(k) for k in range(o.S)]), atol=1e-7)
