"""bench.py's rank evidence on CPU: ``comm.rank_report`` gathers every rank's
record over two gloo ranks and reports the exchange path with the collective's own rank count; the
library group's count comes from RCCL (``phg_group_size`` -> ``ncclCommCount``), and a group whose
RCCL rank disagrees with the host rank is refused."""
import os
import socket
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _pkg  # noqa: E402

_pkg.load()
from mpisppy_amd import _lib, comm  # noqa: E402
from mpisppy_amd.comm import PhgGroupComm, SingleComm, rank_report  # noqa: E402

torch = pytest.importorskip("torch")


def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    p = so.getsockname()[1]
    so.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import _pkg as pk
    pk.load()
    from mpisppy_amd.comm import TorchComm, rank_report as rr
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, rr(TorchComm())))
    finally:
        dist.destroy_process_group()


def test_two_gloo_ranks_report_each_other():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r, rep in got.items():
        assert rep["world_size"] == 2
        assert [x["rank"] for x in rep["ranks"]] == [0, 1]
        assert rep["exchange_path"].startswith("torch.distributed gloo")
        assert rep["collective_ranks"] is None          # gloo: no RCCL communicator
    assert got[0]["ranks"] == got[1]["ranks"]          # every rank holds the same gathered view


def test_single_rank_report():
    rep = rank_report(SingleComm())
    assert rep["world_size"] == 1 and rep["collective_ranks"] is None and len(rep["ranks"]) == 1


class _RcclGroup:
    """A stand-in for _lib.PhgGroup whose size() is what RCCL would report."""
    rccl = (8, 0)

    def __init__(self, nranks, rank, uid, device):
        self.args = (nranks, rank, uid, device)

    @staticmethod
    def unique_id():
        return bytes(128)

    def size(self):
        return self.rccl

    def close(self):
        pass


def test_library_group_reports_rccl_count(monkeypatch):
    monkeypatch.setattr(comm, "_device_count", lambda: 8)
    monkeypatch.setattr(_lib, "PhgGroup", _RcclGroup)
    c = PhgGroupComm(SingleComm(), device=0)
    rep = rank_report(c)
    assert rep["collective_ranks"] == 8 and rep["exchange_path"].startswith("libphg RCCL group")
    _RcclGroup.rccl = (8, 3)                            # RCCL disagrees with the host's rank 0
    with pytest.raises(RuntimeError):
        rank_report(c)
    _RcclGroup.rccl = (8, 0)
