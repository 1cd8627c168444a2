"""comm.PhgGroupComm routing (host side, no GPU): device tensors go to the library's RCCL group
(phg_group_allreduce on the attached engine's handle), everything else to the host communicator;
the 128-byte group id is made by rank 0 and broadcast by the host communicator."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _pkg  # noqa: E402  (spawned ranks import this module without the conftest)

_pkg.load()
from mpisppy_amd import _lib, comm  # noqa: E402
from mpisppy_amd.comm import PhgGroupComm, SingleComm


@pytest.fixture(autouse=True)
def _devices(monkeypatch):
    """No GPU here: pretend 8 visible devices (the routing is what is tested)."""
    monkeypatch.setattr(comm, "_device_count", lambda: 8)


class _FakeGroup:
    made = []

    def __init__(self, nranks, rank, uid, device):
        self.args = (nranks, rank, uid, device)
        self.calls = []
        _FakeGroup.made.append(self)

    @staticmethod
    def unique_id():
        return bytes(range(128))

    def allreduce(self, handle, ptr, count):
        self.calls.append((handle, ptr, count))

    def close(self):
        self.calls.append("closed")


class _DevTensor:
    is_cuda = True

    def data_ptr(self):
        return 0x1000

    def numel(self):
        return 65


class _Host(SingleComm):
    def __init__(self):
        self.bcast = []
        self.summed = []

    def bcast_object(self, obj, root=0):
        self.bcast.append((obj, root))
        return obj

    def allreduce_sum_(self, t):
        self.summed.append(t)
        return t


class _Engine:
    h = "handle"


def test_routing(monkeypatch):
    monkeypatch.setattr(_lib, "PhgGroup", _FakeGroup)
    host = _Host()
    c = PhgGroupComm(host, device=3)
    g = _FakeGroup.made[-1]
    assert g.args == (1, 0, bytes(range(128)), 3) and host.bcast == [(bytes(range(128)), 0)]
    assert c.Get_rank() == 0 and c.Get_size() == 1
    with pytest.raises(RuntimeError):
        c.allreduce_sum_(_DevTensor())          # no engine attached yet
    c.attach(_Engine())
    t = _DevTensor()
    assert c.allreduce_sum_(t) is t and g.calls == [("handle", 0x1000, 65)]
    a = np.ones(3)
    c.allreduce_sum_(a)                          # host data: the host communicator
    assert host.summed == [a]
    assert c.allreduce_array([1.0, 2.0]).tolist() == [1.0, 2.0]   # delegated (SingleComm)
    c.close()
    assert g.calls[-1] == "closed"


class _Host2(_Host):
    """Rank ``rank`` of 2 whose peer reports ``peer_ok`` for the group creation."""

    def __init__(self, rank, peer_ok):
        super().__init__()
        self.rank_, self.peer_ok = rank, peer_ok

    def Get_rank(self):
        return self.rank_

    def Get_size(self):
        return 2

    def allreduce_scalar(self, v):
        return float(v) + (1.0 if self.peer_ok else 0.0)

    def bcast_object(self, obj, root=0):     # rank 0's id reaches rank 1
        return super().bcast_object(obj if self.rank_ == 0 else bytes(range(128)), root)


class _FailingGroup(_FakeGroup):
    def __init__(self, *a):
        raise _lib.PhgError("ncclCommInitRank: unhandled system error")


@pytest.mark.parametrize("rank", [0, 1])
def test_group_or_host_agreement(monkeypatch, rank):
    """Every rank ends on the same exchange path: the library group only when all ranks created it;
    a peer that fails BEFORE ncclCommInitRank (its set-up vote) keeps every rank from entering it
    (no rank blocks in the collective), and all use the host communicator."""
    from mpisppy_amd.comm import group_or_host
    monkeypatch.setattr(_lib, "PhgGroup", _FakeGroup)
    c = group_or_host(_Host2(rank, True), 0)
    assert isinstance(c, PhgGroupComm) and c.group.args[:2] == (2, rank)
    made = len(_FakeGroup.made)
    host, logs = _Host2(rank, False), []
    assert group_or_host(host, 0, log=logs.append) is host
    assert len(_FakeGroup.made) == made and "set-up failed on 1 rank(s)" in logs[0]
    monkeypatch.setattr(_lib, "PhgGroup", _FailingGroup)
    host, logs = _Host2(rank, True), []
    assert group_or_host(host, 0, log=logs.append) is host and "unhandled system error" in logs[0]


def test_uid_failure_still_broadcasts(monkeypatch):
    """Rank 0 failing to make the id still joins the broadcast (its peers would block in it), and
    every rank then raises."""
    class _NoId(_FakeGroup):
        @staticmethod
        def unique_id():
            raise _lib.PhgError("ncclGetUniqueId failed")
    monkeypatch.setattr(_lib, "PhgGroup", _NoId)
    host = _Host()
    with pytest.raises(RuntimeError, match="ncclGetUniqueId failed"):
        PhgGroupComm(host, 0)
    assert host.bcast == [(None, 0)]


def _gloo_worker(rank, port, q):
    """Rank 1 fails before the group's collective init (its library does not load); rank 0's
    stand-in for ncclCommInitRank is a blocking collective (a gloo barrier) that would wait forever
    for rank 1 -- so rank 0 must never reach it."""
    import os
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import _pkg
    _pkg.load()
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from mpisppy_amd import _lib, comm
    from mpisppy_amd.comm import TorchComm, group_or_host
    comm._device_count = lambda: 8

    class _BlockingGroup(_FakeGroup):
        def __init__(self, *a):
            dist.barrier()            # the collective init: only safe when every rank is here
            super().__init__(*a)

    _lib.PhgGroup = _BlockingGroup
    if rank == 1:
        def _no_lib():
            raise OSError("libphg.so: cannot open shared object file")
        _lib.load = _no_lib
    host = TorchComm()
    logs = []
    c = group_or_host(host, 0, log=logs.append)
    q.put((rank, c is host, logs[0] if logs else ""))
    dist.destroy_process_group()


def test_peer_failing_before_init_does_not_hang():
    import socket
    import torch.multiprocessing as mp
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(timeout=120)
    alive = [p.is_alive() for p in ps]
    for p in ps:
        if p.is_alive():
            p.kill()
    assert not any(alive), "a rank hung in the group set-up"
    res = sorted(q.get(timeout=5) for _ in range(2))
    assert all(r[1] for r in res), res                 # both ranks on the host communicator
    assert all("set-up failed on 1 rank(s)" in r[2] for r in res), res
