"""comm.PhgGroupComm routing (host side, no GPU): device tensors go to the library's RCCL group
(phg_group_allreduce on the attached engine's handle), everything else to the host communicator;
the 128-byte group id is made by rank 0 and broadcast by the host communicator."""
import numpy as np
import pytest

from mpisppy_amd import _lib
from mpisppy_amd.comm import PhgGroupComm, SingleComm


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
